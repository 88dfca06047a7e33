#!/bin/bash
# SQ instruction counts of the C3 encoder, one pass of 8 SQ counters per
# library build (GPU box): scripts/sq_changes.sh TAG NAME...  with
# scripts/ab/lib_NAME.so built beforehand (scripts/ab_build.sh).  Per block,
# 4096 x 64 KiB ITB blocks; summary on stdout and in gpurun_out/sqchg_TAG/.
# PMC="..." replaces the counter set (one pass; all its counters are listed);
# OP=decode profiles the fast decoder instead of the C3 encoder.
set -u
TAG=${1:?tag}; shift
OUT=gpurun_out/sqchg_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
SQ=${PMC:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_ANY"}
OP=${OP:-encode}; RE='encode_(fast|gdict)'; [ $OP = decode ] && RE=decode_fast
for v in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-include-regex "$RE" -d $OUT/$v -o sq --output-format csv -- python3 scripts/run_decode.py --op $OP --reps 5 --lib scripts/ab/lib_$v.so ${RUN_ARGS:-} > $OUT/$v.log 2>&1 || { echo "$v failed"; tail -5 $OUT/$v.log; exit 1; }
done
python3 - "$OUT" "$@" <<PY
import csv, collections, glob, sys
out, names = sys.argv[1], sys.argv[2:]
keys = "${PMC:-SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES}".split()
print("| build | " + " | ".join(k[3:] for k in keys) + " |")
print("|---" * (len(keys) + 1) + "|")
for v in names:
    d = collections.defaultdict(list)
    for f in glob.glob(f"{out}/{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(x) / len(x) / 4096 for k, x in d.items()}
    print(f"| {v} | " + " | ".join(f"{m.get(k, 0):.0f}" for k in keys) + " |")
PY
