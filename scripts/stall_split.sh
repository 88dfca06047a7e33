#!/bin/bash
# Where the waves' cycles go (GPU box): SQ_WAVE_CYCLES split into parked on
# s_waitcnt (SQ_WAIT_ANY), stalled at issue (SQ_WAIT_INST_ANY) and issuing
# (SQ_ACTIVE_INST_ANY, by type), one pass of 8 SQ counters per kernel, 4096 x
# 64 KiB ITB blocks.  Counters the box does not list are dropped.
#   bash scripts/stall_split.sh TAG [LIB]  -> gpurun_out/stall_TAG/, summary on stdout
set -u
TAG=${1:?tag}; LIB=${2:-}
OUT=gpurun_out/stall_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || { echo "counter list failed"; exit 1; }
WANT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
SQ=""
for c in $WANT; do grep -qw "$c" $OUT/avail.txt && SQ="$SQ $c"; done
echo "counters:$SQ"
lib=""; [ -n "$LIB" ] && lib="--lib $LIB"
for op in encode decode; do
  re=decode_fast; [ $op = encode ] && re='encode_(fast|gdict)'
  timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-include-regex "$re" -d $OUT/$op -o sq --output-format csv -- python3 scripts/run_decode.py --op $op --reps 5 $lib > $OUT/$op.log 2>&1 || { echo "$op failed"; tail -5 $OUT/$op.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys
out = sys.argv[1]
for op in ("encode", "decode"):
    d = collections.defaultdict(list)
    for f in glob.glob(f"{out}/{op}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(x) / len(x) for k, x in d.items()}
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    print(op, " ".join(f"{k[3:]}={v / 4096:.0f} ({100 * v / wc:.1f}%)" for k, v in sorted(m.items())),
          "(per block, % of wave cycles)")
PY
