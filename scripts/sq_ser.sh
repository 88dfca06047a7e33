#!/bin/bash
# SQ instruction mix per block of the table-walk decoder (lzo1x_decode_ser_kernel),
# its row-executor variant (the same kernel template, ROWS) and the op-set
# decoder, C2 (4096 x 64 KiB ITB blocks).  GPU box.  Usage: sq_ser.sh [kinds]
set -u
KINDS=${1:-"ser row fast"}
mkdir -p gpurun_out/sqser
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_ANY"
for k in $KINDS; do
  kern=$k; [ "$k" = row ] && kern=ser
  timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-include-regex "decode_${kern}_kernel" -d gpurun_out/sqser/$k -o sq --output-format csv -- python3 scripts/dec_compare.py $k c2_4096x64k > gpurun_out/sqser/$k.log 2>&1 || { echo "$k failed"; tail -3 gpurun_out/sqser/$k.log; exit 1; }
done
KINDS="$KINDS" python3 - <<'PY'
import csv, collections, glob, os
for v in os.environ["KINDS"].split():
    kern = "ser" if v == "row" else v
    d = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/sqser/{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if f"decode_{kern}_kernel" in r["Kernel_Name"]:
                d[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: int(sum(x) / len(x) / 4096) for k, x in sorted(d.items())}, "(per block)")
PY
