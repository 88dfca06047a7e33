#!/bin/bash
# SQ instruction mix of the decoder split between its waves: the whole kernel,
# then a build whose executor skips every piece's ops (POM_EXEC_SKIP: the parser
# alone, output not valid).  Per block, 4096 x 64 KiB ITB blocks.  GPU box.
set -u
C=pomegranate_amd/csrc
mkdir -p gpurun_out/sqsplit
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/sqsplit/build.log 2>&1 || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$C -Iinclude -DPOM_EXEC_SKIP -c $C/lzo1x_decode_fast.hip -o /tmp/skip.o || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o /tmp/lib_skip.so $C/lzo1x_kernels.o $C/lzo1x_encode_fast.o /tmp/skip.o $C/lzo_host.o $C/batch_split.o $C/itb_codec.o $C/column_codec.o $C/xnet_frame.o -Wl,-Bsymbolic -lpthread || exit 1
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_SMEM"
for v in full skip; do
  lib=""; [ $v = skip ] && lib="--lib /tmp/lib_skip.so"
  timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-include-regex decode_fast -d gpurun_out/sqsplit/$v -o sq --output-format csv -- python3 scripts/run_decode.py --reps 3 --noverify $lib > gpurun_out/sqsplit/$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/sqsplit/$v.log; exit 1; }
done
python - <<'PY'
import csv, collections, glob
for v in ("full", "skip"):
    d = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/sqsplit/{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "decode_fast" in r["Kernel_Name"]:
                d[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: int(sum(x) / len(x) / 4096) for k, x in sorted(d.items())}, "(per block)")
PY
