#!/bin/bash
# SQ instruction counts: full decoder vs the parser alone (executor skips).
set -u
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
C=pomegranate_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$C -Iinclude -DPOM_EXEC_SKIP=1 -c $C/lzo1x_decode_fast.hip -o /tmp/ponly.o || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o gpurun_out/lib_ponly.so $C/lzo1x_kernels.o $C/lzo1x_encode_fast.o /tmp/ponly.o $C/lzo_host.o $C/batch_split.o $C/itb_codec.o $C/column_codec.o $C/xnet_frame.o -Wl,-Bsymbolic -lpthread || exit 1
export TMPDIR=/tmp
for v in full ponly; do
  lib=""; [ $v = ponly ] && lib="--lib gpurun_out/lib_ponly.so"
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES --kernel-include-regex decode_fast -d gpurun_out/sqs_$v -o sq --output-format csv -- python3 scripts/run_decode.py --reps 3 $lib > gpurun_out/sqs_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/sqs_$v.log; }
done
python - <<'PY'
import csv, collections, glob
for v in ("full", "ponly"):
    d = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/sqs_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "decode_fast" in r["Kernel_Name"]:
                d[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: int(sum(x)/len(x)/4096) for k, x in sorted(d.items())}, "(per block)")
PY
