#!/bin/bash
# SQ instruction counts of the throughput encoder (one launch over 4096 x 64 KiB
# ITB blocks, from scripts/run_decode.py's compression), printed per block:
# the whole kernel, then with the emit wave only draining tokens
# (POM_ENC_NOEMIT, timing experiment) -- the parse wave's share.
set -u
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
C=pomegranate_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$C -Iinclude -DPOM_ENC_NOEMIT=1 -c $C/lzo1x_encode_fast.hip -o /tmp/noemit.o || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o /tmp/lib_noemit.so $C/lzo1x_kernels.o /tmp/noemit.o $C/lzo1x_decode_fast.o $C/lzo_host.o $C/batch_split.o $C/itb_codec.o $C/column_codec.o $C/xnet_frame.o -Wl,-Bsymbolic -lpthread || exit 1
export TMPDIR=/tmp
for v in full noemit; do
  lib=""; [ $v = noemit ] && lib="--lib /tmp/lib_noemit.so"
  # (the noemit build's output is not a valid stream: run_decode's check fails, expected)
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex encode_fast -d gpurun_out/sqe_$v -o sq --output-format csv -- python3 scripts/run_decode.py --reps 1 $lib > gpurun_out/sqe_$v.log 2>&1
done
python - <<'PY'
import csv, collections, glob
for v in ("full", "noemit"):
    d = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/sqe_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "encode_fast" in r["Kernel_Name"]:
                d[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: int(sum(x) / len(x) / 4096) for k, x in sorted(d.items())}, "(per block)")
PY
