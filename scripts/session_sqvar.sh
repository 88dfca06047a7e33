#!/bin/bash
# Build decoder variants ("NAME:FLAGS"), run the fast-only diagnostic REPS
# times and the SQ instruction-mix profile on each.
set -u
REPS=${REPS:-2}
mkdir -p gpurun_out/variants
C=pomegranate_amd/csrc
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  out=gpurun_out/variants/lib_$name.so
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$C -Iinclude $flags -c $C/lzo1x_decode_fast.hip -o /tmp/fast_$name.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out $C/lzo1x_kernels.o $C/lzo1x_encode_fast.o /tmp/fast_$name.o $C/lzo_host.o $C/batch_split.o $C/itb_codec.o $C/column_codec.o $C/xnet_frame.o -Wl,-Bsymbolic -lpthread || exit 1
  for r in $(seq $REPS); do
    echo "== $name rep $r ($flags)"
    timeout -k 10 120 python scripts/diag_decode.py --lib $out --nostamps 2>&1 | grep -v amdgpu.ids || exit 1
  done
  bash scripts/profile_sq.sh $name $out | grep -E "SQ_INSTS_VALU|SQ_INSTS_SALU|SQ_INSTS_LDS |SQ_WAVE_CYCLES|SQ_BUSY_CU|SQ_WAIT_ANY|SQ_INSTS_BRANCH|SQ_ACTIVE_INST_ANY" || exit 1
done
