#!/bin/bash
# Encoder variants ("NAME:FLAGS"): build each library, run diag_encode.py (timing + identity vs LDS).
set -u
mkdir -p gpurun_out/variants
C=pomegranate_amd/csrc
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  out=gpurun_out/variants/libe_$name.so
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$C -Iinclude $flags -c $C/lzo1x_encode_fast.hip -o /tmp/encv_$name.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out $C/lzo1x_kernels.o /tmp/encv_$name.o $C/lzo1x_decode_fast.o $C/lzo_host.o $C/batch_split.o $C/itb_codec.o $C/column_codec.o $C/xnet_frame.o -Wl,-Bsymbolic -lpthread || exit 1
  echo "== $name ($flags)"
  timeout -k 10 200 python scripts/diag_encode.py --lib $out --nostamps ${DIAGARGS:-} 2>&1 | grep -v amdgpu.ids || exit 1
done
