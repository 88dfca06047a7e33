#!/bin/bash
# Build encoder variants (-D knobs on lzo1x_encode_fast.hip) as separate
# libraries and time each with the parse-wave diagnostic: scripts/enc_ab.sh - "NAME:FLAGS" ...
set -u
mkdir -p gpurun_out/encvar
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/encvar/build.log 2>&1 || exit 1
C=pomegranate_amd/csrc
batch=${1:-}; shift
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  out=gpurun_out/encvar/lib_$name.so
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$C -Iinclude $flags -c $C/lzo1x_encode_fast.hip -o /tmp/encf_$name.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out $C/lzo1x_kernels.o /tmp/encf_$name.o $C/lzo1x_decode_fast.o $C/lzo_host.o $C/batch_split.o $C/itb_codec.o $C/column_codec.o $C/xnet_frame.o -Wl,-Bsymbolic -lpthread || exit 1
  echo "== $name ($flags)"
  timeout -k 10 200 python scripts/diag_encode.py --lib $out 2>&1 | grep -E "stamps=False|kernel" | head -3 || exit 1
done
