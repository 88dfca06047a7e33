#!/bin/bash
# Build decoder variants (-D knobs) as separate libraries and run the phase
# diagnostic on each.  Usage: scripts/variants.sh "NAME:-DFOO=1 -DBAR=2" ...
set -u
mkdir -p gpurun_out/variants
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/variants/build.log 2>&1 || exit 1
C=pomegranate_amd/csrc
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  out=gpurun_out/variants/lib_$name.so
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$C -Iinclude $flags -c $C/lzo1x_decode_fast.hip -o /tmp/fast_$name.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out $C/lzo1x_kernels.o /tmp/fast_$name.o $C/lzo_host.o -Wl,-Bsymbolic -lpthread || exit 1
  echo "== $name ($flags)"
  timeout -k 10 120 python scripts/diag_decode.py --lib $out 2>&1 | grep -v amdgpu.ids || exit 1
done
