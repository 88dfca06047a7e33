#!/bin/bash
# Build decoder variants as separate libraries and run the phase diagnostic on
# each, all on the same box (timings vary a few % between boxes).
# Usage: scripts/variants.sh "NAME:-DFOO=1 -DBAR=2" "NAME@path/to/decode_fast.hip:FLAGS" ...
#   NAME@FILE compiles another copy of lzo1x_decode_fast.hip (e.g. a
#   `git show HEAD:...` snapshot saved under scripts/ab/) instead of the tree's.
set -u
mkdir -p gpurun_out/variants
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/variants/build.log 2>&1 || exit 1
C=pomegranate_amd/csrc
for spec in "$@"; do
  head=${spec%%:*}; flags=${spec#*:}
  name=${head%%@*}; file=$C/lzo1x_decode_fast.hip
  [ "$head" != "$name" ] && file=${head#*@}
  out=gpurun_out/variants/lib_$name.so
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$C -Iinclude $flags -c $file -o /tmp/fast_$name.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out $C/lzo1x_kernels.o $C/lzo1x_encode_fast.o /tmp/fast_$name.o $C/lzo_host.o $C/batch_split.o $C/itb_codec.o $C/column_codec.o $C/xnet_frame.o -Wl,-Bsymbolic -lpthread || exit 1
  echo "== $name ($file $flags)"
  timeout -k 10 120 python scripts/diag_decode.py --lib $out 2>&1 | grep -v amdgpu.ids || exit 1
done
