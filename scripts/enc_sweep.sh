#!/bin/bash
# Encoder knob sweep: scripts/enc_sweep.sh "NAME:FLAGS" "NAME@file.hip:FLAGS" ...
# (timing + phase stamps each; NAME@FILE compiles another copy of the encoder)
set -u
mkdir -p gpurun_out/encsweep
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/encsweep/build.log 2>&1 || exit 1
C=pomegranate_amd/csrc
for spec in "$@"; do
  head=${spec%%:*}; flags=${spec#*:}
  name=${head%%@*}; file=$C/lzo1x_encode_fast.hip
  [ "$head" != "$name" ] && file=${head#*@}
  out=gpurun_out/encsweep/lib_$name.so
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$C -Iinclude $flags -c $file -o /tmp/encs_$name.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out $C/lzo1x_kernels.o /tmp/encs_$name.o $C/lzo1x_decode_fast.o $C/lzo_host.o $C/batch_split.o $C/itb_codec.o $C/column_codec.o $C/xnet_frame.o -Wl,-Bsymbolic -lpthread || exit 1
  echo "== $name ($flags)"
  timeout -k 10 120 python scripts/diag_encode.py --lib $out ${MODEL:+--model $MODEL} 2>&1 | grep -v amdgpu.ids || exit 1
done
