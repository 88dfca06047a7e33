#!/bin/bash
# Encoder variants ("NAME:FLAGS" or "NAME@FILE:FLAGS", FILE replacing
# lzo1x_encode_fast.hip): build each library, run diag_encode.py REPS times
# (timing + identity vs LDS).
set -u
REPS=${REPS:-1}
mkdir -p gpurun_out/variants
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/variants/build.log 2>&1 || exit 1
C=pomegranate_amd/csrc
for spec in "$@"; do
  head=${spec%%:*}; flags=${spec#*:}
  name=${head%%@*}; file=$C/lzo1x_encode_fast.hip
  [ "$head" != "$name" ] && file=${head#*@}
  out=gpurun_out/variants/libe_$name.so
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$C -Iinclude $flags -c $file -o /tmp/encv_$name.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out /tmp/encv_$name.o $(ls $C/*.o | grep -v lzo1x_encode_fast.o) -Wl,-Bsymbolic -lpthread || exit 1
  for r in $(seq $REPS); do
    echo "== $name rep $r ($flags)"
    timeout -k 10 200 python scripts/diag_encode.py --lib $out --nostamps ${DIAGARGS:-} 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
