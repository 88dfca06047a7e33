#!/bin/bash
# A/B decoder variants: each "NAME:FLAGS" spec builds liblzo_mi355x.so with the
# decoder compiled with FLAGS, then runs scripts/diag_decode.py REPS times.
# Usage (on the GPU box): REPS=3 bash scripts/ab_decode.sh "base:" "v1:-DPOM_SLOTS=8"
set -u
REPS=${REPS:-3}
mkdir -p gpurun_out/variants
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/variants/build.log 2>&1 || exit 1
C=pomegranate_amd/csrc
for spec in "$@"; do
  head=${spec%%:*}; flags=${spec#*:}
  name=${head%%@*}; file=$C/lzo1x_decode_fast.hip
  [ "$head" != "$name" ] && file=${head#*@}
  out=gpurun_out/variants/lib_$name.so
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$C -Iinclude $flags -c $file -o /tmp/fast_$name.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out /tmp/fast_$name.o $(ls $C/*.o | grep -v lzo1x_decode_fast.o) -Wl,-Bsymbolic -lpthread || exit 1
  for r in $(seq $REPS); do
    echo "== $name rep $r ($flags)"
    timeout -k 10 120 python scripts/diag_decode.py --lib $out --nostamps 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
