#!/bin/bash
# Decoder priority A/B: the C2 phase diagnostic, then C4 (mixed sizes, several
# rounds) with each variant's library swapped in, then the GPU parity suite.
set -u
mkdir -p gpurun_out
bash scripts/variants.sh "on:-DPOM_PRIO=1" "off:-DPOM_PRIO=0" "on2:-DPOM_PRIO=1" "off2:-DPOM_PRIO=0" > gpurun_out/variants.log 2>&1 || { tail gpurun_out/variants.log; exit 1; }
grep -E "^==|stamps=False" gpurun_out/variants.log
cp pomegranate_amd/liblzo_mi355x.so gpurun_out/lib_tree.so
for v in on off; do
  cp gpurun_out/variants/lib_$v.so pomegranate_amd/liblzo_mi355x.so
  echo "== c4 $v"; timeout -k 10 300 python bench.py --workload c4 --c4-blocks 32768 --steps 5 --warmup 1 > gpurun_out/c4_$v.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/c4_$v.log | tr '\n' ' '; echo
done
cp gpurun_out/lib_tree.so pomegranate_amd/liblzo_mi355x.so
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log; exit $rc
