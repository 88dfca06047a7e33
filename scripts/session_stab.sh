#!/bin/bash
# Stability: the whole GPU suite twice, then the fast-only diagnostic REPS times.
set -u
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_stab$r.log 2>&1; rc=$?
  echo "== pytest run $r rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/pytest_stab$r.log | tail -8
  [ $rc -ge 124 ] && exit $rc
done
for r in $(seq ${REPS:-3}); do
  timeout -k 10 120 python scripts/diag_decode.py --nostamps 2>&1 | grep -v amdgpu.ids || exit 1
done
