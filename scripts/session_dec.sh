#!/bin/bash
# Decoder development session: GPU codec tests (all, no -x), then the phase
# diagnostic.  Usage: scripts/session_dec.sh [pytest -k expr]
set -u
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py -q -m gpu --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_dec.log 2>&1; rc=$?
grep -E "passed|failed|Error|error|FAIL" gpurun_out/pytest_dec.log | tail -30
[ $rc -ge 124 ] && exit $rc
timeout -k 10 120 python scripts/diag_decode.py > gpurun_out/diag.log 2>&1; rc2=$?
grep -v amdgpu.ids gpurun_out/diag.log | head -20
exit $rc2
