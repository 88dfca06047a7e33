#!/bin/bash
# A/B decoder variants (phase diagnostic, scripts/variants.sh), then the GPU
# parity suite on the tree's default build.
# Usage: scripts/session_ab_test.sh "NAME:FLAGS" ...
set -u
mkdir -p gpurun_out
bash scripts/variants.sh "$@" > gpurun_out/variants.log 2>&1; rc=$?
grep -E "^==|stamps=False" gpurun_out/variants.log
[ $rc -ne 0 ] && { tail -20 gpurun_out/variants.log; exit $rc; }
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; exit $rc
