#!/bin/bash
# Development GPU session: build, GPU parity tests, decoder phase diagnostic.
set -u
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/diag_decode.py "$@" > gpurun_out/diag.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/diag.log; exit $rc
