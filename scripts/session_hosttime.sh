#!/bin/bash
# GPU tests, then C5 with the host batch phase timers (POM_HOST_TIMING=1).
set -u
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
POM_HOST_TIMING=1 timeout -k 10 300 python bench.py --workload c5 > gpurun_out/c5t.log 2>&1; rc=$?
grep "pom host" gpurun_out/c5t.log | tail -8; grep -v amdgpu.ids gpurun_out/c5t.log | tail -1 | cut -c1-150; exit $rc
