#!/bin/bash
# Encoder A/B: GPU tests, then scripts/enc_sweep.sh over the given specs
# (default: the committed encoder in scripts/ab/enc_head.hip against the tree's).
set -u
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
[ $# -eq 0 ] && set -- "head@scripts/ab/enc_head.hip:" "tree:"
bash scripts/enc_sweep.sh "$@" 2>&1 | grep -v "^stamps=True"
