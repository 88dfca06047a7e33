#!/bin/bash
# One GPU-box session: parity tests, smoke, bench.  Each GPU step has its own
# time limit; a crash, abort or timeout (exit >= 124) ends the session there.
# Usage: scripts/gpu_check.sh [bench args...]
set -u
mkdir -p gpurun_out
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "stopping: $name ended with $rc"; exit $rc
    fi
    return 0
}
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; tail gpurun_out/build.log; exit 1; }
step pytest_gpu 360 python -m pytest tests -q -m gpu -x
step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
step bench 360 python bench.py "$@"
