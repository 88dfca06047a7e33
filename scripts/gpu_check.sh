#!/bin/bash
# One GPU-box session: parity tests, smoke, bench.  Each GPU step has its own
# time limit; a crash, abort or timeout (exit >= 124) ends the session there.
# Usage: scripts/gpu_check.sh [bench args...]
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 25 "$OUT/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "stopping: $name ended with $rc"; exit $rc
    fi
    return 0
}
python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || { echo build failed; tail "$OUT/build.log"; exit 1; }
step pytest_gpu 420 python -u -m pytest tests -v -s -m gpu -x --timeout 120 --timeout-method thread
step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
step bench 360 python bench.py "$@"
