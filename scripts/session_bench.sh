#!/bin/bash
# GPU session: build, GPU tests, smoke, and the bench workloads.
set -u
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 1; }
run() {  # run NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
    echo "== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 6
    return $rc
}
run pytest_gpu 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread &&
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()" &&
run bench_c2 300 python bench.py &&
run bench_c4 400 python bench.py --workload c4 --c4-blocks ${C4_BLOCKS:-16384} --steps 5 --warmup 1 &&
run bench_c5 300 python bench.py --workload c5
