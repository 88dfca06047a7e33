# One GPU-box session: the GPU tests (all of them, not stopping at the first
# failure), smoke, bench, lone-block encoder timing, then the quarter-wave
# decoder's checks.  A step that ends in a fault, abort or timeout ends it.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4a}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # (pytest: passed / some tests failed)
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=15 --timeout 120 --timeout-method thread -k "not quad" > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc > gpurun_out/${T}_rc.txt; ok $rc || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
rc=$?; echo smoke_rc=$rc >> gpurun_out/${T}_rc.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; echo bench_rc=$rc >> gpurun_out/${T}_rc.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/enc_lone.py 5 > gpurun_out/${T}_enc_lone.log 2>&1
rc=$?; echo enc_lone_rc=$rc >> gpurun_out/${T}_rc.txt; ok $rc || exit $rc
timeout -k 10 200 python -u -m pytest tests/test_gpu_codec.py -q --timeout 60 --timeout-method thread -k "quad" > gpurun_out/${T}_quad_tests.log 2>&1
rc=$?; echo quad_rc=$rc >> gpurun_out/${T}_rc.txt; ok $rc || exit $rc
timeout -k 10 200 python -u scripts/quad_debug.py quad > gpurun_out/${T}_quad_debug.log 2>&1
rc=$?; echo qdbg_rc=$rc >> gpurun_out/${T}_rc.txt; ok $rc || exit $rc
timeout -k 10 200 python -u scripts/seg_check.py 5 fast quad > gpurun_out/${T}_seg.log 2>&1
echo seg_rc=$? >> gpurun_out/${T}_rc.txt
