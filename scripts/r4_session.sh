# One GPU-box session of round 4: the GPU tests (all, not stopping at the
# first failure), smoke, the default bench line, then the rocprofv3 evidence
# (scripts/profile_round.sh TAG).  A fault, abort or timeout ends it.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4x}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=15 --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc > gpurun_out/${T}_rc.txt; ok $rc || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
rc=$?; echo smoke_rc=$rc >> gpurun_out/${T}_rc.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; echo bench_rc=$rc >> gpurun_out/${T}_rc.txt; [ $rc -eq 0 ] || exit $rc
[ "${2:-}" = "noprof" ] && exit 0
bash scripts/profile_round.sh $T > gpurun_out/${T}_prof.log 2>&1
echo prof_rc=$? >> gpurun_out/${T}_rc.txt
