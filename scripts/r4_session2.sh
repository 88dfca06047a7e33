# Round 4, second session: GPU tests, smoke, the rejected decoders once more
# (A/B on C2 and lone blocks, scripts/experiments built in-tree), a C5 sweep of
# the host-batch chunk budget.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r04b}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=15 --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc > gpurun_out/${T}_rc.txt; ok $rc || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
rc=$?; echo smoke_rc=$rc >> gpurun_out/${T}_rc.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/seg_check.py 5 fast seg > gpurun_out/${T}_seg.log 2>&1
rc=$?; echo seg_rc=$rc >> gpurun_out/${T}_rc.txt; ok $rc || exit $rc
for mb in 64 128 256; do
  POM_LZO_DEBUG=chunk_mb=$mb timeout -k 10 200 python -u bench.py --workload c5 --steps 15 > gpurun_out/${T}_c5_$mb.json 2>> gpurun_out/${T}_c5.err
  rc=$?; echo c5_${mb}_rc=$rc >> gpurun_out/${T}_rc.txt; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python -u bench.py --workload single --steps 10 > gpurun_out/${T}_single.json 2> gpurun_out/${T}_single.err
echo single_rc=$? >> gpurun_out/${T}_rc.txt
