set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4a}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "not quad" > gpurun_out/${T}_pytest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err && \
timeout -k 10 120 python -u scripts/enc_lone.py 5 > gpurun_out/${T}_enc_lone.log 2>&1
rc=$?
echo base_rc=$rc > gpurun_out/${T}_rc.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -m pytest tests/test_gpu_codec.py -q -x --timeout 60 --timeout-method thread -k "quad" > gpurun_out/${T}_quad_tests.log 2>&1
rc=$?
echo quad_rc=$rc >> gpurun_out/${T}_rc.txt
[ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -u scripts/seg_check.py 5 fast seg quad > gpurun_out/${T}_seg.log 2>&1
echo seg_rc=$? >> gpurun_out/${T}_rc.txt
