# one GPU session: the new single-call test, the table-walk decoder (tests, stamps, A/B), the single-call bench
mkdir -p gpurun_out
T=${1:-r}
timeout -k 10 200 python -u -m pytest tests/test_gpu_codec.py -x -q -k "single_call" --timeout 150 --timeout-method thread > gpurun_out/${T}_single_tests.log 2>&1
echo "single tests rc=$?" >> gpurun_out/${T}_single_tests.log
tail -3 gpurun_out/${T}_single_tests.log
bash scripts/ser_run.sh ${T}s
timeout -k 10 300 python -u bench.py --workload single > gpurun_out/${T}_single.json 2> gpurun_out/${T}_single.err
echo "single bench rc=$?"
cat gpurun_out/${T}_single.json
