# one GPU session: the whole GPU suite, the table-walk decoder's stamps and A/B, SQ counters
mkdir -p gpurun_out
T=${1:-c1}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
echo "pytest rc=$?" >> gpurun_out/${T}_pytest.log
tail -4 gpurun_out/${T}_pytest.log
bash scripts/ser_run.sh ${T}s
bash scripts/sq_ser.sh
