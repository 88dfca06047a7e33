# table-walk decoder: its GPU tests, stamps, and the A/B against the op-set decoder
mkdir -p gpurun_out
T=${1:-ser}
timeout -k 10 200 python -u -m pytest tests/test_gpu_codec.py -x -q -k "window_decoder and ser" --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/${T}_tests.log
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 120 python -u scripts/diag_ser.py > gpurun_out/${T}_diag.log 2>&1
echo "diag rc=$?" >> gpurun_out/${T}_diag.log
cat gpurun_out/${T}_diag.log
timeout -k 10 240 python -u scripts/dec_compare.py ${KINDS:-fast,win,ser} ${ONLY:-c2_4096x64k,lone_64k,lone_536k,c5_like_1024,c4_8192mixed} > gpurun_out/${T}_cmp.log 2>&1
echo rc=$? >> gpurun_out/${T}_cmp.log
cat gpurun_out/${T}_cmp.log | grep -v amdgpu.ids
