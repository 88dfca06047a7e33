#!/bin/bash
# Row executor on the GPU box: decoder-alone tests, A/B against the op-set and
# table-walk decoders, per-phase stamps.  Usage: bash scripts/row_check.sh TAG
set -e
T=${1:-row}
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_codec.py -x -q -k "window_decoder and row" --timeout 120 --timeout-method thread > gpurun_out/$T.log 2>&1
timeout -k 10 150 python -u scripts/dec_compare.py fast,ser,row lone_64k,c2_4096x64k >> gpurun_out/$T.log 2>&1
timeout -k 10 120 python -u scripts/diag_ser.py --row >> gpurun_out/$T.log 2>&1
bash scripts/sq_ser.sh "ser row" >> gpurun_out/$T.log 2>&1
