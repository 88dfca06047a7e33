#!/bin/bash
# SQ counters of the windowed decoder alone, one block per CU (256 x 64 KiB)
set -u
OUT=gpurun_out/prof_win_${1:-a}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY --kernel-include-regex decode_win -d $OUT/sq -o sq --output-format csv -- python3 scripts/run_win.py > $OUT/sq.log 2>&1 || { echo sq failed; tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex decode_win -d $OUT/sq2 -o sq2 --output-format csv -- python3 scripts/run_win.py > $OUT/sq2.log 2>&1 || { echo sq2 failed; tail -5 $OUT/sq2.log; exit 1; }
echo prof_win done
