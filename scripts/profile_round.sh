#!/bin/bash
# rocprofv3 evidence of one round (run on the GPU box):
#   1. kernel trace + stats of the default bench.py run (what the bench line measures)
#   2. PMC FETCH_SIZE and WRITE_SIZE, separate passes, for the decode and the encode kernel
#   3. SQ instruction-mix counters (one pass of 8) for each
# Output under gpurun_out/prof_<tag>/; summarise with scripts/profile_round.py <tag>.
set -u
TAG=${1:?tag}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# (the library is built in-tree before the call: it travels with the snapshot)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-others > $OUT/bench_traced.log 2>&1 || { echo trace failed; tail $OUT/bench_traced.log; exit 1; }
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_ANY"
for op in decode encode; do
  re=decode_fast; [ $op = encode ] && re='encode_(fast|gdict)'
  for ctr in FETCH_SIZE WRITE_SIZE "$SQ"; do
    name=$(echo $ctr | cut -d' ' -f1 | tr A-Z a-z)
    [ "$ctr" = "$SQ" ] && name=sq
    timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "$re" -d $OUT/${op}_$name -o $name --output-format csv -- python3 scripts/run_decode.py --op $op --reps 5 > $OUT/${op}_$name.log 2>&1 || { echo "$op $name failed"; tail -5 $OUT/${op}_$name.log; exit 1; }
  done
done
echo profile done
