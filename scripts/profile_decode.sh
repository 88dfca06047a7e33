#!/bin/bash
# rocprofv3 evidence for the decode kernel (run on the GPU box):
#   1. kernel trace + stats of bench.py (what the bench line measures)
#   2. PMC FETCH_SIZE and WRITE_SIZE in separate passes of the decode driver
# Output under gpurun_out/prof_<tag>/; summarise with scripts/summarize_prof.py.
set -u
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $OUT/bench_traced.log 2>&1 || { echo trace failed; tail $OUT/bench_traced.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex decode_fast -d $OUT/pmc_fetch -o fetch --output-format csv -- python3 scripts/run_decode.py --reps 5 > $OUT/pmc_fetch.log 2>&1 || { echo pmc fetch failed; tail $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex decode_fast -d $OUT/pmc_write -o write --output-format csv -- python3 scripts/run_decode.py --reps 5 > $OUT/pmc_write.log 2>&1 || { echo pmc write failed; tail $OUT/pmc_write.log; exit 1; }
echo profile done; find $OUT -name "*.csv" | head -20
