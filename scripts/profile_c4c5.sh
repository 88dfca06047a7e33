set -u
TAG=${1:-r02e}
OUT=gpurun_out/prof_${TAG}_c4c5
mkdir -p $OUT
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c4 -o c4 --output-format csv -- python3 bench.py --workload c4 --steps 3 --warmup 1 > $OUT/c4_traced.log 2>&1 || { echo c4 trace failed; tail $OUT/c4_traced.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/c5 -o c5 --output-format csv -- python3 bench.py --workload c5 --steps 3 --warmup 1 > $OUT/c5_traced.log 2>&1 || { echo c5 trace failed; tail $OUT/c5_traced.log; exit 1; }
echo done
