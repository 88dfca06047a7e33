# C5 write with and without the append pages allocated ahead (debug key
# abuf_prealloc), alternating, with the per-chunk append times (host_timing).
set -u
mkdir -p gpurun_out/c5ab
for r in 1 2 3 4; do
  for v in 1 0; do
    POM_LZO_DEBUG=abuf_prealloc=$v,host_timing=1 timeout -k 10 200 python bench.py --workload c5 --steps 10 > gpurun_out/c5ab/p${v}_$r.log 2>&1 || exit 1
    echo "prealloc=$v run $r: $(grep -o '"write_gibps": [0-9.]*' gpurun_out/c5ab/p${v}_$r.log) on_chunk ms: $(grep on_chunk gpurun_out/c5ab/p${v}_$r.log | awk '{s+=$3} END {print s/NR*5}')"
  done
done
