# C5 write, alternating: the compress+append batch's appends on a worker thread
# with their page-cache pages allocated ahead (debug keys append_worker=1,
# abuf_prealloc=1) against both off (appends on the pipeline thread).
set -u
mkdir -p gpurun_out/c5w
for r in 1 2 3 4 5 6 7 8; do
  for v in 1 0; do
    POM_LZO_DEBUG=append_worker=$v,abuf_prealloc=$v timeout -k 10 200 python bench.py --workload c5 --steps 10 > gpurun_out/c5w/b${v}_$r.log 2>&1 || exit 1
    echo "both=$v run $r: $(grep -o '"write_gibps": [0-9.]*, "write_serial_gibps": [0-9.]*, "read_gibps": [0-9.]*' gpurun_out/c5w/b${v}_$r.log)"
  done
done
