# C5 write/read with host-batch chunks of CHUNK MiB (debug key chunk_mb) against
# the default, alternating: bash scripts/dbg/c5_chunk_ab.sh CHUNK
set -u
mkdir -p gpurun_out/c5c
for r in 1 2 3 4 5 6; do
  for v in $1 0; do
    k=""; [ $v != 0 ] && k="POM_LZO_DEBUG=chunk_mb=$v"
    env $k timeout -k 10 200 python bench.py --workload c5 --steps 10 > gpurun_out/c5c/c${v}_$r.log 2>&1 || exit 1
    echo "chunk_mb=$v run $r: $(grep -o '"write_gibps": [0-9.]*, "write_serial_gibps": [0-9.]*, "read_gibps": [0-9.]*' gpurun_out/c5c/c${v}_$r.log)"
  done
done
