# C5 read regression: the round-4 tree (5e50ee6, built in
# scripts/ab/r4tree) against this tree, alternating, same box, host_timing=1.
# ROUNDS pairs (default 5); logs under gpurun_out/c5r4${TAG}/.
set -u
O=gpurun_out/c5r4${TAG:-}
mkdir -p $O
for r in $(seq ${ROUNDS:-5}); do
  for v in r4 head; do
    if [ $v = r4 ]; then d=scripts/ab/r4tree; else d=.; fi
    (cd $d && POM_LZO_DEBUG=host_timing=1 timeout -k 10 200 python bench.py --workload c5 --steps 20) > $O/${v}_$r.log 2>&1 || { echo "$v run $r failed"; tail -5 $O/${v}_$r.log; exit 1; }
    echo "$v run $r: $(grep -o '"write_gibps": [0-9.]*, "write_serial_gibps": [0-9.]*, "read_gibps": [0-9.]*, "read_serial_gibps": [0-9.]*, "compress_pcie_gibps": [0-9.]*, "decompress_pcie_gibps": [0-9.]*' $O/${v}_$r.log)"
  done
done
