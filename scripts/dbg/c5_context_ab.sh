# C5 inside the full bench line (as the driver runs it): with the CPU baseline
# legs run before it (the bench's order) against --no-cpu, alternating.
set -u
O=gpurun_out/c5ctx
mkdir -p $O
for r in 1 2 3; do
  for v in cpu nocpu; do
    a=""; [ $v = nocpu ] && a="--no-cpu"
    timeout -k 10 300 python bench.py $a > $O/${v}_$r.log 2>&1 || { echo "$v run $r failed"; tail -5 $O/${v}_$r.log; exit 1; }
    python - $O/${v}_$r.log $v $r <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
c5 = j["other_configs"]["c5"]
print(sys.argv[2], "run", sys.argv[3], "value", j["value"], "c5 read", c5["read_gibps"], "write", c5["write_gibps"],
      "dec_pcie", c5["decompress_pcie_gibps"], "read_serial", c5["read_serial_gibps"], "c4 dec", j["other_configs"]["c4"]["decompress_gibps"])
PY
  done
done
