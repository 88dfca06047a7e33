"""Summarise a profile_decode.sh run into profiles/<tag>_decode_pmc.json and
copy the rocprofv3 CSV summaries into profiles/<tag>/."""
import ast, csv, json, os, shutil, sys, statistics
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = os.path.join("gpurun_out", f"prof_{tag}")
dst = os.path.join("profiles", tag)
os.makedirs(dst, exist_ok=True)
for rel in ("trace/bench_kernel_stats.csv", "trace/bench_kernel_trace.csv", "pmc_fetch/fetch_counter_collection.csv",
            "pmc_write/write_counter_collection.csv", "trace/bench_agent_info.csv"):
    p = os.path.join(src, rel)
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, os.path.basename(p)))
# bench.py's timed decode launches run one at a time on the first stream that
# launches the kernel; its pipelined_gibps leg then overlaps launches on two
# more streams, which stretches those launches' durations.  The stats CSV
# averages both; the one-at-a-time average is what bench's kernel_ms measures.
trace = [r for r in csv.DictReader(open(os.path.join(src, "trace/bench_kernel_trace.csv")))
         if "decode_fast_kernel" in r["Kernel_Name"]]
solo = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace
        if r["Stream_Id"] == trace[0]["Stream_Id"]]
stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(src, "trace/bench_kernel_stats.csv")))}
dec = next(v for k, v in stats.items() if "decode_fast_kernel" in k)
enc = next((v for k, v in stats.items() if "encode_fast_kernel" in k),
           next(v for k, v in stats.items() if "encode_kernel" in k))
def counter(path):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if "decode_fast" in r["Kernel_Name"]]
    return statistics.mean(vals), len(vals)
fetch_kb, nf = counter(os.path.join(src, "pmc_fetch/fetch_counter_collection.csv"))
write_kb, nw = counter(os.path.join(src, "pmc_write/write_counter_collection.csv"))
# workload (scripts/run_decode.py log)
info = {}
for line in open(os.path.join(src, "pmc_fetch.log")):
    if line.startswith("{"):
        info = ast.literal_eval(line)
alg = info["n_bytes"] + info["z_bytes"]
hbm = (2 * fetch_kb + write_kb) * 1024
out = {
    "tag": tag, "kernel": "lzo1x_decode_fast_kernel", "block_bytes": 65536, "nblocks": info["blocks"],
    "kernel_avg_ns": float(dec["AverageNs"]), "kernel_calls": int(dec["Calls"]),
    "solo_launches": len(solo), "solo_avg_ns": statistics.mean(solo),
    "encode_kernel_avg_ns": float(enc["AverageNs"]),
    "FETCH_SIZE_kb_per_launch": fetch_kb, "WRITE_SIZE_kb_per_launch": write_kb,
    "pmc_launches": [nf, nw],
    "hbm_bytes_per_launch": int(hbm),
    "hbm_bytes_formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024  (MI355X_MICROARCH.md: gfx950 FETCH_SIZE "
                         "reads 1/2 of wide streaming reads; this kernel's mixed dword/byte reads are "
                         "uncalibrated, so the read side is an estimate)",
    "algorithmic_bytes_per_launch": alg,
    "traffic_over_algorithmic": hbm / alg,
    "achieved_GBps_from_trace": alg / statistics.mean(solo),
}
with open(os.path.join("profiles", f"{tag}_decode_pmc.json"), "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
