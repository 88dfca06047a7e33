"""Summarise a scripts/profile_round.sh run (gpurun_out/prof_<tag>/) into
profiles/<tag>/ (the rocprofv3 CSV summaries), profiles/<tag>_decode_pmc.json,
profiles/<tag>_encode_pmc.json (HBM bytes per launch, stamped with the kernel
source's hash so bench.py only uses them for that build) and
profiles/<tag>_sq.txt (instruction mix per launch and per block).

HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (KiB units): on gfx950 FETCH_SIZE
reports half the bytes of wide streaming reads (MI355X_MICROARCH.md, HBM);
WRITE_SIZE is exact for 16-B-per-lane stores.  The decoder's narrow reads are
uncalibrated, so its read side is an estimate."""
import ast
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (source_sha16: the same stamp bench.py checks)

tag = sys.argv[1]
src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
dst = os.path.join(ROOT, "profiles", tag)
os.makedirs(dst, exist_ok=True)
for rel in ("trace/bench_kernel_stats.csv", "trace/bench_agent_info.csv"):
    p = os.path.join(src, rel)
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, os.path.basename(p)))
shutil.copy(os.path.join(src, "bench_traced.log"), os.path.join(dst, "bench_traced.log"))

stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(src, "trace/bench_kernel_stats.csv")))}
trace = list(csv.DictReader(open(os.path.join(src, "trace/bench_kernel_trace.csv"))))


def solo_avg_ns(kname):
    """bench.py's timed launches run one at a time on the first stream that
    launches the kernel; its pipelined leg then overlaps launches on more
    streams, which stretches those launches.  The one-at-a-time average is
    what bench's kernel_ms measures."""
    rows = [r for r in trace if kname in r["Kernel_Name"]]
    solo = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows
            if r["Stream_Id"] == rows[0]["Stream_Id"]]
    return statistics.mean(solo), len(solo)
KERNEL = {"decode": ("decode_fast_kernel", "lzo1x_decode_fast_kernel"),
          "encode": ("encode_gdict1_kernel", "lzo1x_encode_gdict1_kernel")}   # (one-wave default)


def counters(op, name):
    d = {}
    for f in glob.glob(os.path.join(src, f"{op}_{name}", "**", "*counter_collection.csv"),
                       recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL[op][0] in r["Kernel_Name"]:
                d.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: (statistics.mean(v), len(v)) for k, v in d.items()}


sq_lines = [f"# SQ counters per launch and per block, 4096 x 64 KiB ITB blocks, profiles/{tag} "
            "(scripts/profile_round.sh)"]
for op in ("decode", "encode"):
    info = {}
    for line in open(os.path.join(src, f"{op}_fetch_size.log")):
        if line.startswith("{"):
            info = ast.literal_eval(line)
    fetch = counters(op, "fetch_size")["FETCH_SIZE"]
    write = counters(op, "write_size")["WRITE_SIZE"]
    st = next(v for k, v in stats.items() if KERNEL[op][0] in k)
    alg = info["n_bytes"] + info["z_bytes"]
    hbm = (2 * fetch[0] + write[0]) * 1024
    out = {
        "tag": tag, "profile": f"profiles/{tag}", "kernel": KERNEL[op][1],
        "source": bench.KERNEL_SOURCES[op], "source_sha16": bench.source_sha16(op),
        "block_bytes": 65536, "nblocks": info["blocks"],
        "bench_trace_avg_ns": float(st["AverageNs"]), "bench_trace_calls": int(st["Calls"]),
        "bench_trace_solo_avg_ns": solo_avg_ns(KERNEL[op][0])[0],
        "bench_trace_solo_calls": solo_avg_ns(KERNEL[op][0])[1],
        "FETCH_SIZE_kb_per_launch": fetch[0], "WRITE_SIZE_kb_per_launch": write[0],
        "pmc_launches": [fetch[1], write[1]],
        "hbm_bytes_per_launch": int(hbm),
        "hbm_bytes_formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024",
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": round(hbm / alg, 3),
        "achieved_GBps_from_trace": round(alg / solo_avg_ns(KERNEL[op][0])[0], 1),
    }
    with open(os.path.join(ROOT, "profiles", f"{tag}_{op}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
    sq = counters(op, "sq")
    sq_lines.append(f"## {KERNEL[op][1]} (launches: {max((n for _, n in sq.values()), default=0)})")
    for k, (v, _) in sorted(sq.items()):
        sq_lines.append(f"{k:22s} {v:16.0f}   per block {v / info['blocks']:12.0f}")
with open(os.path.join(ROOT, "profiles", f"{tag}_sq.txt"), "w") as f:
    f.write("\n".join(sq_lines) + "\n")
print("\n".join(sq_lines))
