#!/usr/bin/env python3
"""LZO1X block codec benchmark on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 4096 x 64 KiB synthetic ITB blocks per
GPU, LZO1X decompress-only, device-resident: inputs (the compressed blocks)
and outputs live in HBM before the timed region starts.  A "step" is one
decompression pass over the whole batch.  value = uncompressed GiB/s over
all GPUs (sum of n over every rank / max-over-ranks time).

Also reported (not the headline): LZO1X-1 compress GiB/s and compress +
decompress round-trip GiB/s on the same blocks, the HBM roofline of the decode
kernel, and the reference's own lib/minilzo.c (oracle/_ref, compiled from the
reference sources) timed on this box's host cores on a bounded sample.

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): global
block i goes to rank i mod N (weak scaling: 4096 blocks per GPU); the only
collective is the RCCL completion barrier (error sum, elapsed max).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
GIB = float(1 << 30)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--blocks", type=int, default=4096, help="blocks per GPU")
    p.add_argument("--block-bytes", type=int, default=65536)
    p.add_argument("--model", default="itb")
    p.add_argument("--compress-steps", type=int, default=3)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu", action="store_true")
    return p.parse_args()


def cpu_baseline(arena, offs, lens, comps, seconds):
    """Reference lib/minilzo.c (oracle/_ref) or, if absent, the oracle port,
    on the host cores: decompress (and compress) of a bounded sample."""
    from concurrent.futures import ThreadPoolExecutor

    ref_path = os.path.join(ROOT, "oracle", "_ref", "libminilzo_ref.so")
    port_path = os.path.join(ROOT, "oracle", "liboracle.so")
    ulong = ctypes.c_ulong
    if os.path.exists(ref_path):
        lib = ctypes.CDLL(ref_path)
        kind = "reference"
        dec = lib.lzo1x_decompress
        comp = lib.lzo1x_1_compress
        for f in (dec, comp):
            f.restype = ctypes.c_int
            f.argtypes = [ctypes.c_void_p, ulong, ctypes.c_void_p, ctypes.POINTER(ulong),
                          ctypes.c_void_p]
        init = getattr(lib, "__lzo_init_v2")
        init(0x2040, 2, 4, 8, 4, 8, 8, 8, 8, 48)
    else:
        lib = ctypes.CDLL(port_path)
        kind = "port"
        dec = None
        comp = None
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 16, os.cpu_count() or 1))
    nsample = min(len(lens), 512)
    srcs = [ctypes.create_string_buffer(comps[b], len(comps[b]) + 64) for b in range(nsample)]
    plain = [arena[int(offs[b]): int(offs[b]) + int(lens[b])].tobytes() for b in range(nsample)]

    def dec_share(t, deadline, nbytes):
        out = ctypes.create_string_buffer(int(max(lens)) + 64)
        done = 0
        b = t
        while time.perf_counter() < deadline:
            ol = ulong(0)
            if kind == "reference":
                rc = dec(srcs[b], len(comps[b]), out, ctypes.byref(ol), None)
            else:
                sz = ctypes.c_size_t(len(out))
                rc = lib.oracle_lzo1x_decompress_safe(srcs[b], ctypes.c_size_t(len(comps[b])),
                                                      out, ctypes.byref(sz))
            assert rc == 0
            done += int(lens[b])
            b = (b + threads) % nsample
        nbytes[t] = done

    def comp_share(t, deadline, nbytes):
        out = ctypes.create_string_buffer(int(max(lens)) * 2 + 128)
        wrk = ctypes.create_string_buffer(131072)
        done = 0
        b = t
        while time.perf_counter() < deadline:
            ol = ulong(0)
            src = plain[b]
            if kind == "reference":
                ctypes.memset(wrk, 0, 131072)
                comp(src, len(src), out, ctypes.byref(ol), wrk)
            else:
                sz = ctypes.c_size_t(0)
                lib.oracle_lzo1x_1_compress(src, ctypes.c_size_t(len(src)), out,
                                            ctypes.byref(sz))
            done += len(src)
            b = (b + threads) % nsample
        nbytes[t] = done

    res = {}
    for name, fn, share in (("decompress", dec_share, 0.6), ("compress", comp_share, 0.4)):
        nbytes = [0] * threads
        t0 = time.perf_counter()
        deadline = t0 + seconds * share
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda t: fn(t, deadline, nbytes), range(threads)))
        dt = time.perf_counter() - t0
        res[name] = sum(nbytes) / dt / GIB
    return {"value": round(res["decompress"], 4), "unit": "GiB/s", "cores": threads,
            "kind": kind, "compress_value": round(res["compress"], 4),
            "sample": f"{nsample} of the same {int(lens[0])}-byte ITB blocks, round-robin over "
                      f"{threads} threads for {seconds:.0f} s (decompress {0.6 * seconds:.0f} s,"
                      f" compress {0.4 * seconds:.0f} s), "
                      + ("lib/minilzo.c built from the reference sources (oracle/_ref)"
                         if kind == "reference" else "oracle/lzo1x_oracle.c port")}


def load_traffic(block_bytes, nblocks):
    """HBM bytes per decode launch from the committed rocprofv3 PMC summary,
    when one exists for this workload (profiles/*decode_pmc.json)."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*decode_pmc.json"))):
        try:
            with open(path) as f:
                j = json.load(f)
        except Exception:
            continue
        if j.get("block_bytes") == block_bytes and j.get("nblocks") == nblocks:
            best = j
    return best


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from pomegranate_amd import lzo, shard, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} but --gpus={args.gpus}", file=sys.stderr)
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (the LZO1X path has no CPU fallback)")
    # One process per GPU.  POM_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs.
    backend = os.environ.get("POM_DIST_BACKEND", "nccl")
    dev = torch.device(f"cuda:{local % torch.cuda.device_count()}")
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    lzo.load()

    model = {v: k for k, v in synth.MODEL_NAMES.items()}[args.model]
    nglobal = args.blocks * world
    mine = shard.round_robin(nglobal, rank, world)       # global ids i = rank mod G
    sizes = [args.block_bytes] * len(mine)
    arena, offs, lens = synth.batch(model, 0, sizes, seeds=mine, threads=16)
    nb = len(mine)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    src = lzo.DeviceBatch(t(arena), t(offs.view(np.int64)), t(lens.view(np.int32)))
    caps = np.array([lzo.worst_compress(int(n)) for n in lens], dtype=np.uint32)
    zoffs = np.zeros(nb, dtype=np.uint64)
    zoffs[1:] = np.cumsum((caps[:-1].astype(np.uint64) + 255) // 256 * 256)
    zarena = torch.zeros(int(zoffs[-1]) + int(caps[-1]) + 256, dtype=torch.uint8, device=dev)
    zdst = lzo.DeviceBatch(zarena, t(zoffs.view(np.int64)), t(caps.view(np.int32)))
    zlen = torch.zeros(nb, dtype=torch.int32, device=dev)
    zst = torch.zeros(nb, dtype=torch.int32, device=dev)
    out = torch.zeros_like(src.arena)
    odst = lzo.DeviceBatch(out, src.off, src.length)
    olen = torch.zeros(nb, dtype=torch.int32, device=dev)
    ost = torch.zeros(nb, dtype=torch.int32, device=dev)
    nscr = lzo.decompress_scratch_bytes(nb)
    scratch = torch.empty(max(nscr, 1), dtype=torch.uint8, device=dev) if nscr else None
    stream = torch.cuda.current_stream()

    # Compress on the GPU (also timed, secondary), check every block decodes back.
    lzo.compress_dev(src, zdst, zlen, zst)
    torch.cuda.synchronize()
    zsrc = lzo.DeviceBatch(zarena, zdst.off, zlen)
    lzo.decompress_dev(zsrc, odst, olen, ost, scratch)
    torch.cuda.synchronize()
    fallback_blocks = int(scratch[:4].view(torch.int32).item()) if scratch is not None else nb
    errors = int((zst != 0).sum().item()) + int((ost != 0).sum().item())
    errors += int((olen != src.length).sum().item()) + (0 if torch.equal(out, src.arena) else 1)
    n_bytes = float(lens.astype(np.float64).sum())
    z_bytes = float(zlen.double().sum().item())

    def timed(fn, steps, warmup):
        for _ in range(warmup):
            fn()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(steps):
            fn()
        ev1.record(stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        wall = time.perf_counter() - t0
        return wall, ev0.elapsed_time(ev1) / 1e3 / max(steps, 1)

    dec_wall, dec_kernel = timed(lambda: lzo.decompress_dev(zsrc, odst, olen, ost, scratch),
                                 args.steps, args.warmup)
    comp_wall, comp_kernel = timed(lambda: lzo.compress_dev(src, zdst, zlen, zst),
                                   args.compress_steps, 1)
    errors += int((ost != 0).sum().item()) + int((zst != 0).sum().item())

    if world > 1:
        errors, dec_wall = shard.completion_barrier(dist, dev, errors, dec_wall)
        _, comp_wall = shard.completion_barrier(dist, dev, 0, comp_wall)
        tot = torch.tensor([n_bytes, z_bytes], dtype=torch.float64,
                           device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(tot)
        n_all, z_all = float(tot[0].item()), float(tot[1].item())
    else:
        n_all, z_all = n_bytes, z_bytes

    ms_per_step = dec_wall / args.steps * 1e3
    value = n_all * args.steps / dec_wall / GIB
    comp_gibps = n_all * args.compress_steps / comp_wall / GIB
    rt_gibps = n_all / (dec_wall / args.steps + comp_wall / args.compress_steps) / GIB
    achieved = (z_bytes + n_bytes) / dec_kernel / 1e9      # per GPU, decode kernel
    traffic_rec = load_traffic(args.block_bytes, args.blocks)
    traffic = traffic_rec.get("hbm_bytes_per_launch") if traffic_rec else None

    result = {
        "metric": "LZO1X compress+decompress GiB/s (device-resident), 4-256 KiB ITB block batches",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic ITB payload images (SURVEY.md Appendix B generator, libpom_synth)",
        "config": {"workload": f"configs[1]: {args.blocks} x {args.block_bytes // 1024} KiB "
                               f"{args.model} blocks per GPU, LZO1X decompress-only, "
                               "device-resident",
                   "blocks_per_gpu": args.blocks, "block_bytes": args.block_bytes,
                   "compression_ratio": round(z_all / n_all, 4),
                   "parallelism": f"round-robin blocks over {world} GPU(s)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": traffic,
                     "kernel_ms": round(dec_kernel * 1e3, 4),
                     "algorithmic_bytes_per_launch": int(z_bytes + n_bytes)},
        "compress_gibps": round(comp_gibps, 3),
        "roundtrip_gibps": round(rt_gibps, 3),
        "compress_kernel_ms": round(comp_kernel * 1e3, 3),
        "errors": errors,
        "fallback_blocks": fallback_blocks,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        lens_np = np.asarray(lens)
        zl = zlen.cpu().numpy()
        zh = zarena.cpu().numpy()
        zo = zoffs
        comps = [zh[int(zo[b]): int(zo[b]) + int(zl[b])].tobytes() for b in range(min(nb, 512))]
        result["cpu_baseline"] = cpu_baseline(arena, offs, lens_np, comps, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if errors:
        raise SystemExit(f"bench: {errors} blocks failed the round trip")


if __name__ == "__main__":
    main()
