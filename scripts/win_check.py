"""GPU check of the throughput decoder selected by POM_DECODER (default: the
windowed decoder): exactness over every synthetic model and a spread of sizes
(output compared with the input, fallback count reported), then the C2 decode
time (4096 x 64 KiB ITB blocks, HIP events on the launch stream)."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pomegranate_amd import lzo, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--blocks", type=int, default=4096)
ap.add_argument("--skip-exact", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def roundtrip(model, sizes, seed):
    arena, offs, lens = synth.batch(model, seed, sizes, threads=16, align=256)
    nb = len(sizes)
    src = lzo.DeviceBatch(t(arena), t(offs.view(np.int64)), t(lens.view(np.int32)))
    caps = np.array([lzo.worst_compress(int(n)) for n in lens], dtype=np.uint32)
    zo = np.zeros(nb, dtype=np.uint64)
    zo[1:] = np.cumsum((caps[:-1].astype(np.uint64) + 255) // 256 * 256)
    za = torch.zeros(int(zo[-1]) + int(caps[-1]) + 256, dtype=torch.uint8, device=dev)
    zb = lzo.DeviceBatch(za, t(zo.view(np.int64)), t(caps.view(np.int32)))
    zl = torch.zeros(nb, dtype=torch.int32, device=dev)
    zs = torch.zeros_like(zl)
    lzo.compress_dev(src, zb, zl, zs)
    torch.cuda.synchronize()
    assert bool((zs == 0).all())
    zsrc = lzo.DeviceBatch(za, zb.off, zl)
    out = torch.full_like(src.arena, 0xAB)
    ob = lzo.DeviceBatch(out, src.off, src.length)
    ol = torch.zeros_like(zl)
    st = torch.zeros_like(zl)
    scr = torch.zeros(lzo.decompress_scratch_bytes(nb), dtype=torch.uint8, device=dev)
    return src, zsrc, ob, out, ol, st, scr, lens


results = {}
if not a.skip_exact:
    rng = np.random.default_rng(5)
    for model in range(6):
        for rnd in range(2):
            sizes = [int(x) for x in rng.choice([1, 2, 3, 7, 64, 100, 1000, 4095, 4096, 4097, 8191,
                                                 12416, 65536, 65537, 100000, 262144, 536192], 40)]
            src, zsrc, ob, out, ol, st, scr, lens = roundtrip(model, sizes, 100 * model + rnd)
            lzo.decompress_dev(zsrc, ob, ol, st, scr)
            torch.cuda.synchronize()
            fb = int(scr[:4].view(torch.int32).item())
            bad = []
            o = out.cpu().numpy(); s = src.arena.cpu().numpy()
            offs = src.off.cpu().numpy(); stn = st.cpu().numpy(); oln = ol.cpu().numpy()
            for i, n in enumerate(lens):
                if not np.array_equal(o[offs[i]:offs[i] + n], s[offs[i]:offs[i] + n]) or \
                        int(stn[i]) != 0 or int(oln[i]) != int(n):
                    bad.append((i, int(n), int(stn[i]), int(oln[i])))
            ok = not bad
            results[f"{synth.MODEL_NAMES[model]}/{rnd}"] = {"ok": ok, "fallbacks": fb, "bad": bad[:5]}
            print(synth.MODEL_NAMES[model], rnd, ok, "fallbacks", fb, bad[:5], flush=True)

# C2 timing
src, zsrc, ob, out, ol, st, scr, lens = roundtrip(synth.ITB, [65536] * a.blocks, 0)
s = torch.cuda.current_stream()
lzo.decompress_dev(zsrc, ob, ol, st, scr)
torch.cuda.synchronize()
fb = int(scr[:4].view(torch.int32).item())
ok = torch.equal(out, src.arena) and bool((st == 0).all())
ev0 = torch.cuda.Event(enable_timing=True)
ev1 = torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(a.reps):
    ev0.record(s)
    lzo.decompress_dev(zsrc, ob, ol, st, scr)
    ev1.record(s)
    torch.cuda.synchronize()
    ts.append(ev0.elapsed_time(ev1))
n = int(lens.astype(np.int64).sum())
ms = float(np.median(ts))
print({"decoder": os.environ.get("POM_DECODER", "win"), "c2_ok": ok, "c2_fallbacks": fb,
       "c2_ms_median": round(ms, 4), "c2_ms_min": round(min(ts), 4),
       "c2_gibps": round(n / (ms / 1e3) / 2**30, 1), "exact_all_ok": all(r["ok"] for r in results.values())},
      flush=True)
