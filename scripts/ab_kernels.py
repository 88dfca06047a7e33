"""A/B of the two C3 kernels between builds of the library (e.g. compiler
flag variants): compress (with the dictionary scratch, as bench.py) and
decompress of 4096 x 64 KiB ITB blocks, median HIP-event time of --reps
launches each, outputs checked.  Usage: python scripts/ab_kernels.py [--lib PATH]"""
import argparse, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from pomegranate_amd import lzo, synth

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
if a.lib:
    lzo.LIB_PATH = a.lib
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
lzo.load()
nb = 4096
arena, offs, lens = synth.batch(synth.ITB, 0, [65536] * nb, align=256, threads=16)
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
src = lzo.DeviceBatch(t(arena), t(offs.view(np.int64)), t(lens.view(np.int32)))
caps = np.array([lzo.worst_compress(int(n)) for n in lens], dtype=np.uint64)
zo = np.zeros(nb, dtype=np.uint64); zo[1:] = np.cumsum((caps[:-1] + 255) // 256 * 256)
za = torch.zeros(int(zo[-1] + caps[-1]) + 256, dtype=torch.uint8, device=dev)
zb = lzo.DeviceBatch(za, t(zo.view(np.int64)), t(caps.astype(np.uint32).view(np.int32)))
zl = torch.zeros(nb, dtype=torch.int32, device=dev); zs = torch.zeros_like(zl)
escr = torch.empty(lzo.compress_scratch_bytes(nb), dtype=torch.uint8, device=dev)


def timed(fn):
    ts = []
    for _ in range(a.reps):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts)), min(ts)


c = timed(lambda: lzo.compress_dev(src, zb, zl, zs, scratch=escr))
zsrc = lzo.DeviceBatch(za, zb.off, zl)
out = torch.zeros_like(src.arena); ob = lzo.DeviceBatch(out, src.off, src.length)
ol = torch.zeros_like(zl); st = torch.zeros_like(zl)
dscr = torch.empty(lzo.decompress_scratch_bytes(nb), dtype=torch.uint8, device=dev)
d = timed(lambda: lzo.decompress_dev(zsrc, ob, ol, st, dscr))
ok = torch.equal(out, src.arena) and bool((st == 0).all()) and bool((zs == 0).all())
fb = int(dscr[:4].view(torch.int32).item())              # blocks the fast decoder handed over
print(f"{os.path.basename(a.lib or lzo.LIB_PATH)}: compress {c[0]:.3f} ms (min {c[1]:.3f}), "
      f"decompress {d[0]:.3f} ms (min {d[1]:.3f}), z {int(zl.long().sum())}, ok {ok}, fallback {fb}", flush=True)
sys.exit(0 if ok else 1)
