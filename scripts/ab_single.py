"""A/B of single-call decompress latency between two builds of the library:
lzo1x_decompress of one 64 KiB and one 536,192-byte ITB block, median of
--calls calls each.  Usage: python scripts/ab_single.py [--lib PATH] [--calls N]"""
import argparse, ctypes, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401  (the library binds to torch's HIP runtime)
from pomegranate_amd import lzo, synth

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--calls", type=int, default=200)
a = ap.parse_args()
if a.lib:
    lzo.LIB_PATH = a.lib
lib = lzo.load()
assert lzo.lzo_init() == 0
res = {}
for n in (65536, 536192):
    blk = synth.block(synth.ITB, 4242, n)
    rc, zb = lzo.lzo1x_1_compress(blk)
    assert rc == 0
    z = ctypes.create_string_buffer(zb, len(zb))
    back = ctypes.create_string_buffer(n + 64)
    ol = ctypes.c_ulong(0)
    for _ in range(5):
        lib.lzo1x_decompress(z, len(zb), back, ctypes.byref(ol), None)
    ts = []
    for _ in range(a.calls):
        t0 = time.perf_counter()
        rc = lib.lzo1x_decompress(z, len(zb), back, ctypes.byref(ol), None)
        ts.append(time.perf_counter() - t0)
    assert rc == 0 and ol.value == n and back.raw[:n] == blk
    res[n] = round(float(np.median(ts)) * 1e6, 1)
print(os.path.basename(a.lib or lzo.LIB_PATH), "decompress us (median):", res, flush=True)
