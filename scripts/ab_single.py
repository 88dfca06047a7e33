"""A/B of single-call latency between two builds of the library (or debug
keys, POM_LZO_DEBUG): lzo1x_decompress (--op decompress) or lzo1x_1_compress
(--op compress) of one 64 KiB and one 536,192-byte ITB block, median of
--calls calls each, outputs checked.
Usage: python scripts/ab_single.py [--lib PATH] [--calls N] [--op OP]"""
import argparse, ctypes, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401  (the library binds to torch's HIP runtime)
from pomegranate_amd import lzo, synth

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--calls", type=int, default=200)
ap.add_argument("--op", choices=("decompress", "compress"), default="decompress")
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
    if a.op == "compress":
        src = ctypes.create_string_buffer(blk, n)
        out = ctypes.create_string_buffer(lzo.worst_compress(n))
        wrk = ctypes.create_string_buffer(lzo.LZO1X_1_MEM_COMPRESS)
        call = lambda: lib.lzo1x_1_compress(src, n, out, ctypes.byref(ol), wrk)
    else:
        call = lambda: lib.lzo1x_decompress(z, len(zb), back, ctypes.byref(ol), None)
    for _ in range(5):
        call()
    ts = []
    for _ in range(a.calls):
        t0 = time.perf_counter()
        rc = call()
        ts.append(time.perf_counter() - t0)
    if a.op == "compress":
        assert rc == 0 and out.raw[:ol.value] == zb
    else:
        assert rc == 0 and ol.value == n and back.raw[:n] == blk
    res[n] = round(float(np.median(ts)) * 1e6, 1)
print(os.path.basename(a.lib or lzo.LIB_PATH), os.environ.get("POM_LZO_DEBUG", ""), a.op,
      "us (median):", res, flush=True)
