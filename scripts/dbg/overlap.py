"""Diagnostic: do the C3 encoder and decoder kernels share the GPU?  Times K
launches of the encoder alone, the decoder alone, and both issued together on
two streams (encoder of one batch copy, decoder of another: no data between
them), median wall per launch pair.  Usage: python scripts/dbg/overlap.py"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
from pomegranate_amd import lzo, synth
import bench

dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
lzo.load()
nb = 4096
R = bench.Resident(torch, lzo, synth, dev, synth.ITB, [65536] * nb, np.arange(nb, dtype=np.uint64))
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
zd2 = lzo.DeviceBatch(torch.empty_like(R.zdst.arena), R.zdst.off, R.zdst.length)
zl2, zs2 = torch.zeros_like(R.zlen), torch.zeros_like(R.zst)
cs2 = torch.empty_like(R.cscratch)


def enc(s):
    lzo.compress_dev(R.src, zd2, zl2, zs2, stream=s, scratch=cs2)


def dec(s):
    lzo.decompress_dev(R.zsrc, R.odst, R.olen, R.ost, R.scratch, stream=s)


def timed(fn, k=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(k):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


te = timed(lambda: enc(s1))
td = timed(lambda: dec(s1))
tb = timed(lambda: (enc(s1), dec(s2)))
tb2 = timed(lambda: (dec(s2), enc(s1)))
ok = torch.equal(R.out, R.src.arena) and bool((R.ost == 0).all()) and bool((zs2 == 0).all())
print(f"encode {te:.3f} ms, decode {td:.3f} ms, sum {te + td:.3f}; together (enc first) {tb:.3f}, "
      f"(dec first) {tb2:.3f} ms; exact {ok}", flush=True)
