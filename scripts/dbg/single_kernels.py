"""Latency of one block alone through the throughput decoder (fast + exact
pass) and through the exact one-wave decoder only (GPU box)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
from pomegranate_amd import lzo, synth
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
for n in (12416, 65536, 536192):
    arena, offs, lens = synth.batch(synth.ITB, 0, [n], align=256, threads=1)
    src = lzo.DeviceBatch(t(arena), t(offs.view(np.int64)), t(lens.view(np.int32)))
    cap = lzo.worst_compress(n)
    za = torch.zeros(cap + 256, dtype=torch.uint8, device=dev)
    zb = lzo.DeviceBatch(za, t(np.zeros(1, np.int64)), t(np.array([cap], np.int32)))
    zl = torch.zeros(1, dtype=torch.int32, device=dev); zs = torch.zeros_like(zl)
    lzo.compress_dev(src, zb, zl, zs, scratch=None); torch.cuda.synchronize()
    zsrc = lzo.DeviceBatch(za, zb.off, zl)
    out = torch.zeros_like(src.arena); ob = lzo.DeviceBatch(out, src.off, src.length)
    ol = torch.zeros_like(zl); st = torch.zeros_like(zl)
    scr = torch.zeros(lzo.decompress_scratch_bytes(1), dtype=torch.uint8, device=dev)
    res = {}
    for name, s in (("fast", scr), ("exact", None)):
        ts = []
        for _ in range(8):
            out.zero_()
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record(); lzo.decompress_dev(zsrc, ob, ol, st, s); e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        res[name] = (round(float(np.median(ts[2:])), 1), bool(torch.equal(out, src.arena)) and int(st.item()) == 0)
    cts = {}
    for name, s in (("gdict1", "auto"), ("lds", None)):
        ts = []
        for _ in range(6):
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record(); lzo.compress_dev(src, zb, zl, zs, scratch=s); e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        cts[name] = round(float(np.median(ts[2:])), 1)
    print(n, "decode us (fast+exact pass, exact only):", res, "compress us:", cts, flush=True)
