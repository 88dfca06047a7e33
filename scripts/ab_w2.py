"""A/B of the encoder kernels on C3 (4096 x 64 KiB ITB blocks) or on lone
blocks (--lone), with byte identity of the outputs: the default kernels (w1)
against 128-position windows (w2, POM_LZO_DEBUG enc_w2=1) and dictionaries
zeroed by a memset before the launch (pre, enc_prezero=1).  w2 and pre are
keys of scripts/experiments/encode_w2.patch (git apply it first); without the
patch every mode runs the default kernels.  DESIGN.md 3.9, profiles/r04c/.
Usage: python scripts/ab_w2.py [--model itb] [--lone [--bytes N]] [--modes w1,w2]"""
import argparse, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from pomegranate_amd import lzo, synth

ap = argparse.ArgumentParser()
ap.add_argument("--blocks", type=int, default=4096)
ap.add_argument("--bytes", type=int, default=65536)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--model", default="itb")
ap.add_argument("--lone", action="store_true",
                help="one block per launch, no scratch (the LDS-dictionary kernels of single calls)")
ap.add_argument("--modes", default="w1,w2,w1,w2",
                help="w1 (default kernels), w2 (enc_w2=1), pre (enc_prezero=1)")
ap.add_argument("--lib", default=None, help="another build of the library (counterfactual A/B)")
a = ap.parse_args()
if a.lib:
    lzo.LIB_PATH = a.lib
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
lzo.load()
model = {v: k for k, v in synth.MODEL_NAMES.items()}[a.model]
nb = 1 if a.lone else a.blocks
arena, offs, lens = synth.batch(model, 0, [a.bytes] * nb, align=256, threads=16)
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
src = lzo.DeviceBatch(t(arena), t(offs.view(np.int64)), t(lens.view(np.int32)))
caps = np.array([lzo.worst_compress(int(n)) for n in lens], dtype=np.uint64)
zo = np.zeros(nb, dtype=np.uint64); zo[1:] = np.cumsum((caps[:-1] + 255) // 256 * 256)
za = torch.zeros(int(zo[-1] + caps[-1]) + 256, dtype=torch.uint8, device=dev)
zb = lzo.DeviceBatch(za, t(zo.view(np.int64)), t(caps.astype(np.uint32).view(np.int32)))
zl = torch.zeros(nb, dtype=torch.int32, device=dev); zs = torch.zeros_like(zl)
scr = torch.empty(max(lzo.compress_scratch_bytes(nb), 1), dtype=torch.uint8, device=dev)
outs = {}
ENV = {"w1": "", "w2": "enc_w2=1", "pre": "enc_prezero=1"}
for mode in a.modes.split(","):
    os.environ["POM_LZO_DEBUG"] = ENV[mode]
    ts = []
    for _ in range(a.reps):
        za.zero_()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        lzo.compress_dev(src, zb, zl, zs, scratch=None if a.lone else scr)
        e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    got = (za.clone(), zl.clone(), zs.clone())
    same = ""
    if mode in outs:
        pass
    elif "w1" in outs:
        r = outs["w1"]
        same = f", identical to w1 {torch.equal(got[0], r[0]) and torch.equal(got[1], r[1])}"
    outs.setdefault(mode, got)
    gib = nb * a.bytes / 2**30
    med = float(np.median(ts))
    print(f"{mode}{' lone ' + str(a.bytes) if a.lone else ''}: {med:.3f} ms (min {min(ts):.3f}) = {gib / med * 1e3:.1f} GiB/s, status ok {bool((zs == 0).all())}{same}",
          flush=True)
