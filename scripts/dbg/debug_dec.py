"""Decode the edge vectors on the GPU; for mismatches print the ops around
the first differing byte."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.dirname(__file__))
import numpy as np, torch
import gpu_util as gu
from lzo_ops import parse
z = np.load(os.path.join(ROOT, "tests/golden/edge.npz"))
def unpack(d, o): return [d[o[i]:o[i+1]].tobytes() for i in range(len(o)-1)]
names = [str(s) for s in z["names"]]; ins = unpack(z["in_data"], z["in_off"]); comps = unpack(z["z_data"], z["z_off"])
dev = torch.device("cuda:0")
outs, st, _ = gu.gpu_decompress(torch, comps, [len(d) for d in ins], dev)
nbad = 0
for n, o, d, c, s in zip(names, outs, ins, comps, st):
    if o == d: continue
    nbad += 1
    if nbad > 6: continue
    i = next((k for k in range(min(len(o), len(d))) if o[k] != d[k]), min(len(o), len(d)))
    print(f"== {n} status {s} len {len(o)}/{len(d)} first diff at {i}")
    ops, _ = parse(c)
    for op in ops:
        if op[1] <= i + 16 and op[1] + op[2] >= i - 48:
            print("   ", op, "OUT" if op[1] <= i < op[1] + op[2] else "")
    print("   got ", o[max(0,i-8):i+24].hex())
    print("   want", d[max(0,i-8):i+24].hex())
print("bad", nbad, "of", len(names))
