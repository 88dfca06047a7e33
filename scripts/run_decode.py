"""Driver for profiling one kernel family on the bench workload (4096 x 64 KiB
ITB blocks): --op decode (default) compresses once on the GPU, then decodes
--reps times; --op encode compresses --reps times (with the dictionary
scratch, as bench.py does), then checks one decode."""
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
ap.add_argument("--lib", default=None, help="alternative liblzo_mi355x.so build")
ap.add_argument("--noverify", action="store_true", help="exit 0 even if the output differs (timing variants)")
ap.add_argument("--op", choices=("decode", "encode"), default="decode")
a = ap.parse_args()
if a.lib:
    lzo.LIB_PATH = a.lib
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
model = {v: k for k, v in synth.MODEL_NAMES.items()}[a.model]
arena, offs, lens = synth.batch(model, 0, [a.bytes] * a.blocks, threads=16)
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
nb = a.blocks
src = lzo.DeviceBatch(t(arena), t(offs.view(np.int64)), t(lens.view(np.int32)))
caps = np.array([lzo.worst_compress(int(n)) for n in lens], dtype=np.uint32)
zo = np.zeros(nb, dtype=np.uint64); zo[1:] = np.cumsum((caps[:-1].astype(np.uint64) + 255) // 256 * 256)
za = torch.zeros(int(zo[-1]) + int(caps[-1]) + 256, dtype=torch.uint8, device=dev)
zb = lzo.DeviceBatch(za, t(zo.view(np.int64)), t(caps.view(np.int32)))
zl = torch.zeros(nb, dtype=torch.int32, device=dev); zs = torch.zeros_like(zl)
for _ in range(a.reps if a.op == "encode" else 1):
    lzo.compress_dev(src, zb, zl, zs)
torch.cuda.synchronize()
zsrc = lzo.DeviceBatch(za, zb.off, zl)
out = torch.zeros_like(src.arena); ob = lzo.DeviceBatch(out, src.off, src.length)
ol = torch.zeros_like(zl); st = torch.zeros_like(zl)
scr = torch.empty(lzo.decompress_scratch_bytes(nb), dtype=torch.uint8, device=dev)
for _ in range(a.reps if a.op == "decode" else 1):
    lzo.decompress_dev(zsrc, ob, ol, st, scr)
torch.cuda.synchronize()
ok = torch.equal(out, src.arena) and bool((st == 0).all())
print({"blocks": nb, "n_bytes": int(lens.astype(np.int64).sum()), "z_bytes": int(zl.long().sum()),
       "reps": a.reps, "op": a.op, "ok": ok}, flush=True)
sys.exit(0 if ok or a.noverify else 1)
