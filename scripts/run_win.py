"""Driver for profiling the windowed decoder alone (lzo_mi355x_launch_decompress_win)
on N x 64 KiB ITB blocks (default 256: one block per CU), R launches."""
import argparse, ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from pomegranate_amd import lzo, synth

ap = argparse.ArgumentParser()
ap.add_argument("--blocks", type=int, default=256)
ap.add_argument("--bytes", type=int, default=65536)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
arena, offs, lens = synth.batch(synth.ITB, 0, [a.bytes] * a.blocks, threads=16, align=256)
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
nb = a.blocks
src = lzo.DeviceBatch(t(arena), t(offs.view(np.int64)), t(lens.view(np.int32)))
caps = np.array([lzo.worst_compress(int(n)) for n in lens], dtype=np.uint32)
zo = np.zeros(nb, dtype=np.uint64); zo[1:] = np.cumsum((caps[:-1].astype(np.uint64) + 255) // 256 * 256)
za = torch.zeros(int(zo[-1]) + int(caps[-1]) + 256, dtype=torch.uint8, device=dev)
zb = lzo.DeviceBatch(za, t(zo.view(np.int64)), t(caps.view(np.int32)))
zl = torch.zeros(nb, dtype=torch.int32, device=dev); zs = torch.zeros_like(zl)
lzo.compress_dev(src, zb, zl, zs)
torch.cuda.synchronize()
lib = lzo.load()
fn = lib.lzo_mi355x_launch_decompress_win
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p] * 10 + [ctypes.c_uint32, ctypes.c_void_p]
out = torch.zeros_like(src.arena); ol = torch.zeros_like(zl); st = torch.zeros_like(zl)
head = torch.zeros(64, dtype=torch.int32, device=dev); ids = torch.zeros(nb, dtype=torch.int32, device=dev)
p = lambda x: x.data_ptr()
for _ in range(a.reps):
    head.zero_()
    fn(p(za), p(zb.off), p(zl), p(out), p(src.off), p(src.length), p(ol), p(st), p(head), p(ids), nb,
       torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
ok = torch.equal(out, src.arena) and int(head[0].item()) == 0
print({"blocks": nb, "ok": ok})
sys.exit(0 if ok else 1)
