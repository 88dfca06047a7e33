"""Per-phase cycle stamps of the windowed decoder (lzo_mi355x_debug_decompress_win_stamps)
on the C2 workload (4096 x 64 KiB ITB blocks, or --blocks/--bytes/--model):
thread 0's view of each block, averaged over blocks."""
import argparse, ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from pomegranate_amd import lzo, synth

ap = argparse.ArgumentParser()
ap.add_argument("--blocks", type=int, default=4096)
ap.add_argument("--bytes", type=int, default=65536)
ap.add_argument("--model", default="itb")
a = ap.parse_args()
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
model = {v: k for k, v in synth.MODEL_NAMES.items()}[a.model]
arena, offs, lens = synth.batch(model, 0, [a.bytes] * a.blocks, threads=16, align=256)
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
out = torch.zeros_like(src.arena)
ol = torch.zeros_like(zl); st = torch.zeros_like(zl)
head = torch.zeros(64, dtype=torch.int32, device=dev)
ids = torch.zeros(nb, dtype=torch.int32, device=dev)
stamps = torch.zeros(nb * 16, dtype=torch.int64, device=dev)
lib = lzo.load()
fn = lib.lzo_mi355x_debug_decompress_win_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p] * 10 + [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
p = lambda x: x.data_ptr()
s = torch.cuda.current_stream()
for rep in range(2):
    head.zero_(); stamps.zero_()
    ev0 = torch.cuda.Event(enable_timing=True); ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(s)
    rc = fn(p(za), p(zb.off), p(zl), p(out), p(src.off), p(src.length), p(ol), p(st), p(head), p(ids),
            nb, p(stamps), s.cuda_stream)
    ev1.record(s)
    torch.cuda.synchronize()
ok = torch.equal(out, src.arena)
S = stamps.view(nb, 16).cpu().numpy().astype(np.float64)
names = ["stage", "spec", "settle", "count+scan", "emit", "w_bitmap", "w_ptrs", "w_chase", "w_gather",
         "windows", "pieces", "chase_rounds", "settle_rounds", "settle_walk_cycles", "settle_walk_tokens"]
tot = S[:, :9].sum(axis=1)
print({"ok": ok, "fallbacks": int(head[0].item()), "kernel_ms": round(ev0.elapsed_time(ev1), 4),
       "cycles_per_block_mean": round(float(tot.mean())), "cycles_per_block_max": round(float(tot.max()))})
for i, n in enumerate(names):
    print(f"  {n:14s} mean {S[:, i].mean():12.1f}   ({100 * S[:, i].mean() / tot.mean():5.1f}% of cycles)" if i < 9
          else f"  {n:14s} mean {S[:, i].mean():12.1f}")
