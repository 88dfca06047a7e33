"""Diagnostic: phase breakdown of the throughput encoder's parse wave
(s_memtime stamps build).  Usage: python scripts/diag_encode.py [--blocks N] [--model itb]"""
import argparse, ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from pomegranate_amd import lzo, synth

ap = argparse.ArgumentParser()
ap.add_argument("--blocks", type=int, default=4096)
ap.add_argument("--model", default="itb")
ap.add_argument("--bytes", type=int, default=65536)
ap.add_argument("--lib", default=None)
ap.add_argument("--nostamps", action="store_true")
a = ap.parse_args()
if a.lib:
    lzo.LIB_PATH = a.lib
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
lib = lzo.load()
model = {v: k for k, v in synth.MODEL_NAMES.items()}[a.model]
arena, offs, lens = synth.batch(model, 0, [a.bytes] * a.blocks, align=256, threads=16)
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
nb = a.blocks
src = lzo.DeviceBatch(t(arena), t(offs.view(np.int64)), t(lens.view(np.int32)))
caps = np.array([lzo.worst_compress(int(n)) for n in lens], dtype=np.uint64)
zo = np.zeros(nb, dtype=np.uint64); zo[1:] = np.cumsum((caps[:-1] + 255) // 256 * 256)
za = torch.zeros(int(zo[-1] + caps[-1]) + 256, dtype=torch.uint8, device=dev)
zb = lzo.DeviceBatch(za, t(zo.view(np.int64)), t(caps.astype(np.uint32).view(np.int32)))
zl = torch.zeros(nb, dtype=torch.int32, device=dev); zs = torch.zeros_like(zl)
SLOTS = 16
stamps = torch.zeros(nb * SLOTS, dtype=torch.int64, device=dev)
fn = getattr(lib, "lzo_mi355x_debug_compress_fast_stamps", None)
if fn is not None:
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p] * 8 + [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
gfn = getattr(lib, "lzo_mi355x_debug_compress_gdict_stamps", None)
if gfn is not None:
    gfn.restype = ctypes.c_int
    gfn.argtypes = [ctypes.c_void_p] * 8 + [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t,
                                            ctypes.c_void_p, ctypes.c_void_p]
g1fn = getattr(lib, "lzo_mi355x_debug_compress_gdict1_stamps", None)
if g1fn is not None:
    g1fn.restype = ctypes.c_int
    g1fn.argtypes = gfn.argtypes
p = lambda x: x.data_ptr()
sh = torch.cuda.current_stream().cuda_stream
scr = torch.empty(max(lzo.compress_scratch_bytes(nb), 1), dtype=torch.uint8, device=dev)
ref_out = None
gstamps = torch.zeros(nb * SLOTS, dtype=torch.int64, device=dev)
g1stamps = torch.zeros(nb * SLOTS, dtype=torch.int64, device=dev)
STAMPED = ("stamps", "gstamps", "g1stamps")
for mode in ("lds", "gdict", "stamps", "gstamps", "g1stamps"):
    if mode in STAMPED and (fn is None or gfn is None or g1fn is None or a.nostamps):
        continue
    ts = []
    for _ in range(1 if mode in STAMPED else 5):
        za.zero_()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        if mode == "stamps":
            fn(p(src.arena), p(src.off), p(src.length), p(za), p(zb.off), p(zb.length), p(zl), p(zs), nb, p(stamps), sh)
        elif mode == "gstamps":
            gfn(p(src.arena), p(src.off), p(src.length), p(za), p(zb.off), p(zb.length), p(zl), p(zs), nb,
                p(scr), scr.numel(), p(gstamps), sh)
        elif mode == "g1stamps":               # (the bench's one-wave kernel)
            g1fn(p(src.arena), p(src.off), p(src.length), p(za), p(zb.off), p(zb.length), p(zl), p(zs), nb,
                 p(scr), scr.numel(), p(g1stamps), sh)
        else:
            lzo.compress_dev(src, zb, zl, zs, scratch=scr if mode == "gdict" else None)
        e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    same = ""
    if mode not in STAMPED:
        got = (za.clone(), zl.clone())
        if ref_out is None:
            ref_out = got
        else:
            same = f", identical to lds {torch.equal(got[0], ref_out[0]) and torch.equal(got[1], ref_out[1])}"
    print(f"{mode}: {float(np.median(ts)):.3f} ms (min {min(ts):.3f}), status ok {bool((zs == 0).all())}{same}")
if fn is None or a.nostamps:
    sys.exit(0)
phases = ["setup", "probe", "cand", "path", "claim", "tok", "dict", "pushwait"]
counts = ["windows", "extend", "tokens", "pathit", "extit", "end_cross", "end_cap", "fwd"]
for name, t_ in (("lds", stamps), ("gdict", gstamps), ("gdict1", g1stamps)):
    st = t_.view(nb, SLOTS).double().cpu().numpy()
    print(name, "parse cycles/block (mean):", {n: int(st[:, i].mean()) for i, n in enumerate(phases)},
          "total", int(st[:, :len(phases)].sum(1).mean()))
    print(name, "counts/block (mean):", {n: round(float(st[:, len(phases) + i].mean()), 1) for i, n in enumerate(counts)})
