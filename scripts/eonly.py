"""Timing experiment: the executor alone.  Build two variants with 16 slots:
  rec:    -DPOM_SLOTS=16 -DPOM_EXPERIMENT_RECORD   (normal decode, pieces kept)
  replay: -DPOM_SLOTS=16 -DPOM_EXPERIMENT_REPLAY   (executor only, on rec's ops)
Usage: python scripts/eonly.py LIB_REC LIB_REPLAY"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from pomegranate_amd import lzo, synth
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
lzo.LIB_PATH = sys.argv[1]
lib = lzo.load()
rep = ctypes.CDLL(sys.argv[2])
nb = 4096
arena, offs, lens = synth.batch(synth.ITB, 0, [65536] * nb, align=256, threads=16)
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
src = lzo.DeviceBatch(t(arena), t(offs.view(np.int64)), t(lens.view(np.int32)))
caps = np.array([lzo.worst_compress(int(n)) for n in lens], dtype=np.uint64)
zo = np.zeros(nb, dtype=np.uint64); zo[1:] = np.cumsum((caps[:-1] + 255) // 256 * 256)
za = torch.zeros(int(zo[-1] + caps[-1]) + 256, dtype=torch.uint8, device=dev)
zb = lzo.DeviceBatch(za, t(zo.view(np.int64)), t(caps.astype(np.uint32).view(np.int32)))
zl = torch.zeros(nb, dtype=torch.int32, device=dev); zs = torch.zeros_like(zl)
lzo.compress_dev(src, zb, zl, zs); torch.cuda.synchronize()
out = torch.zeros_like(src.arena)
ol = torch.zeros_like(zl); st = torch.zeros_like(zl)
fb = torch.zeros(nb + 1, dtype=torch.int32, device=dev)
lib.lzo_mi355x_fast_ops_bytes_per_block.restype = ctypes.c_size_t
ops = torch.zeros(nb * lib.lzo_mi355x_fast_ops_bytes_per_block(), dtype=torch.uint8, device=dev)
p = lambda x: x.data_ptr()
sh = torch.cuda.current_stream().cuda_stream
for name, L in (("rec", lib), ("replay", rep)):
    f = L.lzo_mi355x_launch_decompress_fast
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p] * 10 + [ctypes.c_uint32, ctypes.c_void_p]
    ts = []
    for _ in range(6):
        out.zero_(); fb.zero_()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        f(p(za), p(zb.off), p(zl), p(out), p(src.off), p(src.length), p(ol), p(st), p(fb), p(ops), nb, sh)
        e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(name, f"{float(np.median(ts)):.3f} ms", "fallback", int(fb[0].item()), "equal", torch.equal(out, src.arena))
