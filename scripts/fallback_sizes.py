"""Which block sizes does the fast decoder hand to the exact decoder?"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from pomegranate_amd import lzo, synth
if len(sys.argv) > 1:
    lzo.LIB_PATH = sys.argv[1]
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
cases = [(synth.ITB, k) for k in (4, 64, 96, 124, 128, 160, 192, 256)]
cases += [(m, 64) for m in (synth.RANDOM, synth.ZEROS, synth.ALPHA4, synth.LZLIKE, synth.TEXT)]
for model, kib in cases:
    nb = 64
    arena, offs, lens = synth.batch(model, 0, [kib * 1024] * nb, align=256, threads=16)
    src = lzo.DeviceBatch(t(arena), t(offs.view(np.int64)), t(lens.view(np.int32)))
    caps = np.array([lzo.worst_compress(int(n)) for n in lens], dtype=np.uint64)
    zo = np.zeros(nb, dtype=np.uint64); zo[1:] = np.cumsum((caps[:-1] + 255) // 256 * 256)
    za = torch.zeros(int(zo[-1] + caps[-1]) + 256, dtype=torch.uint8, device=dev)
    zb = lzo.DeviceBatch(za, t(zo.view(np.int64)), t(caps.astype(np.uint32).view(np.int32)))
    zl = torch.zeros(nb, dtype=torch.int32, device=dev); zs = torch.zeros_like(zl)
    lzo.compress_dev(src, zb, zl, zs)
    out = torch.zeros_like(src.arena); ob = lzo.DeviceBatch(out, src.off, src.length)
    ol = torch.zeros_like(zl); st = torch.zeros_like(zl)
    scr = torch.zeros(lzo.decompress_scratch_bytes(nb), dtype=torch.uint8, device=dev)
    lzo.decompress_dev(lzo.DeviceBatch(za, zb.off, zl), ob, ol, st, scr)
    torch.cuda.synchronize()
    fb = int(scr[:4].view(torch.int32).item())
    print(synth.MODEL_NAMES[model], kib, "KiB: zlen", int(zl[0].item()), "fallback", fb, "ok", torch.equal(out, src.arena),
          "zst", int((zs != 0).sum().item()), flush=True)
