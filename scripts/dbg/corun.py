"""Co-residency study: the C3 encoder and the decoder launched at the same time
on two streams (independent batches: decode of the previous round trip's
output while the next one compresses), against each alone.  Kernel wall time
by HIP events around both; outputs checked.  Usage: python scripts/dbg/corun.py [--lib PATH]"""
import argparse, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
from pomegranate_amd import lzo, synth

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--order", default="enc_first", choices=("enc_first", "dec_first"))
a = ap.parse_args()
if a.lib:
    lzo.LIB_PATH = a.lib
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
lzo.load()
nb = 4096
arena, offs, lens = synth.batch(synth.ITB, 0, [65536] * nb, align=256, threads=16)
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
src = lzo.DeviceBatch(t(arena), t(offs.view(np.int64)), t(lens.view(np.int32)))
caps = np.array([lzo.worst_compress(int(n)) for n in lens], dtype=np.uint64)
zo = np.zeros(nb, dtype=np.uint64); zo[1:] = np.cumsum((caps[:-1] + 255) // 256 * 256)


def zbatch():
    za = torch.zeros(int(zo[-1] + caps[-1]) + 256, dtype=torch.uint8, device=dev)
    return lzo.DeviceBatch(za, t(zo.view(np.int64)), t(caps.astype(np.uint32).view(np.int32)))


zb1, zb2 = zbatch(), zbatch()
zl1 = torch.zeros(nb, dtype=torch.int32, device=dev); zs1 = torch.zeros_like(zl1)
zl2 = torch.zeros_like(zl1); zs2 = torch.zeros_like(zl1)
escr = torch.empty(lzo.compress_scratch_bytes(nb), dtype=torch.uint8, device=dev)
lzo.compress_dev(src, zb2, zl2, zs2, scratch=escr)          # the batch the decoder works on
torch.cuda.synchronize()
zsrc2 = lzo.DeviceBatch(zb2.arena, zb2.off, zl2)
out = torch.zeros_like(src.arena); ob = lzo.DeviceBatch(out, src.off, src.length)
ol = torch.zeros_like(zl1); st = torch.zeros_like(zl1)
dscr = torch.empty(lzo.decompress_scratch_bytes(nb), dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def enc(s):
    lzo.compress_dev(src, zb1, zl1, zs1, scratch=escr, stream=s)


def dec(s):
    lzo.decompress_dev(zsrc2, ob, ol, st, dscr, stream=s)


def timed(fn):
    ts = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        torch.cuda.synchronize()
        e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


cur = torch.cuda.current_stream()
te = timed(lambda: enc(cur))
td = timed(lambda: dec(cur))
tseq = timed(lambda: (enc(cur), dec(cur)))


def both():
    s1.wait_stream(cur); s2.wait_stream(cur)
    if a.order == "enc_first":
        enc(s1); dec(s2)
    else:
        dec(s2); enc(s1)
    cur.wait_stream(s1); cur.wait_stream(s2)


tco = timed(both)
ok = torch.equal(out, src.arena) and bool((st == 0).all()) and bool((zs1 == 0).all())
print(f"{os.path.basename(a.lib or lzo.LIB_PATH)} {a.order}: encode {te:.3f} ms, decode {td:.3f} ms, "
      f"sequential {tseq:.3f} ms, co-run {tco:.3f} ms, ok {ok}", flush=True)
sys.exit(0 if ok else 1)
