"""Per-phase cycle stamps of the table-walk decoder (lzo1x_decode_ser.hip,
lzo_mi355x_debug_decompress_ser_stamps): mean cycles per block of each phase
for a lone 64 KiB ITB block and for C2 (4096 x 64 KiB), output checked.
--row: the row executor (lzo_mi355x_debug_decompress_row_stamps)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pomegranate_amd import lzo, synth  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
lib = lzo.load()
ROW = "--row" in sys.argv
fn = lib.lzo_mi355x_debug_decompress_row_stamps if ROW else lib.lzo_mi355x_debug_decompress_ser_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p] * 10 + [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
p = lambda x: x.data_ptr()
NAMES = ["stage+table", "walk", "decode+scan", "one-pass", "slow near", "far", "slow lits", "flush"]
if ROW:
    NAMES = ["stage+table", "walk", "decode+scan", "row set-up", "periodic", "doubling", "gather", "HBM/input"]


def run(sizes):
    arena, offs, lens = synth.batch(synth.ITB, 11, sizes, threads=16, align=256)
    nb = len(sizes)
    src = lzo.DeviceBatch(t(arena), t(offs.view(np.int64)), t(lens.view(np.int32)))
    caps = np.array([lzo.worst_compress(int(n)) for n in lens], dtype=np.uint32)
    zo = np.zeros(nb, dtype=np.uint64)
    zo[1:] = np.cumsum((caps[:-1].astype(np.uint64) + 255) // 256 * 256)
    za = torch.zeros(int(zo[-1]) + int(caps[-1]) + 256, dtype=torch.uint8, device=dev)
    zb = lzo.DeviceBatch(za, t(zo.view(np.int64)), t(caps.view(np.int32)))
    zl = torch.zeros(nb, dtype=torch.int32, device=dev)
    zs = torch.zeros_like(zl)
    lzo.compress_dev(src, zb, zl, zs)
    out = torch.zeros_like(src.arena)
    ol = torch.zeros_like(zl)
    st = torch.zeros_like(zl)
    head = torch.zeros(64, dtype=torch.int32, device=dev)
    ids = torch.zeros(nb, dtype=torch.int32, device=dev)
    stamps = torch.zeros(nb * 16, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream()
    for _ in range(2):
        head.zero_()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(s)
        rc = fn(p(za), p(zb.off), p(zl), p(out), p(src.off), p(src.length), p(ol), p(st), p(head),
                p(ids), nb, p(stamps), s.cuda_stream)
        ev1.record(s)
        torch.cuda.synchronize()
        assert rc == 0
    ok = int(head[0].item()) == 0 and torch.equal(out, src.arena)
    a = stamps.view(nb, 16).cpu().numpy().astype(np.float64).mean(axis=0)
    tot = a[:8].sum()          # (the walker's phases 0-1 overlap the executor's 2-7)
    print(f"blocks {nb}: kernel {ev0.elapsed_time(ev1):.3f} ms, exact {ok}, cycles/block {tot:.0f}")
    for i, nm in enumerate(NAMES):
        print(f"  {nm:12s} {a[i]:10.0f}  {100 * a[i] / tot:5.1f}%")
    if ROW:
        print("  windows %.1f  instructions %.1f  rows %.1f  doubling rounds %.1f  HBM/input rows %.1f"
              "  periodic rows %.1f  3+-instruction rows %.1f" % (a[8], a[9], a[10], a[11], a[12], a[14], a[15]))
    else:
        print("  windows %.1f  instructions %.1f  slow near %.1f  far %.1f  slow lits %.1f" % tuple(a[8:13]))
    print("  executor barrier waits %.0f cycles/block (walker: stage+table+walk %.0f; executor phases 2-7 %.0f)"
          % (a[13], a[0] + a[1], a[2:8].sum()))


run([65536])
run([65536] * 4096)
