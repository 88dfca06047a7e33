"""A/B of the throughput decoders (fast, win, ser, row) on one GPU: the round-2 op-set decoder
(lzo_mi355x_launch_decompress_fast) and the windowed decoder
(lzo_mi355x_launch_decompress_win), kernel time by HIP events, output checked.
Workloads: C2 (4096 x 64 KiB ITB), lone blocks (one 64 KiB, one 536,192 B ITB
block), and a C5-like batch (1024 ITB records, 12,416-536,192 B)."""
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
fast = lib.lzo_mi355x_launch_decompress_fast
fast.restype = ctypes.c_int
fast.argtypes = [ctypes.c_void_p] * 13 + [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
win = lib.lzo_mi355x_launch_decompress_win
win.restype = ctypes.c_int
win.argtypes = [ctypes.c_void_p] * 10 + [ctypes.c_uint32, ctypes.c_void_p]
# the table-walk and row decoders are experiments outside the product library
_exp = ctypes.CDLL(os.path.join(ROOT, "scripts", "experiments", "libdecode_ser.so"))
ser = _exp.lzo_mi355x_launch_decompress_ser
ser.restype = ctypes.c_int
ser.argtypes = win.argtypes
row = _exp.lzo_mi355x_launch_decompress_row
row.restype = ctypes.c_int
row.argtypes = win.argtypes
lib.lzo_mi355x_fast_ops_bytes_per_block.restype = ctypes.c_size_t
lib.lzo_mi355x_fast_resident_blocks.restype = ctypes.c_uint32
p = lambda x: x.data_ptr()
mix_streams = (torch.cuda.Stream(), torch.cuda.Stream())


def setup(sizes, seed):
    arena, offs, lens = synth.batch(synth.ITB, seed, sizes, threads=16, align=256)
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
    torch.cuda.synchronize()
    return src, za, zb, zl, nb


def run(kind, src, za, zb, zl, nb, reps):
    out = torch.zeros_like(src.arena)
    ol = torch.zeros_like(zl)
    st = torch.zeros_like(zl)
    head = torch.zeros(64 + 2048, dtype=torch.int32, device=dev)
    ids = torch.zeros(nb, dtype=torch.int32, device=dev)
    nsets = min(nb, int(lib.lzo_mi355x_fast_resident_blocks()))
    ring = torch.zeros(max(nsets, 1), dtype=torch.int64, device=dev)
    ops = torch.empty(max(nsets, 1) * lib.lzo_mi355x_fast_ops_bytes_per_block(), dtype=torch.uint8,
                      device=dev)
    s = torch.cuda.current_stream()
    head2 = torch.zeros(64, dtype=torch.int32, device=dev)
    ids2 = torch.zeros(nb, dtype=torch.int32, device=dev)
    ts = []
    for _ in range(reps):
        head.zero_()
        head2.zero_()
        ring.zero_()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(s)
        if kind.startswith("mix"):
            # blocks [0, nf) on the op-set decoder, [nf, nb) on the table-walk
            # decoder, on two streams at once: their workgroups share the CUs
            # (op-set: SALU-heavy; table-walk: VALU-heavy)
            nf = nb * (100 - int(kind[3:])) // 100
            s1, s2 = mix_streams
            s1.wait_stream(s)
            s2.wait_stream(s)
            rc = fast(p(za), p(zb.off), p(zl), p(out), p(src.off), p(src.length), p(ol), p(st),
                      p(head), p(ids), p(head) + 256, p(ring), p(ops), nsets, nf, s1.cuda_stream)
            rc |= ser(p(za), p(zb.off) + 8 * nf, p(zl) + 4 * nf, p(out), p(src.off) + 8 * nf,
                      p(src.length) + 4 * nf, p(ol) + 4 * nf, p(st) + 4 * nf, p(head2), p(ids2),
                      nb - nf, s2.cuda_stream)
            s.wait_stream(s1)
            s.wait_stream(s2)
        elif kind == "fast":
            rc = fast(p(za), p(zb.off), p(zl), p(out), p(src.off), p(src.length), p(ol), p(st),
                      p(head), p(ids), p(head) + 256, p(ring), p(ops), nsets, nb, s.cuda_stream)
        else:
            rc = {"ser": ser, "row": row}.get(kind, win)(p(za), p(zb.off), p(zl), p(out), p(src.off), p(src.length), p(ol), p(st),
                     p(head), p(ids), nb, s.cuda_stream)
        ev1.record(s)
        torch.cuda.synchronize()
        assert rc == 0
        ts.append(ev0.elapsed_time(ev1))
    fb = int(head[0].item()) + int(head2[0].item())
    ok = fb == 0 and torch.equal(out, src.arena)
    return float(np.median(ts)), ok, fb


KINDS = (sys.argv[1] if len(sys.argv) > 1 else "fast,win,ser").split(",")
ONLY = sys.argv[2].split(",") if len(sys.argv) > 2 else None
res = {}
cases = {
    "c2_4096x64k": [65536] * 4096,
    "lone_64k": [65536],
    "lone_536k": [536192],
    "c5_like_1024": [int(x) for x in np.random.default_rng(3).choice(
        [12416, 40000, 65536, 131072, 262144, 536192], 1024, p=[.3, .2, .2, .15, .1, .05])],
}
cases["c4_8192mixed"] = [int(x) for x in synth.mixed_sizes(8192, 5)]
for name, sizes in cases.items():
    if ONLY and name not in ONLY:
        continue
    src, za, zb, zl, nb = setup(sizes, 11)
    n = int(src.length.long().sum())
    for kind in KINDS:
        ms, ok, fb = run(kind, src, za, zb, zl, nb, 5)
        res[f"{name}/{kind}"] = {"ms": round(ms, 4), "gibps": round(n / (ms / 1e3) / 2**30, 2), "ok": ok,
                                 "fallbacks": fb}
        print(name, kind, res[f"{name}/{kind}"], flush=True)
