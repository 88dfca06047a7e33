"""Segment-row decoder (lzo1x_decode_seg.hip) against the op-set decoder
(lzo1x_decode_fast.hip) on one GPU: kernel time by HIP events on the launch
stream, output checked against the input, blocks handed to the exact decoder
counted.  Workloads: C2 (4096 x 64 KiB ITB), C4-like (8192 mixed 4-256 KiB),
C5-like (1024 ITB records), lone 64 KiB and 536,192 B blocks.

    python scripts/seg_check.py [reps] [kinds...]   (kinds: fast seg ser)
"""
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
p = lambda x: x.data_ptr()
fast = lib.lzo_mi355x_launch_decompress_fast
fast.restype = ctypes.c_int
fast.argtypes = [ctypes.c_void_p] * 13 + [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
one = {}
for k in ("seg", "ser", "win", "quad"):
    f = getattr(lib, f"lzo_mi355x_launch_decompress_{k}", None)
    xp = os.path.join(ROOT, "scripts", "experiments", f"libdecode_{k}.so")
    if f is None and os.path.exists(xp):           # (rejected decoders: scripts/experiments)
        f = getattr(ctypes.CDLL(xp), f"lzo_mi355x_launch_decompress_{k}", None)
    if f is not None:
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p] * 10 + [ctypes.c_uint32, ctypes.c_void_p]
        one[k] = f
lib.lzo_mi355x_fast_ops_bytes_per_block.restype = ctypes.c_size_t
lib.lzo_mi355x_fast_resident_blocks.restype = ctypes.c_uint32


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
    assert int((zs != 0).sum().item()) == 0
    return src, zb, zl, nb


def variant(kind):
    """kind "seg@path.so": the seg launcher of a variant build (scripts/ab/)."""
    if "@" in kind and kind not in one:
        v = ctypes.CDLL(os.path.join(ROOT, kind.split("@", 1)[1]))
        f = v.lzo_mi355x_launch_decompress_seg
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p] * 10 + [ctypes.c_uint32, ctypes.c_void_p]
        one[kind] = f


def run(kind, src, zb, zl, nb, reps):
    variant(kind)
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
    ts = []
    for _ in range(reps):
        head.zero_()
        ring.zero_()
        out.zero_()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(s)
        if kind == "fast":
            rc = fast(p(zb.arena), p(zb.off), p(zl), p(out), p(src.off), p(src.length), p(ol), p(st),
                      p(head), p(ids), p(head[64:]), p(ring), p(ops), nsets, nb, s.cuda_stream)
        else:
            rc = one[kind](p(zb.arena), p(zb.off), p(zl), p(out), p(src.off), p(src.length), p(ol), p(st),
                           p(head), p(ids), nb, s.cuda_stream)
        ev1.record(s)
        assert rc == 0
        torch.cuda.synchronize()
        ts.append(ev0.elapsed_time(ev1))
    nfb = int(head[0].item())
    okb = bool(torch.equal(out, src.arena)) if nfb == 0 else False
    bad_st = int((st != 0).sum().item())
    return min(ts), sorted(ts)[len(ts) // 2], nfb, okb, bad_st


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    kinds = sys.argv[2:] or ["fast", "seg"]
    cases = [
        ("C2 4096x64KiB", [65536] * 4096, 0),
        ("C4-like 8192 mixed", list(synth.mixed_sizes(8192, 5)), 1),
        ("C5-like 1024 ITB", [11904 + 512 * int(k) for k in np.random.default_rng(3).integers(1, 1025, 1024)], 2),
        ("lone 64KiB", [65536], 3),
        ("lone 536192", [536192], 4),
    ]
    for name, sizes, seed in cases:
        src, zb, zl, nb = setup(sizes, seed)
        n = float(sum(int(x) for x in sizes))
        zsum = float(zl.sum().item())
        for k in kinds:
            tmin, tmed, nfb, okb, bad = run(k, src, zb, zl, nb, reps)
            print(f"{name:22s} {k:5s} min {tmin:8.4f} ms  med {tmed:8.4f} ms  {n / tmin / 1e6 / 1.073741824:8.1f} GiB/s"
                  f"  frac {(n + zsum) / (tmin * 1e-3) / 8e12:.4f}  fallbacks {nfb}  exact {okb}  bad_status {bad}",
                  flush=True)


if __name__ == "__main__" and not os.environ.get("SEG_STAMPS"):
    main()


def stamps():
    """Per-phase cycles per block (stamps build; read the shares, not the total)."""
    f = lib.lzo_mi355x_debug_decompress_seg_stamps
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p] * 10 + [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    names = ["stage+table", "walk", "decode", "far", "rows", "rare", "-", "-",
             "windows", "instrs", "rows", "subpasses", "farbatches", "rares", "rows_w_starts", "-"]
    for name, sizes, seed in (("lone 64KiB", [65536], 3), ("C2", [65536] * 4096, 0)):
        src, zb, zl, nb = setup(sizes, seed)
        out = torch.zeros_like(src.arena)
        ol = torch.zeros_like(zl)
        st = torch.zeros_like(zl)
        head = torch.zeros(64, dtype=torch.int32, device=dev)
        ids = torch.zeros(nb, dtype=torch.int32, device=dev)
        dbg = torch.zeros(nb * 16, dtype=torch.int64, device=dev)
        s = torch.cuda.current_stream()
        for _ in range(3):
            head.zero_()
            dbg.zero_()
            assert f(p(zb.arena), p(zb.off), p(zl), p(out), p(src.off), p(src.length), p(ol), p(st),
                     p(head), p(ids), nb, p(dbg), s.cuda_stream) == 0
            torch.cuda.synchronize()
        a = dbg.view(nb, 16).double().mean(0).cpu().numpy()
        tot = a[:6].sum()
        print(name, "cycles/block %.0f" % tot, " ".join(f"{names[i]}={a[i]:.0f}({a[i] / tot * 100:.0f}%)" for i in range(6)))
        print(name, "counts", " ".join(f"{names[i]}={a[i]:.1f}" for i in range(8, 15)), flush=True)


if __name__ == "__main__" and os.environ.get("SEG_STAMPS"):
    stamps()
