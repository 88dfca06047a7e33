"""Lone-block compress latency on one GPU: the LDS-dictionary encoder
(compress_dev without scratch, what single calls launch) against the
global-dictionary one; kernel time by HIP events, outputs compared between
the kernels.  (A lone-block encoder with an LDS input ring measured slower
than the LDS-dictionary one: scripts/experiments/encode_ring.patch)  Cases: one 12,416 / 65,536 /
536,192 B ITB record, and 256 C5-like records (12-536 KB) in one launch.

    python scripts/enc_lone.py [reps]"""
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


def case(sizes, reps):
    arena, offs, lens = synth.batch(synth.ITB, 11, sizes, align=256, threads=8)
    src = lzo.DeviceBatch(t(arena), t(offs.view(np.int64)), t(lens.view(np.int32)))
    caps = np.array([lzo.worst_compress(int(n)) for n in sizes], dtype=np.uint32)
    zo = np.zeros(len(sizes), dtype=np.uint64)
    zo[1:] = np.cumsum((caps[:-1].astype(np.uint64) + 255) // 256 * 256)
    za = torch.zeros(int(zo[-1]) + int(caps[-1]) + 256, dtype=torch.uint8, device=dev)
    zb = lzo.DeviceBatch(za, t(zo.view(np.int64)), t(caps.view(np.int32)))
    res, outs = {}, {}
    for name, dbg, scr in (("lds", "", None), ("gdict1", "", "auto")):
        os.environ["POM_LZO_DEBUG"] = dbg
        zl = torch.zeros(len(sizes), dtype=torch.int32, device=dev)
        zs = torch.full_like(zl, 99)
        ts = []
        for _ in range(reps):
            za.zero_()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            lzo.compress_dev(src, zb, zl, zs, scratch=scr)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        assert int((zs != 0).sum().item()) == 0, name
        outs[name] = (za.cpu().numpy().tobytes(), zl.cpu().numpy().tolist())
        res[name] = (round(min(ts), 1), round(float(np.median(ts)), 1))
    os.environ["POM_LZO_DEBUG"] = ""
    same = all(outs[k] == outs["lds"] for k in outs)
    return res, same


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    rng = np.random.default_rng(3)
    for name, sizes in (("12416", [12416]), ("65536", [65536]), ("536192", [536192]),
                        ("256 C5-like", [11904 + 512 * int(k) for k in rng.integers(1, 1025, 256)])):
        res, same = case(sizes, reps)
        print(f"{name:12s} compress us (min, median): {res}  outputs identical: {same}", flush=True)


if __name__ == "__main__":
    main()
