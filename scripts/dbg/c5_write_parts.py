"""Where C5's write time goes: compress batch, AppendFile open, append_batch,
close (GPU box).  Usage: python scripts/dbg/c5_write_parts.py"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np
import torch  # noqa: F401  (HIP runtime first)
from pomegranate_amd import itb, lzo
if len(sys.argv) > 1:
    lzo.LIB_PATH = sys.argv[1]
rng = np.random.default_rng(5)
ites = rng.integers(1, 1025, 1024)
recs = [itb.make_record(100000 + i, int(k)) for i, k in enumerate(ites)]
tmps = [bytearray(itb.ITB_FULL) for _ in recs]
itb.compress_batch(recs[:4], tmps[:4])
path = "/dev/shm/pom_c5_parts.itb"
for rep in range(4):
    t0 = time.perf_counter()
    which, err = itb.compress_batch(recs, tmps)
    t1 = time.perf_counter()
    af = itb.AppendFile(path)
    t2 = time.perf_counter()
    outs = [t if w else r for r, t, w in zip(recs, tmps, which)]
    lens = [itb.header_fields(o)[0] for o in outs]
    t3 = time.perf_counter()
    locs = af.append_batch(outs, lens)
    t4 = time.perf_counter()
    af.close()
    t5 = time.perf_counter()
    if rep == 0:
        import hashlib
        print("file sha256", hashlib.sha256(open(path, "rb").read()).hexdigest()[:16], locs[-1])
    os.unlink(path)
    print(f"compress {1e3*(t1-t0):.2f} open {1e3*(t2-t1):.2f} lists {1e3*(t3-t2):.2f} "
          f"append {1e3*(t4-t3):.2f} close {1e3*(t5-t4):.2f} ms; appended {sum(lens)/1e6:.1f} MB")
