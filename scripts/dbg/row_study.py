"""Design study for a row decoder: ITB blocks of 64 KiB, output in
rows of 256 B.  Per row: the longest chain of in-row source hops (periodic
matches reduced to their last period), the share of bytes whose source lies
further back than a 4 KiB or 8 KiB LDS ring would hold, and instruction starts
per row.  CPU only; the oracle compresses.  Usage: python scripts/dbg/row_study.py"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "scripts", "dbg"))
sys.path.insert(0, ROOT)
import numpy as np
from dep_model import compress, origins, jacobi_rounds
from lzo_ops import parse
from pomegranate_amd import synth
H = {}
far4 = far8 = rows4 = rows8 = nrows = 0
segs_per_row = []
for b in range(6):
    data = synth.block(synth.ITB, 1000 + b, 65536)
    ops, n = parse(compress(data))
    src, kind, opid = origins(ops, n)
    hops = np.array(jacobi_rounds(src, 256)) - 1
    for h in hops: H[h] = H.get(h, 0) + 1
    pos = np.arange(n)
    m = src >= 0
    dist = np.where(m, pos - src, 0)
    for S in range(0, n, 256):
        sl = slice(S, S + 256)
        f4 = (m[sl] & (src[sl] < S + 256 - 3840)).sum(); f8 = (m[sl] & (src[sl] < S + 256 - 7936)).sum()
        far4 += f4; far8 += f8; rows4 += f4 > 0; rows8 += f8 > 0; nrows += 1
    # segments per row
    st = np.zeros(n, bool)
    for o in ops: st[o[1]] = True
    segs_per_row += [int(st[S:S+256].sum()) for S in range(0, n, 256)]
print("in-row hops per row (max over bytes):", sorted(H.items()))
print(f"far bytes ring4K {far4/(6*65536):.3f} rows {rows4/nrows:.3f}; ring8K {far8/(6*65536):.3f} rows {rows8/nrows:.3f}")
print("segments(op starts) per row pct 50/90/99/max:", np.percentile(segs_per_row, [50, 90, 99, 100]))
