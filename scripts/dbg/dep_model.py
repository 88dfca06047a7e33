"""CPU model of decode dependency structures on ITB streams (design study for the
round-3 decoder).  Compresses synthetic ITB blocks with the oracle, parses the op
stream and reports:
  - op statistics (count, literal/match bytes, distance/length histograms)
  - per-byte origin depth (how many match hops to a literal byte)
  - steps of fixed-size output windows: pointer-jump rounds needed when a byte's
    source inside the window is resolved by doubling
Usage: python scripts/dbg/dep_model.py [nblocks] [size]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts", "dbg"))
from pomegranate_amd import synth  # noqa: E402
from lzo_ops import parse  # noqa: E402

orc = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))


def compress(data):
    out = ctypes.create_string_buffer(len(data) + len(data) // 16 + 64 + 3)
    ol = ctypes.c_size_t(0)
    orc.oracle_lzo1x_1_compress(data, ctypes.c_size_t(len(data)), out, ctypes.byref(ol))
    return out.raw[: ol.value]


def origins(ops, n):
    """src[x]: -1-inpos for literal bytes, else the output position copied from
    (periodic matches reduced to before the op start)."""
    src = np.zeros(n, dtype=np.int64)
    kind = np.zeros(n, dtype=np.int8)
    opid = np.zeros(n, dtype=np.int32)
    for i, o in enumerate(ops):
        if o[0] == 'L':
            _, p, ln, s = o
            src[p:p + ln] = -1 - (s + np.arange(ln))
            kind[p:p + ln] = 0
        else:
            _, p, ln, d = o
            k = np.arange(ln)
            src[p:p + ln] = p - d + (k % d)
            kind[p:p + ln] = 1
        opid[o[1]:o[1] + o[2]] = i
    return src, kind, opid


def depth(src):
    n = len(src)
    dep = np.zeros(n, dtype=np.int32)
    for x in range(n):
        y = src[x]
        dep[x] = 0 if y < 0 else dep[y] + 1
    return dep


def window_rounds(src, W):
    """per window of W output bytes: doubling rounds until every byte's source is
    a literal or lies before the window."""
    n = len(src)
    rounds = []
    for S in range(0, n, W):
        E = min(n, S + W)
        t = src[S:E].copy()
        r = 0
        while True:
            pend = (t >= S)
            if not pend.any():
                break
            r += 1
            t2 = t.copy()
            idx = np.nonzero(pend)[0]
            t2[idx] = src_final(t, S, t[idx])
            t = t2
        rounds.append(r)
    return rounds


def src_final(t, S, y):
    return t[y - S]


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    tot = {}
    for b in range(nb):
        data = synth.block(synth.ITB, 1000 + b, size)
        z = compress(data)
        ops, n = parse(z)
        assert n == size
        src, kind, opid = origins(ops, n)
        lits = [o for o in ops if o[0] == 'L']
        ms = [o for o in ops if o[0] == 'M']
        dists = np.array([o[3] for o in ms])
        lens = np.array([o[2] for o in ms])
        dep = depth(src)
        print(f"block {b}: z={len(z)} ops={len(ops)} lit_ops={len(lits)} lit_bytes={sum(o[2] for o in lits)} "
              f"matches={len(ms)} match_bytes={lens.sum()}")
        print("  dist pct(10,50,90):", np.percentile(dists, [10, 50, 90]).astype(int).tolist(),
              " d<16:", int((dists < 16).sum()), " d==1:", int((dists == 1).sum()),
              " d>=1024:", int((dists >= 1024).sum()), " d>=4096:", int((dists >= 4096).sum()))
        print("  len pct(10,50,90):", np.percentile(lens, [10, 50, 90]).astype(int).tolist(),
              " periodic(d<len):", int((dists < lens).sum()))
        print("  byte depth max/mean:", int(dep.max()), round(float(dep.mean()), 1))
        for W in (256, 1024, 4096):
            r = window_rounds(src, W)
            print(f"  W={W}: windows={len(r)} rounds max={max(r)} mean={np.mean(r):.2f} sum={sum(r)}")


if __name__ == "__main__":
    main()


def jacobi_rounds(src, W):
    """per window: rounds of 'every byte copies its source' until fixed
    (byte chain length inside the window)."""
    n = len(src)
    out = []
    for S in range(0, n, W):
        E = min(n, S + W)
        d = np.zeros(E - S, dtype=np.int32)
        for x in range(S, E):
            y = src[x]
            d[x - S] = 1 if (y < 0 or y < S) else d[y - S] + 1
        out.append(int(d.max()))
    return out


def pieces_per_chunk(ops, n, W, C=16):
    starts = np.zeros(n + 1, dtype=np.int32)
    for o in ops:
        starts[o[1]] = 1
    res = []
    for S in range(0, n, W):
        mx = 0
        for c in range(S, min(n, S + W), C):
            k = 1 + int(starts[c + 1:min(n, c + C)].sum())
            mx = max(mx, k)
        res.append(mx)
    return res


def main2():
    size = 65536
    for b in range(2):
        data = synth.block(synth.ITB, 1000 + b, size)
        ops, n = parse(compress(data))
        src, kind, opid = origins(ops, n)
        for W in (512, 1024, 2048):
            j = jacobi_rounds(src, W)
            p = pieces_per_chunk(ops, n, W)
            print(f"b{b} W={W}: jacobi rounds mean={np.mean(j):.2f} max={max(j)} sum={sum(j)}; "
                  f"max pieces/chunk per window mean={np.mean(p):.2f} max={max(p)}")


def final_src_far(src, W, rings=(2048, 4096, 8192, 16384, 32768)):
    """after in-window doubling, bytes whose final source is an output byte
    before the window: how many are more than R bytes behind the window start."""
    n = len(src)
    cnt = {R: 0 for R in rings}
    nb = 0
    for S in range(0, n, W):
        E = min(n, S + W)
        t = src[S:E].copy()
        while True:
            pend = t >= S
            if not pend.any():
                break
            t[pend] = t[t[pend] - S]
        m = t >= 0
        nb += int(m.sum())
        for R in rings:
            cnt[R] += int((m & (t < S - R + W)).sum())
    return nb, cnt


def main3():
    size = 65536
    for b in range(2):
        data = synth.block(synth.ITB, 1000 + b, size)
        ops, n = parse(compress(data))
        src, kind, opid = origins(ops, n)
        for W in (256, 1024):
            nb, cnt = final_src_far(src, W)
            print(f"b{b} W={W}: match bytes={nb} beyond ring R: {cnt}")


def final_origin(src):
    n = len(src)
    org = np.zeros(n, dtype=np.int64)
    for x in range(n):
        y = src[x]
        org[x] = y if y < 0 else org[y]
    return org


def main4():
    size = 65536
    for b in range(2):
        data = synth.block(synth.ITB, 1000 + b, size)
        ops, n = parse(compress(data))
        src, kind, opid = origins(ops, n)
        org = final_origin(src)
        runs = 1 + int((org[1:] != org[:-1] - 1).sum())    # origins are -1-inpos: contiguous means decreasing
        same = int((org[1:] == org[:-1]).sum())
        # runs at 16-byte chunk granularity: chunks whose 16 origins are contiguous
        ch = org[: n // 16 * 16].reshape(-1, 16)
        contig = int((np.diff(ch, axis=1) == -1).all(axis=1).sum())
        const = int((np.diff(ch, axis=1) == 0).all(axis=1).sum())
        print(f"b{b}: final-origin runs={runs} (bytes equal to previous origin: {same}); "
              f"chunks contiguous={contig} constant={const} of {ch.shape[0]}")


def window_final(src, W):
    n = len(src)
    t_all = src.copy()
    for S in range(0, n, W):
        E = min(n, S + W)
        t = src[S:E].copy()
        while True:
            pend = t >= S
            if not pend.any():
                break
            t[pend] = t[t[pend] - S]
        t_all[S:E] = t
    return t_all


def classify(fin, lit_as_neg=True):
    n = len(fin) // 16 * 16
    ch = fin[:n].reshape(-1, 16)
    d = np.diff(ch, axis=1)
    lit = (ch < 0)
    # literal pointers are -1-inpos (contiguous = step -1); output pointers step +1
    contig = ((d == 1) & ~lit[:, 1:]).all(axis=1) | ((d == -1) & lit[:, 1:]).all(axis=1)
    const = (d == 0).all(axis=1)
    # "two runs": at most one break
    breaks = (~(((d == 1) & ~lit[:, 1:]) | ((d == -1) & lit[:, 1:]))).sum(axis=1)
    return int(contig.sum()), int(const.sum()), int((breaks == 1).sum()), int((breaks >= 2).sum()), ch.shape[0]


def main5():
    size = 65536
    for b in range(2):
        data = synth.block(synth.ITB, 1000 + b, size)
        ops, n = parse(compress(data))
        src, kind, opid = origins(ops, n)
        for W in (256, 1024, 4096):
            fin = window_final(src, W)
            c, k, one, many, tot = classify(fin)
            print(f"b{b} W={W}: chunks contiguous={c} constant={k} one-break={one} 2+breaks={many} of {tot}")
        c, k, one, many, tot = classify(src)
        print(f"b{b} initial src: contiguous={c} constant={k} one-break={one} 2+breaks={many}")


def row_rounds(src, W, R=64, reduce_periodic=True):
    n = len(src)
    tot_rows = 0
    rr = 0
    maxr = []
    for S in range(0, n, W):
        E = min(n, S + W)
        t = src[S:E].copy()
        r = 0
        while True:
            pend = t >= S
            if not pend.any():
                break
            r += 1
            rows = pend[: (E - S) // R * R].reshape(-1, R).any(axis=1)
            rr += int(rows.sum())
            t[pend] = t[t[pend] - S]
        tot_rows += (E - S) // R
        maxr.append(r)
    return tot_rows, rr, maxr


def origins_noreduce(ops, n):
    src = np.zeros(n, dtype=np.int64)
    for o in ops:
        if o[0] == 'L':
            _, p, ln, s = o
            src[p:p + ln] = -1 - (s + np.arange(ln))
        else:
            _, p, ln, d = o
            src[p:p + ln] = np.arange(p, p + ln) - d
    return src


def main6():
    size = 65536
    for b in range(2):
        data = synth.block(synth.ITB, 1000 + b, size)
        ops, n = parse(compress(data))
        src, kind, opid = origins(ops, n)
        src2 = origins_noreduce(ops, n)
        for W in (512, 1024, 2048, 4096):
            tr, rr, mx = row_rounds(src, W)
            tr2, rr2, mx2 = row_rounds(src2, W)
            print(f"b{b} W={W}: rows={tr} pending row-rounds reduced={rr} (max rounds {max(mx)}, sum {sum(mx)}) "
                  f"unreduced={rr2} (max {max(mx2)}, sum {sum(mx2)})")
