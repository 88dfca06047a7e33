"""Window counts of the encoder's parse (lzo1x_encode_fast.hip) under three
conflict tests, simulated on the CPU from the sequential LZO1X-1 parse of ITB
blocks: "current" cuts a window at the first path lane
sharing either of its two slots with an earlier path lane (the old claim
bitmap); "precise" only where an earlier path lane writes a slot the lane
reads; "none" ignores conflicts (the floor).  Usage: python scripts/enc_window_sim.py"""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pomegranate_amd import synth
K = 16384
def prim(b, p):
    v = ((((b[p+3] << 6) ^ b[p+2]) << 5) ^ b[p+1]); v = (v << 5) ^ b[p]
    return ((v * 33) >> 5) & (K - 1)
def sec(h): return (h & 0x7FF) ^ 0x201F
def ref_parse(b):
    n = len(b); d = [0] * K; ip = 4; ip_end = n - 13; rec = {}
    while True:
        h1 = prim(b, ip); slot = h1; c = d[h1]; ok = False; h2r = False
        if c and ip - (c - 1) <= 0xBFFF:
            cc = c - 1
            if ip - cc <= 0x800 or b[cc+3] == b[ip+3]: ok = True
            else:
                slot = sec(h1); h2r = True; c = d[slot]
                if c and ip - (c - 1) <= 0xBFFF:
                    cc = c - 1
                    if ip - cc <= 0x800 or b[cc+3] == b[ip+3]: ok = True
        if ok and not (b[cc] == b[ip] and b[cc+1] == b[ip+1] and b[cc+2] == b[ip+2]): ok = False
        d[slot] = ip + 1
        L = 0
        if ok:
            L = 3
            while ip + L < n and b[cc+L] == b[ip+L]: L += 1
        rec[ip] = (h1, sec(h1), h2r, slot, L)
        if not ok:
            ip += 1
            if ip >= ip_end: break
            continue
        ip += L
        if ip >= ip_end: break
    return rec, ip_end
def windows(rec, ip_end, mode):
    ip = 4; nw = 0; pathit = 0
    while ip < ip_end:
        nw += 1
        lanes = []; q = ip
        while q < ip + 64 and q < ip_end and q in rec:
            lanes.append(q); L = rec[q][4]; q += L if L else 1
        end = q   # where the path leaves the window
        cut = None
        writes = {}; touched = set()
        for i, q in enumerate(lanes):
            h1, h2, h2r, w, L = rec[q]
            if mode == "none":
                break
            if mode == "current":
                s = {h1, h2}
                if s & touched: cut = q; break
                touched |= s
            else:
                reads = {h1, h2} if h2r else {h1}
                if reads & touched: cut = q; break
                touched.add(w)
        if cut is not None:
            if cut == ip:
                cut = lanes[1] if len(lanes) > 1 else end
            end = min(end, cut)
        pathit += len(lanes)
        ip = end
    return nw
blocks = []
a, offs, lens = synth.batch(synth.ITB, 0, [65536] * 4)
for i in range(4):
    b = a[int(offs[i]): int(offs[i]) + 65536].tobytes()
    rec, ip_end = ref_parse(b)
    print(i, "probes", len(rec), {m: windows(rec, ip_end, m) for m in ("current", "precise", "none")})
