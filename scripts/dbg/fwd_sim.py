"""CPU study: of the encoder's forwarding conflicts (a path lane
reading a slot an earlier path lane of its 64-position window writes), how many
leave the lane's decision (match or literal, and length) unchanged once the
lane sees the earlier write.  Usage: python scripts/dbg/fwd_sim.py"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pomegranate_amd import synth
K = 16384
def prim(b, p):
    v = ((((b[p+3] << 6) ^ b[p+2]) << 5) ^ b[p+1]); v = (v << 5) ^ b[p]
    return ((v * 33) >> 5) & (K - 1)
def sec(h): return (h & 0x7FF) ^ 0x201F
def decide(b, d, ip, n):
    h1 = prim(b, ip); slot = h1; c = d[h1]; ok = False; h2r = False; cc = 0
    if c and ip - (c - 1) <= 0xBFFF:
        cc = c - 1
        if ip - cc <= 0x800 or b[cc+3] == b[ip+3]: ok = True
        else:
            slot = sec(h1); h2r = True; c = d[slot]
            if c and ip - (c - 1) <= 0xBFFF:
                cc = c - 1
                if ip - cc <= 0x800 or b[cc+3] == b[ip+3]: ok = True
    if ok and not (b[cc] == b[ip] and b[cc+1] == b[ip+1] and b[cc+2] == b[ip+2]): ok = False
    L = 0
    if ok:
        L = 3
        while ip + L < n and b[cc+L] == b[ip+L]: L += 1
    return h1, sec(h1), h2r, slot, ok, L
def run(b):
    n = len(b); d = [0] * K; ip = 4; ip_end = n - 13
    same = diff = same_slot = windows = 0
    while ip < ip_end:
        windows += 1
        snap = list(d)
        q = ip; written = {}; nm = 0
        while q < ip + 64 and q < ip_end:
            h1, h2, h2r, slot, ok, L = decide(b, d, q, n)
            reads = {h1, h2} if h2r else {h1}
            if reads & set(written):
                s = decide(b, snap, q, n)
                if (s[4], s[5] if s[4] else 0) == (ok, L if ok else 0):
                    same += 1
                    same_slot += s[3] == slot
                else:
                    diff += 1
            d[slot] = q + 1
            written[slot] = q
            if ok:
                q += L; nm += 1
                if nm >= 6: break
            else:
                q += 1
        ip = q
    return windows, same, same_slot, diff
a, offs, lens = synth.batch(synth.ITB, 0, [65536] * 3)
for i in range(3):
    b = a[int(offs[i]): int(offs[i]) + 65536].tobytes()
    print(i, "windows, conflicts same (same slot), changed:", run(b))
