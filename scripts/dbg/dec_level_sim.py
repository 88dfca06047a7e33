"""CPU study for the op-set decoder (lzo1x_decode_fast.hip): executor steps per
64 KiB ITB block under the shipped batch rule (a batch ends at the first op
whose source reaches the batch's own output) against a level schedule (an op
runs one step after the ops its source bytes come from; each level's chunks
fill steps of 64).  Ops come from a plain LZO1X parse of the oracle's
compressed blocks (lib/minilzo.c:3367-3668 grammar), windows of 64 ops, the
kernel's three source-forwarding rounds applied first.
Usage: python scripts/dbg/dec_level_sim.py [--blocks N]"""
import argparse, ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from pomegranate_amd import synth

ap = argparse.ArgumentParser()
ap.add_argument("--blocks", type=int, default=8)
ap.add_argument("--bytes", type=int, default=65536)
a = ap.parse_args()

lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
lib.oracle_lzo1x_1_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                        ctypes.POINTER(ctypes.c_size_t)]


def compress(data):
    src = ctypes.create_string_buffer(data, len(data))
    out = ctypes.create_string_buffer(len(data) + len(data) // 16 + 67)
    ol = ctypes.c_size_t(0)
    lib.oracle_lzo1x_1_compress(src, len(data), out, ctypes.byref(ol))
    return out.raw[: ol.value]


def ops_of(z):
    """[(o, L, dist)] in output order; dist 0 = literals."""
    ops, ip, o = [], 0, 0

    def ext(t, base):
        nonlocal ip
        if t:
            return t
        n = 0
        while z[ip] == 0:
            n += 255
            ip += 1
        n += base + z[ip]
        ip += 1
        return n

    def lit(n):
        nonlocal ip, o
        ops.append((o, n, 0))
        ip += n
        o += n

    def match(L, d):
        nonlocal o
        ops.append((o, L, d))
        o += L

    state = "top"
    t = z[ip]
    if t > 17:
        ip += 1
        lit(t - 17)
        state = "after_first" if t - 17 >= 4 else "trail"
    while True:
        t = z[ip]; ip += 1
        if state == "top" and t < 16:
            lit(ext(t, 15) + 3)
            state = "after_first"
            continue
        if t < 16:
            if state == "after_first":       # 3-byte M1, dist > M2_MAX_OFFSET
                d = 1 + 0x0800 + (t >> 2) + (z[ip] << 2); ip += 1
                match(3, d)
            else:                            # 2-byte M1 after trailing literals
                d = 1 + (t >> 2) + (z[ip] << 2); ip += 1
                match(2, d)
        elif t >= 64:
            d = 1 + ((t >> 2) & 7) + (z[ip] << 3); ip += 1
            match((t >> 5) + 1, d)
        elif t >= 32:
            L = ext(t & 31, 31) + 2
            d = 1 + ((z[ip] | (z[ip + 1] << 8)) >> 2); ip += 2
            match(L, d)
        else:
            hi = (t & 8) << 11
            L = ext(t & 7, 7) + 2
            d = hi + ((z[ip] | (z[ip + 1] << 8)) >> 2); ip += 2
            if d == 0:
                break                        # EOF
            match(L, d + 0x4000)
        tr = z[ip - 2] & 3
        if tr:
            lit(tr)
            state = "trail"
        else:
            state = "top"
    return ops


def window_steps(w):
    n = len(w)
    o = [x[0] for x in w]
    L = [x[1] for x in w]
    lin = [x[2] == 0 for x in w]
    db = [0 if lin[i] else o[i] - w[i][2] for i in range(n)]
    dp = [0 if lin[i] or w[i][2] >= L[i] else w[i][2] for i in range(n)]
    o_first = o[0]
    for _ in range(3):                       # source forwarding (the kernel's rounds)
        nd = list(db); nl = list(lin)
        for i in range(n):
            if lin[i]:
                continue
            span = dp[i] or L[i]
            if db[i] + span <= o_first:
                continue
            k = max((j for j in range(n) if o[j] <= db[i]), default=-1)
            if k < 0 or k >= i:
                continue
            r = db[i] - o[k]
            if dp[k]:
                r %= dp[k]
            if db[i] + span <= o[k] + L[k] and (not dp[k] or r + span <= dp[k]):
                nd[i] = db[k] + r                # (k's source; k's linear flag)
                nl[i] = lin[k]
        db, lin = nd, nl
    chunks = [(x + 15) // 16 for x in L]
    send = [0 if lin[i] else db[i] + (dp[i] or L[i]) for i in range(n)]
    # batches
    steps_b, s = 0, 0
    while s < n:
        e = next((i for i in range(s + 1, n) if not lin[i] and send[i] > o[s]), n)
        steps_b += -(-sum(chunks[s:e]) // 64)
        s = e
    # levels
    lev = [0] * n
    for i in range(n):
        if lin[i] or send[i] <= o_first:
            continue
        lo, hi = db[i], send[i]
        lev[i] = 1 + max((lev[j] for j in range(i) if o[j] < hi and o[j] + L[j] > lo), default=-1)
    per = {}
    for i in range(n):
        per[lev[i]] = per.get(lev[i], 0) + chunks[i]
    steps_l = sum(-(-c // 64) for c in per.values())
    return steps_b, steps_l, max(lev) + 1


tb = tl = tw = tlev = 0
for b in range(a.blocks):
    data = synth.block(synth.ITB, 4242 + b, a.bytes)
    ops = ops_of(compress(data))
    assert sum(x[1] for x in ops) == len(data)
    for w0 in range(0, len(ops), 64):
        sb, sl, nl = window_steps(ops[w0: w0 + 64])
        tb += sb; tl += sl; tw += 1; tlev += nl
print(f"{a.blocks} blocks, {tw / a.blocks:.1f} windows/block: steps per block batches {tb / a.blocks:.1f}, "
      f"levels {tl / a.blocks:.1f} (levels per window {tlev / tw:.2f})")
