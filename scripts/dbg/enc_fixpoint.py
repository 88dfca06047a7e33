"""CPU study for a latency encoder: does the LZO1X-1 greedy parse
(lib/minilzo.c:2922-3157, restated in oracle/lzo1x_oracle.c parse_core) reach
its exact result by Jacobi iteration over all positions at once?

State of an iteration: the set V of visited positions and, for each, the
dictionary slot it wrote.  One iteration, every position in parallel: the
candidate at p is the last q < p in V that wrote p's slot (with the slots of
the previous iteration); p's decision (match and length, or literal) and the
slot it writes follow; the path from position 4 through those decisions is the
new V.  Prints, per block, the iterations until V and the slots stop changing
and whether the result equals the sequential parse.
Usage: python scripts/dbg/enc_fixpoint.py [nblocks] [size]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from pomegranate_amd import synth  # noqa: E402

SLOTS, FAR, NEAR, GUARD = 1 << 14, 0xBFFF, 0x0800, 13


def prim(a, p):
    v = ((((int(a[p + 3]) << 6) ^ int(a[p + 2])) << 5) ^ int(a[p + 1]))
    v = (v << 5) ^ int(a[p])
    return ((v * 33) >> 5) & (SLOTS - 1)


def decide(a, n, p, dct):
    """decision at p with dictionary dct (slot -> position + 1): (slot written, len)"""
    slot = prim(a, p)
    cand = dct[slot]
    ok = False
    c = 0
    if cand and p - (cand - 1) <= FAR:
        c = cand - 1
        if p - c <= NEAR or a[c + 3] == a[p + 3]:
            ok = True
        else:
            slot = (slot & 0x7FF) ^ 0x201F
            cand = dct[slot]
            if cand and p - (cand - 1) <= FAR:
                c = cand - 1
                if p - c <= NEAR or a[c + 3] == a[p + 3]:
                    ok = True
    if ok and not (a[c] == a[p] and a[c + 1] == a[p + 1] and a[c + 2] == a[p + 2]):
        ok = False
    if not ok:
        return slot, 0
    ln = 3
    while ln < 9 and a[c + ln] == a[p + ln]:
        ln += 1
    if ln == 9:
        while p + ln < n and a[c + ln] == a[p + ln]:
            ln += 1
    return slot, ln


def sequential(a, n):
    dct = [0] * SLOTS
    ip, end = 4, n - GUARD
    V = {}
    while True:
        slot, ln = decide(a, n, ip, dct)
        dct[slot] = ip + 1
        V[ip] = (slot, ln)
        ip += ln if ln else 1
        if ip >= end:
            return V


def jacobi(a, n, limit=60):
    end = n - GUARD
    # start: every position visited, writing its primary slot
    V = {p: (prim(a, p), 0) for p in range(4, end)}
    for it in range(1, limit + 1):
        dct = [0] * SLOTS
        dec = {}
        for p in range(4, end):
            dec[p] = decide(a, n, p, dct)
            if p in V:
                dct[V[p][0]] = p + 1         # the previous iteration's writer
        ip, W = 4, {}
        while ip < end:
            W[ip] = dec[ip]
            ip += dec[ip][1] if dec[ip][1] else 1
        if W == V:
            return it, W
        V = W
    return None, V


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    for b in range(nb):
        a = np.frombuffer(synth.block(synth.ITB, 500 + b, size), dtype=np.uint8)
        seq = sequential(a, size)
        it, V = jacobi(a, size)
        print(f"block {b} ({size} B): {len(seq)} visited positions; Jacobi iterations {it}; "
              f"exact {V == seq}", flush=True)


if __name__ == "__main__":
    main()
