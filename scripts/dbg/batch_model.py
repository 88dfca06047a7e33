"""Model of the throughput decoder's executor scheduling on real LZO1X op
lists (CPU, no GPU): steps per 64 KiB ITB block under
  cur   -- the kernel's rule: op-level source forwarding (3 Jacobi rounds),
           a batch ends at the first op reading output at/after the batch start;
  chunk -- the same forwarding, but a STEP ends at the first 16-byte chunk
           whose source reaches into the step (batches no longer matter);
  cfwd  -- chunk rule plus chunk-level forwarding (a chunk whose source lies
           inside one earlier op of the window reads that op's source).
Usage: python scripts/dbg/batch_model.py [nblocks]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pomegranate_amd import synth
from lzo_ops import parse
import conftest

LIT = 1 << 31


def windows(ops):
    for w in range(0, len(ops), 64):
        yield ops[w:w + 64]


def prep(win):
    """per op: o, L, db (LIT flag for input), dp (period)"""
    out = []
    for kind, o, L, a in win:
        if kind == 'L':
            out.append([o, L, LIT | a, 0])
        else:
            out.append([o, L, o - a, a if a < L else 0])
    return out


def forward(w, rounds=3):
    o_first = w[0][0]
    for _ in range(rounds):
        new = [r[2] for r in w]
        anyneed = False
        for l, (o, L, db, dp) in enumerate(w):
            span = dp if dp else L
            if db & LIT or db + span <= o_first:
                continue
            anyneed = True
            k2 = max((i for i in range(len(w)) if w[i][0] <= db), default=0)
            ko, kL, kb, kp = w[k2]
            ok = k2 < l and ko <= db and db + span <= ko + kL
            r = db - ko
            if ok and kp:
                r %= kp
                ok = r + span <= kp
            if ok:
                new[l] = kb + r
        for l in range(len(w)):
            w[l][2] = new[l]
        if not anyneed:
            break
    return w


def chunks(w):
    """(x, len, src_end or None) per 16-byte chunk"""
    out = []
    for o, L, db, dp in w:
        for k in range(0, L, 16):
            n = min(16, L - k)
            if db & LIT:
                end = None
            elif dp:
                end = db + dp
            else:
                end = db + k + n
            out.append((o + k, n, end, (o, L, db, dp, k)))
    return out


def steps_cur(w):
    steps = 0
    s = 0
    n = len(w)
    while s < n:
        os_ = w[s][0]
        e = n
        for l in range(s + 1, n):
            o, L, db, dp = w[l]
            span = dp if dp else L
            if not (db & LIT) and db + span > os_:
                e = l
                break
        nch = sum((w[j][1] + 15) // 16 for j in range(s, e))
        steps += max(1, -(-nch // 64))
        s = e
    return steps


def steps_chunk(cs):
    steps = 0
    i = 0
    while i < len(cs):
        xs = cs[i][0]
        j = i + 1
        while j < len(cs) and j - i < 64:
            end = cs[j][2]
            if end is not None and end > xs:
                break
            j += 1
        steps += 1
        i = j
    return steps


def chunk_forward(w, cs):
    """chunk source -> inside one earlier op of the window: that op's source"""
    out = []
    for x, n, end, (o, L, db, dp, k) in cs:
        if end is None or dp:
            out.append((x, n, end))
            continue
        a = db + k
        for _ in range(8):
            hit = None
            for (o2, L2, db2, dp2) in w:
                if o2 <= a and a + n <= o2 + L2 and o2 < x:
                    hit = (o2, L2, db2, dp2)
                    break
            if hit is None:
                break
            o2, L2, db2, dp2 = hit
            if db2 & LIT:
                a = None
                break
            r = a - o2
            if dp2:
                r %= dp2
                if r + n > dp2:
                    break
            a = db2 + r
        out.append((x, n, None if a is None else a + n))
    return out


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    orc = conftest.Oracle()
    tot = {"cur": 0, "chunk": 0, "cfwd": 0, "ops": 0, "win": 0}
    for b in range(nb):
        d = synth.block(synth.ITB, b, 65536)
        ops, n = parse(orc.compress(d))
        assert n == 65536
        tot["ops"] += len(ops)
        for win in windows(ops):
            w = forward(prep(win))
            tot["win"] += 1
            tot["cur"] += steps_cur(w)
            cs = chunks(w)
            tot["chunk"] += steps_chunk(cs)
            cf = chunk_forward(w, cs)
            tot["cfwd"] += steps_chunk([(x, n, e, None) for x, n, e in cf])
    print({k: round(v / nb, 1) for k, v in tot.items()}, "(per block)")


if __name__ == "__main__":
    main()
