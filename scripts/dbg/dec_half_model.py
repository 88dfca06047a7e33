"""CPU model (round 6): executor steps and windows per 64 KiB ITB
block when a window holds W ops and a step C 16-byte chunks -- the kernel (64, 64)
against half-wave windows/steps (32, 32), the shape an executor wave running two
blocks side by side (32 lanes each) would have.  Same forwarding and batch rule as
scripts/dbg/batch_model.py (cur).  Usage: python scripts/dbg/dec_half_model.py"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import batch_model as bm
from batch_model import synth, parse, conftest, prep, forward, LIT

def steps_cap(w, cap):
    steps = 0; s = 0; n = len(w)
    while s < n:
        os_ = w[s][0]; e = n
        for l in range(s + 1, n):
            o, L, db, dp = w[l]; span = dp if dp else L
            if not (db & LIT) and db + span > os_:
                e = l; break
        nch = sum((w[j][1] + 15) // 16 for j in range(s, e))
        steps += max(1, -(-nch // cap)); s = e
    return steps

orc = conftest.Oracle(); nb = 32
for W, cap in ((64, 64), (32, 32), (64, 32), (32, 64)):
    tot = 0; nwin = 0
    for b in range(nb):
        d = synth.block(synth.ITB, b, 65536)
        ops, n = parse(orc.compress(d))
        for i in range(0, len(ops), W):
            w = forward(prep(ops[i:i + W])); nwin += 1
            tot += steps_cap(w, cap)
    print(f"window {W} ops, {cap} chunks/step: steps/block {tot/nb:.1f}, windows/block {nwin/nb:.1f}")
