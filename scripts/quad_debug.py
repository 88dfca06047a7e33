"""Quarter-wave decoder (lzo1x_decode_quad.hip) alone on small block sets,
one set per line: blocks handed over, blocks with wrong bytes (first
differing offset, produced length), kernel time.  GPU box.

    python scripts/quad_debug.py [kind]      (kind: quad, seg, win; default quad)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import gpu_util as gu  # noqa: E402
import lzo_streams  # noqa: E402
from pomegranate_amd import synth  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
kind = sys.argv[1] if len(sys.argv) > 1 else "quad"


def run(name, blocks=None, streams=None):
    if streams is None:
        comps, st = gu.gpu_compress(torch, blocks, dev)
        assert all(s == 0 for s in st)
        want = blocks
    else:
        comps = [z for z, _ in streams]
        want = [o for _, o in streams]
    t0 = time.perf_counter()
    outs, st2, handed = gu.gpu_decompress_win(torch, comps, [len(w) for w in want], dev, kind)
    dt = time.perf_counter() - t0
    bad = []
    for i, (o, w) in enumerate(zip(outs, want)):
        if i in handed:
            continue
        if o != w or st2[i] != 0:
            k = next((x for x in range(min(len(o), len(w))) if o[x] != w[x]), min(len(o), len(w)))
            bad.append((i, len(w), len(o), st2[i], k))
    print(f"{name:28s} n={len(want):4d} handed={handed[:12]}{'...' if len(handed) > 12 else ''} "
          f"bad={bad[:6]}{'...' if len(bad) > 6 else ''} {dt * 1e3:.1f} ms", flush=True)


run("one ITB 64K", [synth.block(synth.ITB, 1, 65536)])
run("four ITB 64K", [synth.block(synth.ITB, 2 + i, 65536) for i in range(4)])
run("tiny", [b"", b"a", b"ab" * 7, bytes(14), b"abcdefghijklmnopqrstuvwxyz" * 3])
for m in range(6):
    run(f"model {m} 1..300K", [synth.block(m, 100 + m * 10 + i, n) for i, n in
                               enumerate((1, 13, 14, 100, 4096, 65536, 300000))])
run("ITB sizes", [synth.block(synth.ITB, 200 + i, n) for i, n in
                  enumerate((4096, 12416, 65536, 100000, 262144, 536192))])
run("full grammar", streams=[lzo_streams.stream(1000 + s, [50, 300, 5000, 40000, 150000][s % 5])
                             for s in range(40)])
run("LZ-like 1 MiB", [synth.block(synth.LZLIKE, 77, 1 << 20)])
run("C2 4096 x 64K", [synth.block(synth.ITB, 3000 + i, 65536) for i in range(4096)])
