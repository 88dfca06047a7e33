"""Random valid LZO1X streams over the whole grammar the decoder accepts
(lib/minilzo.c:3308-3699), including forms the
LZO1X-1 compressor never writes: M1 matches after a literal run (3 bytes,
distance 0x801..0xC00) and after trailing literals (2 bytes, distance
1..1024), long-form length extensions, M4 distances above 0x8000, and
first instructions of 1-3 literals.  The generator knows the output, so a
stream checks a decoder by itself; tests/test_oracle.py pins it against the
oracle decoder.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


def _ext(out: bytearray, x: int) -> None:
    """x >= 1 as (x - 1) // 255 zero bytes, then the rest."""
    while x > 255:
        out.append(0)
        x -= 255
    out.append(x)


def stream(seed: int, n_target: int) -> Tuple[bytes, bytes]:
    """(compressed stream, decoded output) of about n_target output bytes."""
    rng = np.random.default_rng(seed)
    z = bytearray()
    out = bytearray()

    def lits(k: int) -> None:
        b = rng.integers(0, 256, k, dtype=np.uint8).tobytes()
        z.extend(b)
        out.extend(b)

    def copy(dist: int, length: int) -> None:
        for _ in range(length):
            out.append(out[-dist])

    def trailing() -> int:
        return int(rng.choice([0, 0, 1, 2, 3]))

    # first instruction: t > 17 is a literal run of t - 17 (1..238) bytes
    first = int(rng.integers(1, 239)) if rng.random() < 0.8 else int(rng.integers(1, 4))
    z.append(17 + first)
    lits(first)
    state = "C" if first < 4 else "B"
    while len(out) < n_target:
        r = rng.random()
        if state == "A" and r < 0.35:                     # literal run (4.. bytes)
            k = int(rng.choice([4, 5, 18, 19, 200, 300, 1000])) if rng.random() < 0.3 else int(rng.integers(4, 40))
            if k <= 18:
                z.append(k - 3)
            else:
                z.append(0)
                _ext(z, k - 18)
            lits(k)
            state = "B"
            continue
        t_lo = trailing()
        op = len(out)
        kind = rng.random()
        if state == "B" and kind < 0.25 and op >= 0xC00:  # M1 after a literal run: 3 bytes
            d = int(rng.integers(0x801, 0xC01))
            dd = d - 0x801
            z.append(((dd & 3) << 2) | t_lo)
            z.append(dd >> 2)
            copy(d, 3)
        elif state == "C" and kind < 0.25 and op >= 1:    # M1 after trailing literals: 2 bytes
            d = int(rng.integers(1, min(op, 1024) + 1))
            dd = d - 1
            z.append(((dd & 3) << 2) | t_lo)
            z.append(dd >> 2)
            copy(d, 2)
        elif kind < 0.5 and op >= 1:                      # M2: 3..8 bytes, distance <= 2048
            L = int(rng.integers(3, 9))
            d = int(rng.integers(1, min(op, 2048) + 1))
            dd = d - 1
            z.append(((L - 1) << 5) | ((dd & 7) << 2) | t_lo)
            z.append(dd >> 3)
            copy(d, L)
        elif kind < 0.8 and op >= 1:                      # M3: distance <= 16384
            L = int(rng.choice([3, 4, 33, 34, 300])) if rng.random() < 0.3 else int(rng.integers(3, 60))
            d = int(rng.integers(1, min(op, 16384) + 1))
            if L <= 33:
                z.append(32 | (L - 2))
            else:
                z.append(32)
                _ext(z, L - 33)
            v = ((d - 1) << 2) | t_lo
            z += bytes([v & 255, v >> 8])
            copy(d, L)
        elif op > 0x4000:                                 # M4: 0x4001..0xBFFF
            L = int(rng.choice([3, 9, 10, 500])) if rng.random() < 0.3 else int(rng.integers(3, 40))
            d = int(rng.integers(0x4001, min(op, 0xBFFF) + 1))
            dd = d - 0x4000
            hi = (dd & 0x4000) >> 11
            if L <= 9:
                z.append(16 | hi | (L - 2))
            else:
                z.append(16 | hi)
                _ext(z, L - 9)
            v = ((dd & 0x3FFF) << 2) | t_lo
            z += bytes([v & 255, v >> 8])
            copy(d, L)
        else:
            continue
        if t_lo:
            lits(t_lo)
            state = "C"
        else:
            state = "A"
    z += b"\x11\x00\x00"                                  # EOF: M4 with distance 0x4000
    return bytes(z), bytes(out)
