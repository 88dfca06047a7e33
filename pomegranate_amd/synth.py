"""Deterministic synthetic blocks (libpom_synth.so), identical here and on the GPU box.

Models follow SURVEY.md section 8(d) and Appendix B: RANDOM for config C1,
ITB (ITB payload images, include/xtable.h:136-144) for C2-C5, plus extra
content models used only for parity breadth.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence, Tuple

import numpy as np

RANDOM, ITB, ZEROS, ALPHA4, LZLIKE, TEXT = range(6)
MODEL_NAMES = {RANDOM: "random", ITB: "itb", ZEROS: "zeros", ALPHA4: "alpha4",
               LZLIKE: "lzlike", TEXT: "text"}

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def _load():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "libpom_synth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build()")
        lib = ctypes.CDLL(path)
        lib.pom_synth_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p,
                                       ctypes.c_size_t]
        lib.pom_synth_batch.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_size_t,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int]
        lib.pom_synth_batch_seeds.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p,
                                              ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_int]
        _lib = lib
    return _lib


def block(model: int, seed: int, n: int) -> bytes:
    buf = ctypes.create_string_buffer(max(n, 1))
    _load().pom_synth_fill(model, seed, buf, n)
    return buf.raw[:n]


def batch(model: int, seed0: int, sizes: Sequence[int], align: int = 16,
          threads: int = 8, seeds: Optional[Sequence[int]] = None
          ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Blocks b = 0..len(sizes)-1 (seed seed0 + b, or seeds[b]) packed into one
    arena.  Returns (arena uint8, offsets uint64, sizes uint32)."""
    sizes = np.asarray(sizes, dtype=np.uint64)
    padded = (sizes + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    offsets = np.zeros(len(sizes), dtype=np.uint64)
    if len(sizes) > 1:
        offsets[1:] = np.cumsum(padded[:-1])
    total = int(padded.sum()) if len(sizes) else 0
    arena = np.zeros(max(total, 1), dtype=np.uint8)
    if len(sizes):
        sd = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint64)
        _load().pom_synth_batch_seeds(model, seed0, None if sd is None else sd.ctypes.data,
                                      len(sizes), offsets.ctypes.data, sizes.ctypes.data,
                                      arena.ctypes.data, threads)
    return arena, offsets, sizes.astype(np.uint32)


def mixed_sizes(count: int, seed: int, lo_kib: int = 4, hi_kib: int = 256,
                step_kib: int = 4) -> np.ndarray:
    """Config C4 block sizes: uniform over {lo, lo+step, ..., hi} KiB."""
    rng = np.random.default_rng(seed)
    k = rng.integers(lo_kib // step_kib, hi_kib // step_kib + 1, size=count)
    return (k * step_kib * 1024).astype(np.uint64)
