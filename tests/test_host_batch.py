"""Host-resident batches (lzo_mi355x_compress_batch / _decompress_batch) as
the chunked, two-stream pipeline of lzo_host.c: many chunks under a small
staging budget, the device split at G = 1 (the GPU box has one GPU; G = 2, 4,
8 are covered on the CPU by tests/test_split.py), and a batch of more than
8 GiB that runs through bounded staging.  Outputs are checked byte for byte
against the oracle or the original data."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

from pomegranate_amd import lzo, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture
def env(monkeypatch):
    return monkeypatch


def _ptrs(addrs):
    a = np.ascontiguousarray(np.asarray(addrs, dtype=np.uint64))
    return (ctypes.c_void_p * len(a)).from_buffer_copy(a.tobytes()), a


def _sizes(n):
    a = np.ascontiguousarray(np.asarray(n, dtype=np.uint64))
    return (ctypes.c_size_t * len(a)).from_buffer_copy(a.tobytes())


def test_many_chunks_match_oracle(oracle, env):
    """A 1 MiB chunk budget cuts 300 mixed blocks into dozens of chunks; every
    block's output is still the oracle's, at its own destination."""
    env.setenv("POM_LZO_DEBUG", "chunk_mb=1")
    lzo.debug_reload()
    env.setenv("POM_LZO_DEVICES", "0")
    rng = np.random.default_rng(4)
    sizes = [int(x) for x in rng.integers(0, 200000, 300)]
    sizes[7] = 3 << 20                                # larger than a chunk: a chunk of its own
    blocks = [synth.block(synth.ITB, 3000 + i, n) for i, n in enumerate(sizes)]
    rc, st, comps = lzo.compress_batch(blocks)
    assert rc == 0 and st == [0] * len(blocks)
    for i in range(0, len(blocks), 7):
        assert comps[i] == oracle.compress(blocks[i]), i
    rc, st, outs = lzo.decompress_batch(comps, [len(b) for b in blocks])
    assert rc == 0 and st == [0] * len(blocks)
    assert outs == blocks


def test_split_g1_is_bit_exact(env):
    """POM_LZO_DEVICES with one GPU and the default (every visible GPU) give
    the same bytes."""
    blocks = [synth.block(synth.ITB, 4000 + i, 65536 + 97 * i) for i in range(64)]
    env.setenv("POM_LZO_DEVICES", "0")
    a = lzo.compress_batch(blocks)
    env.delenv("POM_LZO_DEVICES")
    b = lzo.compress_batch(blocks)
    assert a == b and a[0] == 0


def test_host_batch_over_8_gib():
    """131,072 blocks of 64 KiB (8 GiB) compress and decompress through
    staging bounded by the chunk budget; the round trip is exact."""
    nb, bs = 131072, 65536
    base_n = 4096                                      # 256 MiB of distinct data
    arena, offs, lens = synth.batch(synth.ITB, 0, [bs] * base_n, threads=16)
    assert int(offs[1] - offs[0]) == bs
    base = arena.ctypes.data
    src_addr = base + (np.arange(nb, dtype=np.uint64) % base_n) * bs
    cap = lzo.worst_compress(bs)
    cstride = (cap + 15) // 16 * 16
    zarena = np.empty(nb * cstride, dtype=np.uint8)
    z_addr = zarena.ctypes.data + np.arange(nb, dtype=np.uint64) * cstride
    lib = lzo.load()
    sp, _ = _ptrs(src_addr)
    zp, _ = _ptrs(z_addr)
    slen = _sizes([bs] * nb)
    zlen = (ctypes.c_size_t * nb)()
    st = (ctypes.c_int * nb)()
    assert lib.lzo_mi355x_compress_batch(sp, slen, zp, zlen, st, nb) == 0
    stv = np.frombuffer(st, dtype=np.int32)
    zl = np.frombuffer(zlen, dtype=np.uint64).copy()
    assert (stv == 0).all()
    # blocks of equal content compress to equal bytes
    assert (zl[base_n: 2 * base_n] == zl[:base_n]).all()
    out = np.empty(nb * bs, dtype=np.uint8)
    o_addr = out.ctypes.data + np.arange(nb, dtype=np.uint64) * bs
    op, _ = _ptrs(o_addr)
    olen = _sizes([bs] * nb)
    st2 = (ctypes.c_int * nb)()
    assert lib.lzo_mi355x_decompress_batch(zp, _sizes(zl), op, olen, st2, nb) == 0
    assert (np.frombuffer(st2, dtype=np.int32) == 0).all()
    assert (np.frombuffer(olen, dtype=np.uint64) == bs).all()
    data = arena[: base_n * bs]
    view = out.reshape(nb // base_n, base_n * bs)
    for k in range(view.shape[0]):
        assert np.array_equal(view[k], data), k
