"""Host-batch planner of liblzo_mi355x.so (pomegranate_amd/csrc/batch_split.c)
on the CPU: the device split (rank r of the largest-first order goes to
device r mod G), the chunking under a staging budget, and the reassembly of
every block's output at its own destination, at mock device counts G = 1, 2,
4 and 8 (tests/native/split_mock.c stands in for each GPU's work).  The
reference codes one ITB per call (mds/txg.c:700-770); the batch result must
not depend on how it was split."""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "native", "libsplit_mock.so")


@pytest.fixture(scope="module")
def mock():
    if not os.path.exists(LIB):
        import subprocess
        subprocess.run(["make", "-C", os.path.dirname(LIB)], check=True)
    lib = ctypes.CDLL(LIB)
    lib.mock_batch.restype = ctypes.c_int
    lib.mock_batch.argtypes = [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.POINTER(ctypes.c_int)]
    return lib


def run(mock, blocks, g, min_dev, budget, max_blocks=1 << 20):
    n = len(blocks)
    srcs = [ctypes.create_string_buffer(b, max(len(b), 1)) for b in blocks]
    dsts = [ctypes.create_string_buffer(max(len(b), 1)) for b in blocks]
    sp = (ctypes.c_void_p * max(n, 1))(*[ctypes.addressof(s) for s in srcs])
    dp = (ctypes.c_void_p * max(n, 1))(*[ctypes.addressof(d) for d in dsts])
    ln = (ctypes.c_size_t * max(n, 1))(*[len(b) for b in blocks])
    dev = np.full(max(n, 1), -1, np.int32)
    chunk = np.full(max(n, 1), -1, np.int64)
    seq = np.full(max(n, 1), -1, np.int64)
    used = ctypes.c_int(0)
    rc = mock.mock_batch(n, sp, ln, dp, g, min_dev, budget, max_blocks, dev.ctypes.data,
                         chunk.ctypes.data, seq.ctypes.data, ctypes.byref(used))
    assert rc == 0
    outs = [d.raw[: len(b)] for d, b in zip(dsts, blocks)]
    return outs, dev[:n], chunk[:n], seq[:n], used.value


def _blocks(seed, n, hi=300000):
    rng = np.random.default_rng(seed)
    sizes = rng.integers(0, hi, n)
    sizes[::17] = 0                                  # empty blocks ride along
    sizes[5::23] = 4096                              # ties in cost
    return [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]


@pytest.mark.parametrize("g", [1, 2, 4, 8])
def test_split_partition_and_reassembly(mock, g):
    blocks = _blocks(g, 300)
    budget = 3 << 20
    outs, dev, chunk, seq, used = run(mock, blocks, g, min_dev=1 << 20, budget=budget)
    total = sum(2 * len(b) for b in blocks)
    assert used == min(g, len(blocks), max(1, total // (1 << 20)))
    # every block handled once, its output at its own destination
    assert outs == [b[::-1] for b in blocks]
    assert (dev >= 0).all() and (seq >= 0).all()
    # rank r of the largest-first order (ties: lower id first) -> device r mod G
    order = sorted(range(len(blocks)), key=lambda b: (-len(blocks[b]), b))
    for r, b in enumerate(order):
        assert dev[b] == r % used
    # within a device: that order, cut into greedy chunks under the budget
    for d in range(used):
        mine = [b for b in order if dev[b] == d]
        assert [int(seq[b]) for b in mine] == list(range(len(mine)))
        cost = {}
        for b in mine:
            cost.setdefault(int(chunk[b]), []).append(2 * len(blocks[b]))
        assert sorted(cost) == list(range(len(cost)))
        for c, cs in cost.items():
            assert sum(cs) <= budget or len(cs) == 1
            if c + 1 in cost:                        # greedy: the next block did not fit
                assert sum(cs) + cost[c + 1][0] > budget


def test_split_small_batches_stay_on_one_device(mock):
    blocks = _blocks(9, 40, hi=20000)
    outs, dev, chunk, seq, used = run(mock, blocks, 8, min_dev=64 << 20, budget=256 << 20)
    assert used == 1 and (dev == 0).all() and (chunk == 0).all()
    assert outs == [b[::-1] for b in blocks]


def test_split_oversized_block_is_its_own_chunk(mock):
    blocks = [bytes(range(256)) * 40, b"x" * 100, b"y" * 5000, b""]
    outs, dev, chunk, seq, used = run(mock, blocks, 1, min_dev=1, budget=4096)
    assert outs == [b[::-1] for b in blocks]
    assert int(chunk[0]) == 0 and int(chunk[2]) == 1       # 20 KiB, then 10 KB each alone
    assert int(chunk[1]) == int(chunk[3]) == 2             # 200 B + 0 B fit together


def test_split_max_blocks_per_chunk(mock):
    blocks = [b"z" * 10] * 25
    outs, dev, chunk, seq, used = run(mock, blocks, 1, min_dev=1, budget=1 << 30, max_blocks=10)
    assert sorted(np.bincount(chunk)) == [5, 10, 10]


def test_split_empty_batch(mock):
    outs, dev, chunk, seq, used = run(mock, [], 4, min_dev=1, budget=1 << 20)
    assert outs == [] and used == 1


def test_split_concurrent_callers(mock):
    """Host batches from several threads at once (MDS commit threads) are
    independent: each gets its own plan and device threads."""
    errs = []

    def worker(seed):
        try:
            blocks = _blocks(100 + seed, 120, hi=50000)
            outs, dev, *_ = run(mock, blocks, 4, min_dev=1 << 18, budget=1 << 20)
            assert outs == [b[::-1] for b in blocks]
        except AssertionError as e:                  # pragma: no cover
            errs.append(e)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs


@pytest.mark.parametrize("spec,count,want", [
    ("0,0", 8, [0]),                      # duplicate: one helper thread per device
    ("1,0,1,2,0", 4, [1, 0, 2]),
    ("3,9,2", 4, [3, 2]),                 # out of range dropped
    ("", 4, []),
    ("2,,1", 4, [2]),                     # parsing stops at a malformed entry
])
def test_parse_devices_drops_duplicates(mock, spec, count, want):
    """POM_LZO_DEVICES (lzo_host.c batch_devices): a device listed twice must
    not get two helper threads sharing the caller's slots."""
    mock.mock_parse_devices.restype = ctypes.c_int
    mock.mock_parse_devices.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p]
    devs = (ctypes.c_int * 16)()
    n = mock.mock_parse_devices(spec.encode(), count, 16, devs)
    assert list(devs[:n]) == want


@pytest.mark.parametrize("step", [1, 3, 7, 100, 1 << 20])
def test_pwritev_resumes_short_writes(mock, step):
    """MDSL append file (itb_codec.c, mdsl/storage.c:455-519): a gathered
    write that the kernel cuts short, possibly twice inside one iovec, or
    interrupts with EINTR, must still land every byte once, in order."""
    rng = np.random.default_rng(step)
    lens = [0, 5, 17, 0, 1, 64, 3, 250]
    bufs = [ctypes.create_string_buffer(rng.integers(0, 256, n, dtype=np.uint8).tobytes(), max(n, 1))
            for n in lens]
    file = ctypes.create_string_buffer(sum(lens) + 40)
    mock.mock_pwritev_all.restype = ctypes.c_int
    mock.mock_pwritev_all.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_int, ctypes.c_size_t, ctypes.c_long]
    arr = (ctypes.c_void_p * len(bufs))(*[ctypes.cast(b, ctypes.c_void_p).value for b in bufs])
    ln = (ctypes.c_size_t * len(lens))(*lens)
    assert mock.mock_pwritev_all(file, arr, ln, len(lens), step, 40) == 0
    want = b"".join(b.raw[:n] for b, n in zip(bufs, lens))
    assert file.raw[40:40 + len(want)] == want
    assert file.raw[:40] == b"\0" * 40
