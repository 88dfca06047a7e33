"""CPU: block sharding across GPUs and the completion barrier,
exercised with the gloo backend at world size 2 (the N>1 bench path uses the
same functions over RCCL)."""
from __future__ import annotations

import hashlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pomegranate_amd import shard, synth


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_round_robin_partitions_every_block_once(world):
    n = 1000
    seen = []
    for r in range(world):
        ids = shard.round_robin(n, r, world)
        assert all(i % world == r for i in ids)
        seen += ids
    assert sorted(seen) == list(range(n))


def test_round_robin_rejects_bad_rank():
    with pytest.raises(ValueError):
        shard.round_robin(10, 2, 2)


def test_per_rank_bytes_reports_mixed_size_imbalance():
    sizes = synth.mixed_sizes(4096, 4)
    per = shard.per_rank_bytes(sizes, 8)
    assert sum(per) == int(sizes.sum())
    assert max(per) / min(per) < 1.2          # round-robin of uniform sizes stays close


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(__file__)))
        from conftest import Oracle
        oracle = Oracle()
        nglobal = 64
        mine = shard.round_robin(nglobal, rank, world)
        arena, offs, lens = synth.batch(synth.ITB, 0, [16384] * len(mine), seeds=mine)
        h = hashlib.sha256()
        errors = 0
        for b in range(len(mine)):
            d = arena[int(offs[b]): int(offs[b]) + int(lens[b])].tobytes()
            z = oracle.compress(d)
            rc, back = oracle.decompress_safe(z, len(d))
            errors += int(rc != 0 or back != d)
            h.update(z)
        errors_all, elapsed = shard.completion_barrier(dist, torch.device("cpu"), errors,
                                                       0.5 + rank)
        q.put((rank, mine, errors_all, elapsed, h.hexdigest()))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_completion_barrier():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, ids0, e0, t0, _), (r1, ids1, e1, t1, _) = res
    assert sorted(ids0 + ids1) == list(range(64))
    assert e0 == e1 == 0                       # summed over ranks
    assert t0 == t1 == pytest.approx(1.5)      # max over ranks
