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
    """A rank: its round-robin share through the library's planner with a
    stand-in for the codec (tests/native/split_mock.c: output = input
    reversed), then the completion barrier."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import ctypes
        lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "native", "libsplit_mock.so"))
        lib.mock_batch.restype = ctypes.c_int
        nglobal = 64
        mine = shard.round_robin(nglobal, rank, world)
        arena, offs, lens = synth.batch(synth.ITB, 0, [16384] * len(mine), seeds=mine)
        blocks = [arena[int(offs[b]): int(offs[b]) + int(lens[b])].tobytes()
                  for b in range(len(mine))]
        n = len(blocks)
        srcs = [ctypes.create_string_buffer(b, len(b)) for b in blocks]
        dsts = [ctypes.create_string_buffer(len(b)) for b in blocks]
        vp = lambda bufs: (ctypes.c_void_p * n)(*[ctypes.addressof(x) for x in bufs])
        ln = (ctypes.c_size_t * n)(*[len(b) for b in blocks])
        dev_of = (ctypes.c_int * n)()
        chunk_of = (ctypes.c_long * n)()
        seq_of = (ctypes.c_long * n)()
        used = ctypes.c_int(0)
        rc = lib.mock_batch(ctypes.c_size_t(n), vp(srcs), ln, vp(dsts), 2, ctypes.c_size_t(1 << 16),
                            ctypes.c_size_t(1 << 17), ctypes.c_size_t(1 << 20), dev_of, chunk_of,
                            seq_of, ctypes.byref(used))
        errors = int(rc != 0) + sum(int(d.raw != b[::-1]) for d, b in zip(dsts, blocks))
        h = hashlib.sha256(b"".join(blocks)).hexdigest()
        errors_all, elapsed = shard.completion_barrier(dist, torch.device("cpu"), errors,
                                                       0.5 + rank)
        q.put((rank, mine, errors_all, elapsed, h))
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


def _gpu_worker(rank, world, port, q):
    """A rank on the GPU box: its share through the real library (host
    batches on cuda:0, both ranks sharing the one GPU), checked by round trip;
    the compressed bytes go back to the parent, which checks them against the
    oracle."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["POM_LZO_DEVICES"] = "0"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pomegranate_amd import lzo
        mine = shard.round_robin(48, rank, world)
        blocks = [synth.block(synth.ITB, 7000 + i, 4096 + 1024 * (i % 13)) for i in mine]
        rc, st, comps = lzo.compress_batch(blocks)
        rc2, st2, outs = lzo.decompress_batch(comps, [len(b) for b in blocks])
        errors = int(rc != 0 or rc2 != 0) + sum(int(x != 0) for x in st + st2) + \
            sum(int(o != b) for o, b in zip(outs, blocks))
        errors_all, elapsed = shard.completion_barrier(dist, torch.device("cpu"), errors, 1.0)
        q.put((rank, mine, errors_all, comps))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_two_ranks_share_the_gpu_codec(oracle):
    """The N>1 bench path in rehearsal with the real GPU codec: two gloo ranks
    (one GPU box), round-robin shares, completion barrier; every compressed
    block equals the oracle's."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(res[0][1] + res[1][1]) == list(range(48))
    assert res[0][2] == res[1][2] == 0
    for rank, mine, _, comps in res:
        for i, z in zip(mine, comps):
            assert z == oracle.compress(synth.block(synth.ITB, 7000 + i, 4096 + 1024 * (i % 13)))


def _rccl_worker(port, q):
    """World size 1 over RCCL exactly as bench.py:main initialises it (nccl
    backend, device_id), then the completion barrier on device tensors and a
    small C4 share through bench.run_resident, whose barriers and all-reduces
    now run over RCCL."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = "0"
    os.environ["WORLD_SIZE"] = "1"
    try:
        import argparse
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        from pomegranate_amd import lzo
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        try:
            assert dist.get_backend() == "nccl"
            barrier = shard.completion_barrier(dist, dev, 3, 1.25)
            args = argparse.Namespace(workload="c4", c4_blocks=256, steps=2, warmup=1,
                                      compress_steps=1, model="itb", block_bytes=65536,
                                      blocks=4096, no_cpu=True, cpu_seconds=0.0)
            lzo.load()
            res, errors = bench.run_resident(args, torch, dist, lzo, synth, shard, dev, 1, 0,
                                             "nccl")
            q.put(("ok", barrier, errors, res["value"], res["config"]["blocks_per_gpu"]))
        finally:
            dist.destroy_process_group()
    except Exception as exc:                     # reported to the parent
        q.put(("error", repr(exc)))


@pytest.mark.gpu
def test_rccl_world_one_barrier_and_c4_share():
    """the RCCL (nccl backend) path runs once on a GPU
    before any scaling run needs it."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert res[0] == "ok", res
    _, barrier, errors, value, nblocks = res
    assert barrier == (3, 1.25)
    assert errors == 0 and nblocks == 256 and value > 0
    assert p.exitcode == 0


def _bench(args, env_extra, timeout=240):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_gpus_n_without_launcher_starts_n_ranks():
    """`bench.py --gpus 2` with no WORLD_SIZE starts two
    rank processes itself (torch.distributed.run on 127.0.0.1) instead of
    measuring one GPU; each rank sees world size 2."""
    import json
    r = _bench(["--gpus", "2"], {"POM_DIST_BACKEND": "gloo", "POM_BENCH_PLAN_ONLY": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    plans = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert sorted(p["rank"] for p in plans) == [0, 1]
    assert all(p["n_gpus"] == 2 for p in plans)


def test_bench_gpus_n_never_reports_one_gpu():
    """Without a GPU the ranks fail, and so does the whole run: no one-GPU
    JSON line for a two-GPU request; a WORLD_SIZE that disagrees with --gpus
    is refused."""
    r = _bench(["--gpus", "2"], {"POM_DIST_BACKEND": "gloo"})
    assert r.returncode != 0
    assert '"n_gpus": 1' not in r.stdout
    r = _bench(["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0",
                                 "POM_BENCH_PLAN_ONLY": "1"}, timeout=60)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
