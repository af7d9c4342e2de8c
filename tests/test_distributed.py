"""N>1 path on CPU: world_size-2 gloo ranks each take their shard of one batch
(sharedhashfile_amd.shard, the split bench.py and the *_multi ABI use), hash it
(with the CPU oracle standing in for the GPU: test infrastructure), and rank 0
checks that the gathered shards equal the whole batch's hashes -- i.e. the split
is disjoint, covering and needs no data exchange beyond returning results.
Also rehearses bench.py's barrier + max-over-ranks timing reduction.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sharedhashfile_amd.shard import shard_fixed, shard_range, shard_var


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.oracle_py import Oracle

        o = Oracle()
        rng = np.random.default_rng(123)  # same batch on every rank
        fixed = rng.integers(0, 256, size=1001 * 16, dtype=np.uint8)
        lens = rng.integers(0, 300, size=777)
        off = np.zeros(lens.size + 1, dtype=np.uint64)
        off[1:] = np.cumsum(lens)
        data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)

        lo, hi, part = shard_fixed(fixed, 16, rank, world)
        mine_f = o.hash_fixed(part, 16)
        lo_v, hi_v, pdata, poff = shard_var(data, off, rank, world)
        mine_v = o.hash_var(pdata, poff)

        # results return to rank 0 (the caller's process); the hashing itself exchanged nothing
        gathered = [None] * world
        dist.all_gather_object(gathered, (lo, hi, mine_f, lo_v, hi_v, mine_v))

        # bench.py's timing reduction: barrier, local elapsed, MAX over ranks
        dist.barrier()
        t = torch.tensor([0.5 + rank, 1.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            full_f = o.hash_fixed(fixed, 16)
            full_v = o.hash_var(data, off)
            cat_f = np.concatenate([g[2] for g in gathered])
            cat_v = np.concatenate([g[5] for g in gathered])
            ranges = [(g[0], g[1]) for g in gathered]
            ok = (np.array_equal(cat_f, full_f) and np.array_equal(cat_v, full_v)
                  and ranges[0][0] == 0 and ranges[-1][1] == 1001
                  and all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
                  and float(t[0]) == 0.5 + world - 1)
            result_q.put(bool(ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_sharded_batch(world):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert q.get() is True


def test_shard_range_properties():
    for n in [0, 1, 7, 64, 1001, 10**9]:
        for world in [1, 2, 3, 8]:
            rs = [shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            sizes = [hi - lo for lo, hi in rs]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)
