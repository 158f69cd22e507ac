"""Multi-rank path on CPU (gloo, world_size 2): SSTable sharding is disjoint
and covers config 4, lookups shard exactly, the max-over-ranks time is the
max, and two ranks' CPU-oracle filters for their shards equal a single-process
build of the same tables (no data-path collective needed)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    from dlsm_amd import sharding as SH

    # weak scaling: every rank has its own 16 tables; ranks never share keys
    T, N = 16, 2000
    vals = set()
    digests = []
    for s in range(T):
        first, step = SH.table_values(rank, s, T, N)
        v = first + step * np.arange(N, dtype=np.uint64)
        vals.update(v.tolist())
        f = oracle.full_build(oracle.keys_from_values(v), N)
        digests.append(oracle.fnv1a64(f))
    # strong-scaling assignment s -> s mod G
    mine = SH.tables_for_rank(rank, world, 16)
    lo, hi = SH.shard_range(100_000_000, rank, world)
    t = SH.max_over_ranks(1.0 + rank, dist)
    gathered = [None] * world
    dist.all_gather_object(gathered, (sorted(vals)[:5], len(vals), mine, (lo, hi), digests))
    if rank == 0:
        q.put((t, gathered))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_sharding():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    t, gathered = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert t == 2.0  # max over ranks
    (v0, n0, m0, r0, d0), (v1, n1, m1, r1, d1) = gathered
    assert n0 == n1 == 16 * 2000
    assert sorted(m0 + m1) == list(range(16)) and not set(m0) & set(m1)
    assert r0 == (0, 50_000_000) and r1 == (50_000_000, 100_000_000)
    # rank 0's tables are SURVEY config 4 (v = 16 i + s)
    import oracle

    for s in (0, 7, 15):
        v = s + 16 * np.arange(2000, dtype=np.uint64)
        assert oracle.fnv1a64(oracle.full_build(oracle.keys_from_values(v), 2000)) == d0[s]
    assert d0 != d1  # disjoint key sets -> different filters


def test_single_rank_max_is_identity():
    from dlsm_amd import sharding as SH

    assert SH.max_over_ranks(3.5, None) == 3.5
    assert SH.shard_range(10, 0, 1) == (0, 10)
