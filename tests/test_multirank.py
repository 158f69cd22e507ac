"""Multi-rank path (one process per GPU) without an 8-GPU box:
gloo, world_size 2.

* CPU: the strong-scaling plan (dlsm_amd/sharding.py) covers config 4 exactly
  once -- the 16 SSTables split s mod G, the ONE lookup stream split into
  contiguous shards -- and the per-rank oracle filters union to the 1-rank job.
* GPU (-m gpu): two spawned ranks share GPU 0 and run the bench's own per-rank
  code (sharding.plan / make_inputs / step: filters built once on rank 0 and
  broadcast, lookups sharded); the union of their filters and the
  concatenation of their mask shards must be byte-identical to the oracle's
  single-process answer.
"""
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


def _collect(procs, q, timeout):
    """rank 0's result from the queue; fails as soon as a rank dies instead
    of waiting out the timeout."""
    import queue
    import time

    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            return q.get(timeout=2)
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead:
                for p in procs:
                    p.kill()
                raise AssertionError(f"a rank exited with {dead}")
    for p in procs:
        p.kill()
    raise AssertionError("ranks timed out")


def _cpu_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    from dlsm_amd import sharding as SH

    T, N, Q = 16, 2000, 100_000
    work = SH.plan(rank, world, T, N, Q, "strong")
    digests = {}
    for s, (first, step) in zip(work.tables, work.values):
        v = first + step * np.arange(N, dtype=np.uint64)
        digests[s] = oracle.fnv1a64(oracle.full_build(oracle.keys_from_values(v), N))
    qv = SH.lookup_values(work, 2 * 8 * N)
    t = SH.max_over_ranks(1.0 + rank, dist)
    weak = SH.plan(rank, world, T, N, Q, "weak")
    gathered = [None] * world
    dist.all_gather_object(gathered, (work.tables, (work.lookup_lo, work.lookup_hi), digests,
                                      qv.tolist(), weak.values, weak.lookup_seed))
    if rank == 0:
        q.put((t, gathered))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_strong_plan():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    t, gathered = _collect(procs, q, 300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert t == 2.0  # max over ranks
    (m0, r0, d0, q0, w0, s0), (m1, r1, d1, q1, w1, s1) = gathered
    # config 4: every table exactly once, s -> s mod 2
    assert m0 == list(range(0, 16, 2)) and m1 == list(range(1, 16, 2))
    assert r0 == (0, 50_000) and r1 == (50_000, 100_000)
    # the two lookup shards concatenate to the single-rank stream (mt19937_64(1000))
    import oracle
    from dlsm_amd import sharding as SH

    whole = SH.lookup_values(SH.plan(0, 1, 16, 2000, 100_000, "strong"), 2 * 8 * 2000)
    assert np.array_equal(np.array(q0 + q1, dtype=np.uint64), whole)
    assert np.array_equal(oracle.mt_values(1000, 2 * 8 * 2000, 100_000), whole)
    # union of the ranks' filters == the 1-rank job's filters (table s <- v = 16 i + s)
    union = {**d0, **d1}
    assert sorted(union) == list(range(16))
    for s in (0, 7, 15):
        v = s + 16 * np.arange(2000, dtype=np.uint64)
        assert oracle.fnv1a64(oracle.full_build(oracle.keys_from_values(v), 2000)) == union[s]
    # weak scaling: every rank its own 16 tables and lookup stream, disjoint keys
    assert w0 != w1 and s0 == 1000 and s1 == 1001


def test_single_rank_plan_is_the_whole_job():
    from dlsm_amd import sharding as SH

    assert SH.max_over_ranks(3.5, None) == 3.5
    assert SH.shard_range(10, 0, 1) == (0, 10)
    w = SH.plan(0, 1, 16, 100, 1000, "strong")
    assert w.tables == list(range(16)) and (w.lookup_lo, w.lookup_hi) == (0, 1000)
    assert w.values == [(s, 16) for s in range(16)]
    for G in (1, 2, 4, 8):
        plans = [SH.plan(r, G, 16, 100, 1000, "strong") for r in range(G)]
        assert sorted(sum((p.tables for p in plans), [])) == list(range(16))
        assert sum(p.n_lookups for p in plans) == 1000
        assert all(plans[r].lookup_hi == plans[r + 1].lookup_lo for r in range(G - 1))


# ---------------------------------------------------------------------------
# GPU: two ranks on GPU 0 through gloo, the bench's own per-rank code
# ---------------------------------------------------------------------------
_T, _N, _Q, _F = 16, 20_000, 1_000_003, 8


def _gpu_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import dlsm_amd
    from dlsm_amd import sharding as SH

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ctx = dlsm_amd.Context(0)
    stream = torch.cuda.Stream(device=dev)  # as bench.py: torch and the context share it
    ctx.set_stream(stream)
    work = SH.plan(rank, world, _T, _N, _Q, "strong")
    inp = SH.make_inputs(ctx, work, _N, _F, 10, dev, stream=stream, dist=dist)
    for _ in range(2):  # the bench's step, twice (the second reuses the job table)
        SH.step(ctx, inp, 10)
    ctx.sync()
    torch.cuda.synchronize()
    L = inp.lens.cpu().numpy()
    filters = {s: inp.outs[j][: int(L[j])].cpu().numpy().tobytes() for j, s in enumerate(work.tables)}
    out = (work.tables, filters, inp.mask[: work.n_lookups].cpu().numpy().tobytes(),
           [f.cpu().numpy().tobytes() for f in inp.filters])
    inp.fs.close()
    ctx.close()
    gathered = [None] * world
    dist.all_gather_object(gathered, out)
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_ranks_on_gpu_strong_scaling_parity(orc):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered = _collect(procs, q, 240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    (t0, f0, m0, s0), (t1, f1, m1, s1) = gathered
    assert t0 == list(range(0, 16, 2)) and t1 == list(range(1, 16, 2))
    union = {**f0, **f1}
    for s in range(_T):
        want = orc.full_build(orc.dbbench_keys(s, _T, _N), _N)
        assert union[s] == want, s
    # the replicated filter set: rank 1 received rank 0's bytes
    filters = [orc.full_build(orc.dbbench_keys(f, _F, _N), _N) for f in range(_F)]
    assert s0 == filters and s1 == filters
    qk = orc.keys_from_values(orc.mt_values(1000, 2 * _F * _N, _Q))
    want = orc.full_probe(filters, qk, _Q, nthreads=8)
    got = np.frombuffer(m0 + m1, dtype=np.uint8)
    assert got.size == _Q and np.array_equal(got, want)
