"""Work partitioning across GPUs (one process per GPU).

SSTables are independent: each filter depends only on its own keys (one
FullFilterBlockBuilder per TableBuilder, table_builder_computeside.cc:62-64;
one builder thread per subcompaction, db/db_impl.cc:3373-3386), so the
SSTables of one flush/compaction round split over the GPUs with no
collective.  Probes replicate the (small) stacked filter set to every GPU once
and shard the lookup stream; nothing in the hot loop communicates.

Two shapes (BASELINE configs 3 and 4):

* strong (the north star's "16 SSTables sharded across 1/2/4/8 GPUs"): ONE
  fixed job -- the 16 config-4 SSTables (table s <- v = 16 i + s) split
  s mod G, and ONE 100 M-key lookup stream (mt19937_64(1000)) split into
  contiguous shards -- against ONE filter set built once (rank 0) and
  broadcast to every rank.  Rank r's masks are the slice r of the 1-GPU run's
  masks, its filters the tables s = r mod G of the 1-GPU run's filters.
* weak: every rank builds its own 16 tables and probes its own 100 M lookups.
"""
from __future__ import annotations

from dataclasses import dataclass, field


def table_values(rank: int, table: int, tables_per_rank: int, keys_per_table: int):
    """Weak scaling: (first, step) of the db_bench key values of `table` on
    `rank`: v = first + step * i, i < keys_per_table.  Rank 0 is SURVEY.md
    §8d's config 4 (table s <- v = 16 i + s); ranks never share a key."""
    T, N = tables_per_rank, keys_per_table
    return table + rank * T * N, T


def tables_for_rank(rank: int, world: int, n_tables: int):
    """Strong-scaling assignment (table s -> GPU s mod G) of one fixed set of
    SSTables (e.g. one compaction round's outputs)."""
    return [s for s in range(n_tables) if s % world == rank]


def lookup_seed(rank: int) -> int:
    """Weak scaling: mt19937_64 seed of rank's own lookup stream (config 3: 1000)."""
    return 1000 + rank


def shard_range(n: int, rank: int, world: int):
    """Contiguous [lo, hi) share of n lookups for `rank`."""
    return n * rank // world, n * (rank + 1) // world


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """The bench's max-over-ranks wall time (barrier semantics are the caller's)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    import torch

    if dist.get_backend() != "nccl":
        device = "cpu"  # gloo reduces host tensors
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


@dataclass
class RankWork:
    """What one rank builds and probes per step."""
    scaling: str
    tables: list = field(default_factory=list)   # table ids of the job
    values: list = field(default_factory=list)   # (first, step) of each table's keys
    lookup_seed: int = 1000
    lookup_lo: int = 0                           # [lo, hi) of the lookup stream
    lookup_hi: int = 0

    @property
    def n_lookups(self) -> int:
        return self.lookup_hi - self.lookup_lo


def plan(rank: int, world: int, n_tables: int, keys_per_table: int, n_lookups: int,
         scaling: str = "strong") -> RankWork:
    if scaling == "strong":
        tabs = tables_for_rank(rank, world, n_tables)
        lo, hi = shard_range(n_lookups, rank, world)
        return RankWork("strong", tabs, [(s, n_tables) for s in tabs], 1000, lo, hi)
    if scaling == "weak":
        tabs = list(range(n_tables))
        vals = [table_values(rank, s, n_tables, keys_per_table) for s in tabs]
        return RankWork("weak", tabs, vals, lookup_seed(rank), 0, n_lookups)
    raise ValueError(scaling)


def filter_values(f: int, n_filters: int):
    """(first, step) of stacked filter f's keys: v = F i + f (config 3)."""
    return f, n_filters


def lookup_values(work: RankWork, modulus: int):
    """This rank's lookup values: the [lo, hi) slice of mt19937_64(seed) mod
    modulus (only the prefix up to hi is generated)."""
    import numpy as np

    from . import workload as W

    v = W.mt19937_64(work.lookup_seed, work.lookup_hi)[work.lookup_lo:]
    return v % np.uint64(modulus)


@dataclass
class RankInputs:
    tables: list        # dlsm_amd.Keys (device)
    outs: list          # device uint8 slots, one per table
    lens: object        # device uint64[len(tables)]
    filters: list       # device uint8 tensors (the replicated filter set)
    fs: object          # dlsm_amd.FilterSet over `filters`
    lookups: object     # dlsm_amd.Keys (device), this rank's shard
    mask: object        # device uint8[n_lookups * mask_bytes]


def make_inputs(ctx, work: RankWork, keys_per_table: int, n_filters: int, bits_per_key: int,
                dev, stream=None, dist=None, lookup_shard=None) -> RankInputs:
    """Materialise a rank's inputs in HBM (untimed set-up).  The filter set is
    built once -- by rank 0 in strong scaling, then broadcast to every rank
    (the one-time exchange of SURVEY.md §8e; RCCL over xGMI with the nccl
    backend, host memory with gloo) -- and every rank keeps its own copy.
    Without `dist` (one process, a thread per GPU) each device builds the set
    from the same keys.  `lookup_shard`: this rank's shard of the lookup
    stream when the caller generated the stream once (else generated here)."""
    import contextlib

    import numpy as np
    import torch

    import dlsm_amd

    from . import workload as W

    N, F, bpk = keys_per_table, n_filters, bits_per_key
    # torch makes the inputs on `stream` (or its current stream); every library
    # call below starts after a device synchronise, so nothing depends on the
    # context using the same stream
    ctxm = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
    with ctxm:
        tables, outs = [], []
        for first, step in work.values:
            v = torch.arange(N, device=dev, dtype=torch.int64) * step + first
            tables.append(dlsm_amd.Keys(W.dbbench_keys_torch(v), N, 20))
            outs.append(torch.zeros(dlsm_amd.full_size(N, bpk)[0], dtype=torch.uint8, device=dev))
        lens = torch.zeros(max(1, len(tables)), dtype=torch.uint64, device=dev)
        flen = dlsm_amd.full_size(N, bpk)[0]  # distinct keys: the speculative length is exact
        fouts = [torch.zeros(flen, dtype=torch.uint8, device=dev) for _ in range(F)]
    builder = work.scaling != "strong" or dist is None or dist.get_rank() == 0
    if builder:
        with ctxm:
            ftabs = []
            for f in range(F):
                first, step = filter_values(f, F)
                v = torch.arange(N, device=dev, dtype=torch.int64) * step + first
                ftabs.append(dlsm_amd.Keys(W.dbbench_keys_torch(v), N, 20))
            flens = torch.zeros(F, dtype=torch.uint64, device=dev)
        torch.cuda.synchronize(dev)
        ctx.full_build_dev(ftabs, fouts, flens, bpk)
        ctx.sync()
        assert all(int(x) == flen for x in flens.cpu().numpy())
        del ftabs
    if work.scaling == "strong" and dist is not None and dist.get_world_size() > 1:
        torch.cuda.synchronize(dev)  # the receive buffers were zeroed on `stream`
        for f in range(F):
            if dist.get_backend() == "nccl":
                dist.broadcast(fouts[f], src=0)
            else:
                h = fouts[f].cpu()
                dist.broadcast(h, src=0)
                fouts[f].copy_(h.to(dev))
    torch.cuda.synchronize(dev)
    fs = ctx.filterset(fouts, on_device=True)
    qv = lookup_shard if lookup_shard is not None else lookup_values(work, 2 * F * N)
    with ctxm:
        q = W.dbbench_keys_torch(torch.from_numpy(qv.astype(np.int64)).to(dev))
        mask = torch.empty(max(1, work.n_lookups) * fs.mask_bytes, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    return RankInputs(tables, outs, lens, fouts, fs, dlsm_amd.Keys(q, work.n_lookups, 20), mask)


def step(ctx, inp: RankInputs, bits_per_key: int):
    """One step of the path on this rank: build its SSTables' filters, probe
    its lookup shard.  Asynchronous on ctx's stream."""
    if inp.tables:
        ctx.full_build_dev(inp.tables, inp.outs, inp.lens, bits_per_key)
    if inp.lookups.n:
        ctx.full_probe_dev(inp.fs, inp.lookups, inp.mask)
