"""Work partitioning across GPUs (one process per GPU).

SSTables are independent: each filter depends only on its own keys
(one FullFilterBlockBuilder per TableBuilder, table_builder_computeside.cc:62-64),
so tables shard one-per-GPU with no collective.  Probes replicate the (small)
filter set per GPU and shard the lookups.  The only cross-rank operations are
the bench's barrier and its max-over-ranks time.
"""
from __future__ import annotations


def table_values(rank: int, table: int, tables_per_rank: int, keys_per_table: int):
    """(first, step) of the db_bench key values of `table` on `rank`:
    v = first + step * i, i < keys_per_table.  Rank 0 is SURVEY.md §8d's
    config 4 (table s <- v = 16 i + s); ranks never share a key."""
    T, N = tables_per_rank, keys_per_table
    return table + rank * T * N, T


def tables_for_rank(rank: int, world: int, n_tables: int):
    """Strong-scaling assignment (table s -> GPU s mod G), for callers that split
    one fixed set of SSTables (e.g. one compaction round) across GPUs."""
    return [s for s in range(n_tables) if s % world == rank]


def lookup_seed(rank: int) -> int:
    """mt19937_64 seed of rank's lookup stream (1000)."""
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
