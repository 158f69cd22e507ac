"""Synthetic workloads in the reference's own shapes (bench harness helpers).

* db_bench keys: ``GenerateKeyFromInt`` (benchmarks/db_bench.cc:677-711) --
  big-endian v in the first 8 bytes, '0' padding to key_size (20).
* lookup stream: ``std::mt19937_64(seed)() % modulus`` -- the engine behind
  Random64 (util/random.h:140-165); vectorised MT19937-64 in numpy.

These build inputs only; they are not on the measured path.
"""
from __future__ import annotations

import numpy as np

_NN, _MM = 312, 156
_MATRIX = np.uint64(0xB5026F5AA96619E9)
_UM = np.uint64(0xFFFFFFFF80000000)
_LM = np.uint64(0x7FFFFFFF)


def mt19937_64(seed: int, n: int) -> np.ndarray:
    """First n outputs of std::mt19937_64(seed)."""
    mt = np.zeros(_NN, dtype=np.uint64)
    mt[0] = np.uint64(seed)
    with np.errstate(over="ignore"):
        for i in range(1, _NN):
            prev = int(mt[i - 1])
            mt[i] = np.uint64((6364136223846793005 * (prev ^ (prev >> 62)) + i) & 0xFFFFFFFFFFFFFFFF)
    out = np.empty(((n + _NN - 1) // _NN) * _NN, dtype=np.uint64)
    one = np.uint64(1)
    for t in range(len(out) // _NN):
        # i in [0, 156): old mt[i], mt[i+1], mt[i+156]
        x = (mt[0:_MM] & _UM) | (mt[1:_MM + 1] & _LM)
        mt[0:_MM] = mt[_MM:_NN] ^ (x >> one) ^ ((x & one) * _MATRIX)
        # i in [156, 311): new mt[i-156], old mt[i], mt[i+1]
        x = (mt[_MM:_NN - 1] & _UM) | (mt[_MM + 1:_NN] & _LM)
        mt[_MM:_NN - 1] = mt[0:_NN - 1 - _MM] ^ (x >> one) ^ ((x & one) * _MATRIX)
        # i = 311: mt[0] new
        x = (mt[_NN - 1] & _UM) | (mt[0] & _LM)
        mt[_NN - 1] = mt[_MM - 1] ^ (x >> one) ^ ((x & one) * _MATRIX)
        out[t * _NN:(t + 1) * _NN] = mt
    y = out[:n].copy()
    y ^= (y >> np.uint64(29)) & np.uint64(0x5555555555555555)
    y ^= (y << np.uint64(17)) & np.uint64(0x71D67FFFEDA60000)
    y ^= (y << np.uint64(37)) & np.uint64(0xFFF7EEE000000000)
    y ^= y >> np.uint64(43)
    return y


def dbbench_keys_np(values: np.ndarray, key_size: int = 20) -> np.ndarray:
    """Pack db_bench keys for the given u64 values: uint8[n * key_size]."""
    v = np.ascontiguousarray(values, dtype=np.uint64)
    n = v.size
    fill = min(key_size, 8)
    out = np.full((n, key_size), ord("0"), dtype=np.uint8)
    be = v.astype(">u8").view(np.uint8).reshape(n, 8)
    out[:, :fill] = be[:, 8 - fill:]
    return out.reshape(-1)


def dbbench_keys_torch(values, key_size: int = 20):
    """Same as dbbench_keys_np but from a torch int64 tensor, on its device."""
    import torch

    v = values.to(torch.int64)
    n = v.numel()
    fill = min(key_size, 8)
    out = torch.full((n, key_size), ord("0"), dtype=torch.uint8, device=v.device)
    for i in range(fill):
        sh = 8 * (fill - 1 - i)
        out[:, i] = ((v >> sh) & 0xFF).to(torch.uint8)
    return out.reshape(-1)


def arith_values(first: int, step: int, n: int) -> np.ndarray:
    return (np.uint64(first) + np.uint64(step) * np.arange(n, dtype=np.uint64)).astype(np.uint64)


# The version of db_bench's final state at config 5 (the replay of DESIGN.md
# §7: 5 + 40 + 377 files on levels 1-3 for 100 M keys, the key space spread
# over the levels as 1 : 10 : 100) plus 4 level-0 flush files of 153,846 keys
# over random ranges.  Level files partition [0, V); each file's filter holds
# every key of its range on that level (stride 100 / 10 / 1).
VERSION_SHAPE = ((1, 5, 100), (2, 40, 10), (3, 377, 1))


def dbbench_version(ctx, dev, space: int = 100_000_000, seed: int = 11):
    """Build the version's filters on the GPU (ctx.full_build_dev, 10 bits /
    key) and return its dlsm_amd.VersionFile list (device filters)."""
    import torch

    from . import Keys, VersionFile, full_size

    def key(v):
        return dbbench_keys_np(np.array([v], dtype=np.uint64)).tobytes()

    def build(values_dev):
        n = int(values_dev.numel())
        keys = Keys(dbbench_keys_torch(values_dev), n, 20)
        out = torch.zeros(full_size(n)[0] + 16, dtype=torch.uint8, device=dev)
        lens = torch.zeros(1, dtype=torch.uint64, device=dev)
        ctx.full_build_dev([keys], [out], lens, 10)
        ctx.sync()
        return out[: int(lens.cpu()[0])].clone()

    files = []
    rng = np.random.default_rng(seed)
    seq = 1 << 30
    for level, nf, stride in VERSION_SHAPE:
        edges = np.linspace(0, space, nf + 1).astype(np.int64)
        for q in range(nf):
            lo, hi = int(edges[q]) + (level - 1), int(edges[q + 1]) - 1
            vals = torch.arange(lo, hi, stride, device=dev, dtype=torch.int64)
            files.append(VersionFile(level, 10_000 * level + q, key(lo), key(int(vals[-1])), (seq << 8) | 1,
                                     build(vals)))
            seq -= 1
    for j in range(4):  # level 0: flush files of 153,846 keys over random ranges
        lo = int(rng.integers(0, space - 153_846 * 600))
        step = int(rng.integers(50, 600))
        vals = torch.arange(lo, lo + 153_846 * step, step, device=dev, dtype=torch.int64)
        files.append(VersionFile(0, 900_000 + j, key(lo), key(int(vals[-1])), ((seq + 10 + j) << 8) | 1,
                                 build(vals)))
    return files
