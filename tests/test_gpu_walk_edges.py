"""Segment-walk edge shapes of the sliced probe (bloom_kernels.hip SegWalk,
seg_locate_set_lds) that uniformly random lookups almost never produce:

* sparse: every 8,192-key chunk sends all its keys to ONE slice, so nearly
  every (slice, 64-chunk group) is empty -- the walk's empty-group loop, and
  groups whose only run spans dozens of windows;
* aligned: every chunk sends exactly 256 keys (64 16-byte units, no padding)
  to each of 32 slices, so every run starts exactly on a window boundary --
  window 0 and window 1 of a set both begin with a new run (the flag of lane
  0 is ignored and the run is counted at the window start instead);
* one slice: every key of every chunk in slice 0; all other slices walk only
  empty groups to the end of their part.

Lookup keys are drawn from a random pool by the slice their BloomHash line
falls in (numpy restatement of util/hash.cc Hash for 20-byte keys, checked
against the oracle), at the bench's 256 stacked lines per slice; answers are
compared with the CPU oracle on the forced sliced path."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 1_000_000  # keys per filter: L = 19,532 lines, 77 slices of 256 lines
F = 8
C = 8192
R = 256


def bloom_hash20(keys: np.ndarray) -> np.ndarray:
    """util/hash.cc Hash(key, 20, 0xbc9f1d34) for [n, 20] uint8 keys."""
    m = np.uint32(0xC6A4A793)
    w = keys.reshape(-1, 20).view("<u4").astype(np.uint32)  # five little-endian words
    with np.errstate(over="ignore"):
        h = np.full(w.shape[0], np.uint32(0xBC9F1D34) ^ np.uint32((20 * 0xC6A4A793) & 0xFFFFFFFF), dtype=np.uint32)
        for i in range(5):
            h = (h + w[:, i]) * m
            h ^= h >> np.uint32(16)
    return h


@pytest.fixture(scope="module")
def setup(orc):
    filters = [orc.full_build(orc.dbbench_keys(f, F, N), N) for f in range(F)]
    _, L = orc.full_filter_bytes(N)
    rng = np.random.default_rng(20261016)
    pool = rng.integers(0, 256, size=(400_000, 20), dtype=np.uint8)
    h = bloom_hash20(pool)
    for i in range(0, 400_000, 40_009):  # the restatement agrees with the oracle's BloomHash
        assert int(h[i]) == orc.bloom_hash(pool[i].tobytes())
    sl = (h % np.uint32(L)) >> np.uint32(8)
    S = int(sl.max()) + 1
    by_slice = [np.nonzero(sl == s)[0] for s in range(S)]
    assert all(b.size > 0 for b in by_slice)
    return filters, L, S, pool, by_slice, rng


def _draw(pool, by_slice, rng, s, n):
    return pool[rng.choice(by_slice[s], size=n, replace=True)]


def _run(gpu, orc, filters, q: np.ndarray):
    import torch

    import dlsm_amd

    nq = q.shape[0]
    flat = np.ascontiguousarray(q).reshape(-1)
    want = orc.full_probe(filters, flat, nq, nthreads=16)
    fs = gpu.filterset(filters, on_device=False)
    qd = torch.from_numpy(flat).cuda()
    mask = torch.full((nq,), 0xEE, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    gpu.set_path(2)  # sliced, forced
    try:
        gpu.full_probe_dev(fs, dlsm_amd.Keys(qd, nq, 20), mask)
        gpu.sync()
    finally:
        gpu.set_path(0)
        fs.close()
    got = mask.cpu().numpy()
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} wrong answers, first at {bad[:8].tolist()} (chunks {np.unique(bad // C)[:8].tolist()})"
    assert want.any() and not want.all()


def test_sparse_one_slice_per_chunk(gpu, orc, setup):
    filters, L, S, pool, by_slice, rng = setup
    assert S == -(-L // R) and S > 64
    nC = 200
    q = np.concatenate([_draw(pool, by_slice, rng, (c * 7) % S, C) for c in range(nC)]
                       + [pool[rng.integers(0, pool.shape[0], 777)]])
    _run(gpu, orc, filters, q)


def test_runs_aligned_to_windows(gpu, orc, setup):
    filters, L, S, pool, by_slice, rng = setup
    assert S % 2 == 1 and S > 64  # the 32 slices (5c + 2j) mod S of a chunk are distinct
    nC = 150
    chunks = []
    for c in range(nC):
        parts = [_draw(pool, by_slice, rng, (5 * c + 2 * j) % S, 256) for j in range(32)]
        chunks.append(np.concatenate(parts)[rng.permutation(C)])
    q = np.concatenate(chunks + [pool[rng.integers(0, pool.shape[0], 1000)]])
    _run(gpu, orc, filters, q)


def test_every_key_in_one_slice(gpu, orc, setup):
    filters, L, S, pool, by_slice, rng = setup
    q = _draw(pool, by_slice, rng, 0, 130 * C + 5)
    _run(gpu, orc, filters, q)
