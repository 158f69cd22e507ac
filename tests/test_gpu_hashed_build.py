"""Builds from host-computed BloomHash values (dlsm_bloom_full_build_hashed):
the path of an AddKey that hashes on the host like the reference's
(table/full_filter_block.cc:39-49) and hands Finish 4 bytes per key.  Filters
must equal the oracle's built from the keys themselves, with the hashes given
deduplicated or not (the GPU drops consecutive equal hashes like AddKey)."""
import numpy as np
import pytest


def bloom_hash_k20(keys: np.ndarray) -> np.ndarray:
    """BloomHash of packed 20-byte keys (util/hash.cc:22-62: 5 LE words, no
    tail), vectorised -- test helper; checked against dlsm_bloom_hash."""
    w = keys.reshape(-1, 20).view("<u4").astype(np.uint64)
    m = np.uint64(0xC6A4A793)
    mask = np.uint64(0xFFFFFFFF)
    h = np.full(w.shape[0], (0xBC9F1D34 ^ ((20 * 0xC6A4A793) & 0xFFFFFFFF)), dtype=np.uint64)
    for j in range(5):
        h = (h + w[:, j]) & mask
        h = (h * m) & mask
        h ^= h >> np.uint64(16)
    return h.astype(np.uint32)


def test_vectorised_hash_matches_library(orc):
    import dlsm_amd

    k = orc.dbbench_keys(7, 3, 500)
    h = bloom_hash_k20(k)
    for i in (0, 1, 250, 499):
        assert int(h[i]) == dlsm_amd.bloom_hash(k[20 * i: 20 * i + 20].tobytes())


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 52, 5000, 153_846, 1_600_000])
def test_gpu_hashed_build_matches_oracle(gpu, orc, n):
    keys = orc.dbbench_keys(3, 5, n)
    h = bloom_hash_k20(keys)
    got = gpu.full_build_hashed([h])[0]
    assert got == orc.full_build(keys, n)


@pytest.mark.gpu
def test_gpu_hashed_build_dedups_like_addkey(gpu, orc):
    """Every key twice in a row: the hashes repeat, the line count is that of
    the distinct keys (AddKey's consecutive-hash check)."""
    n = 40_000
    keys = orc.dbbench_keys(11, 2, n)
    h = bloom_hash_k20(keys)
    twice = np.repeat(h, 2)
    dup_keys = np.repeat(keys.reshape(n, 20), 2, axis=0).reshape(-1)
    want = orc.full_build(dup_keys, 2 * n)
    assert want == orc.full_build(keys, n)
    got = gpu.full_build_hashed([h, twice])
    assert got[0] == want and got[1] == want


@pytest.mark.gpu
def test_gpu_hashed_batch_of_tables(gpu, orc):
    """16 tables in one call (the batcher's shape), mixed sizes."""
    sizes = [153_846, 1000, 0, 77_777] * 4
    keys = [orc.dbbench_keys(s, 16, n) for s, n in enumerate(sizes)]
    got = gpu.full_build_hashed([bloom_hash_k20(k) for k in keys])
    for k, n, g in zip(keys, sizes, got):
        assert g == orc.full_build(k, n)
