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


def _runs(orc, seed, n, max_rep):
    """n distinct keys, key i repeated 1..max_rep times in a row (and one run
    of max_rep * 50): the hash stream AddKey sees for several versions of a
    user key."""
    rng = np.random.default_rng(seed)
    keys = orc.dbbench_keys(seed, 9, n).reshape(n, 20)
    rep = rng.integers(1, max_rep + 1, size=n)
    if n > 10:
        rep[n // 2] = max_rep * 50
    dup = np.repeat(keys, rep, axis=0).reshape(-1)
    return dup, int(rep.sum())


@pytest.mark.gpu
@pytest.mark.parametrize("small", [True, False])
@pytest.mark.parametrize("n", [1, 3_000, 153_846, 209_664, 209_665])
def test_gpu_hashed_small_and_sliced_paths(gpu, orc, small, n):
    """The one-launch path for small hashed jobs (<= 4,096 lines: n <= 209,664
    at 10 bits/key) and the count + partition + slice path give the same
    bytes as the oracle -- at the boundary, with and without repeated keys."""
    import dlsm_amd

    was = gpu.get_option(dlsm_amd.OPT_SMALL_BUILD)
    gpu.set_small_build(small)
    try:
        keys = orc.dbbench_keys(5, 7, n)
        assert gpu.full_build_hashed([bloom_hash_k20(keys)])[0] == orc.full_build(keys, n)
        dup, m = _runs(orc, n, max(1, n // 3), 3)
        want = orc.full_build(dup, m)
        assert gpu.full_build_hashed([bloom_hash_k20(dup)])[0] == want
    finally:
        gpu.set_option(dlsm_amd.OPT_SMALL_BUILD, was)


@pytest.mark.gpu
def test_gpu_hashed_small_batch_and_bpk(gpu, orc):
    """Many small jobs of different sizes in one launch (the batcher's shape),
    including empty and one-hash-repeated jobs, at several bits_per_key."""
    import dlsm_amd

    was = gpu.get_option(dlsm_amd.OPT_SMALL_BUILD)
    gpu.set_small_build(True)
    sizes = [0, 1, 2, 63, 64, 65, 1000, 4097, 30_000, 153_846, 200_000]
    for bpk in (1, 6, 10, 16):
        keys = [orc.dbbench_keys(s + 40, 3, n) for s, n in enumerate(sizes)]
        hs = [bloom_hash_k20(k) for k in keys]
        same = np.repeat(hs[-2][:1], 5000)  # one key 5,000 times: one distinct hash
        got = gpu.full_build_hashed(hs + [same], bpk)
        for k, n, g in zip(keys, sizes, got):
            assert g == orc.full_build(k, n, bpk=bpk), (bpk, n)
        one = np.tile(keys[-2][:20], 5000)
        assert got[-1] == orc.full_build(one, 5000, bpk=bpk)
    gpu.set_option(dlsm_amd.OPT_SMALL_BUILD, was)


@pytest.mark.gpu
@pytest.mark.parametrize("small", [True, False])
def test_gpu_hashed_capacity_error(gpu, orc, small):
    import dlsm_amd

    was = gpu.get_option(dlsm_amd.OPT_SMALL_BUILD)
    gpu.set_small_build(small)
    try:
        keys = orc.dbbench_keys(0, 1, 5000)
        need = dlsm_amd.full_size(5000)[0]
        with pytest.raises(dlsm_amd.DlsmError) as e:
            gpu.full_build_hashed([bloom_hash_k20(keys)], 10, caps=[need - 1])
        assert e.value.status == -2
        assert gpu.full_build_hashed([bloom_hash_k20(keys)], 10, caps=[need])[0] == orc.full_build(keys, 5000)
    finally:
        gpu.set_option(dlsm_amd.OPT_SMALL_BUILD, was)


@pytest.mark.gpu
@pytest.mark.parametrize("small", [True, False])
def test_gpu_hashed_dev_unaligned_hashes(gpu, orc, small):
    """Device hashes at every 4-byte offset from a 16-byte boundary, with the
    words just before and after equal to the first / last hash (a sweep that
    read them as neighbours would drop the first hash or add one)."""
    import torch

    import dlsm_amd

    n = 20_011
    keys = orc.dbbench_keys(21, 5, n)
    h = bloom_hash_k20(keys).view(np.int32)
    want = orc.full_build(keys, n)
    was = gpu.get_option(dlsm_amd.OPT_SMALL_BUILD)
    gpu.set_small_build(small)
    try:
        for off in range(4):
            host = np.zeros(n + 8, dtype=np.int32)
            host[off:off + n] = h
            if off:
                host[off - 1] = h[0]
            host[off + n] = h[-1]
            base = torch.from_numpy(host).cuda()
            out = torch.zeros(len(want) + 64, dtype=torch.uint8, device="cuda")
            lens = torch.zeros(1, dtype=torch.uint64, device="cuda")
            torch.cuda.synchronize()
            gpu.full_build_hashed_dev([base[off:off + n]], [out], lens)
            gpu.sync()
            ln = int(lens.cpu()[0])
            assert ln == len(want) and bytes(out[:ln].cpu().numpy()) == want, off
    finally:
        gpu.set_option(dlsm_amd.OPT_SMALL_BUILD, was)
