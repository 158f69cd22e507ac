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
@pytest.mark.parametrize("n", [1, 3_000, 153_846, 209_664, 209_665])
def test_gpu_hashed_runs_of_repeats(gpu, orc, n):
    """Hash streams with runs of repeated keys (several versions of a user
    key, one run of 150) give the oracle's bytes from the keys themselves."""
    keys = orc.dbbench_keys(5, 7, n)
    assert gpu.full_build_hashed([bloom_hash_k20(keys)])[0] == orc.full_build(keys, n)
    dup, m = _runs(orc, n, max(1, n // 3), 3)
    assert gpu.full_build_hashed([bloom_hash_k20(dup)])[0] == orc.full_build(dup, m)


@pytest.mark.gpu
def test_gpu_hashed_small_batch_and_bpk(gpu, orc):
    """Many small jobs of different sizes in one call (the batcher's shape),
    including empty and one-hash-repeated jobs, at several bits_per_key."""
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


@pytest.mark.gpu
def test_gpu_hashed_capacity_error(gpu, orc):
    import dlsm_amd

    keys = orc.dbbench_keys(0, 1, 5000)
    need = dlsm_amd.full_size(5000)[0]
    with pytest.raises(dlsm_amd.DlsmError) as e:
        gpu.full_build_hashed([bloom_hash_k20(keys)], 10, caps=[need - 1])
    assert e.value.status == -2
    assert gpu.full_build_hashed([bloom_hash_k20(keys)], 10, caps=[need])[0] == orc.full_build(keys, 5000)


@pytest.mark.gpu
def test_gpu_hashed_dev_unaligned_hashes(gpu, orc):
    """Device hashes at every 4-byte offset from a 16-byte boundary, with the
    words just before and after equal to the first / last hash (a sweep that
    read them as neighbours would drop the first hash or add one)."""
    import torch

    n = 20_011
    keys = orc.dbbench_keys(21, 5, n)
    h = bloom_hash_k20(keys).view(np.int32)
    want = orc.full_build(keys, n)
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


@pytest.mark.gpu
@pytest.mark.parametrize("hashed", [False, True])
def test_gpu_host_build_into_pinned_slots(gpu, orc, hashed):
    """Host-API builds whose slots are page-locked (the kernels store the
    filter straight into host memory) or pageable / not 16-byte aligned
    (page-locked staging, then a copy), side by side in one batch, with the
    lengths in page-locked memory: one synchronisation per call."""
    import ctypes as C

    import dlsm_amd

    sizes = [153_846, 0, 77, 40_000]
    keys = [orc.dbbench_keys(s + 3, 11, n) for s, n in enumerate(sizes)]
    want = [orc.full_build(k, n) for k, n in zip(keys, sizes)]
    pins = [dlsm_amd.PinnedArray(dlsm_amd.full_size(n)[0] + 64) for n in sizes]
    try:
        if hashed:
            hs = [bloom_hash_k20(k) if n else np.zeros(1, np.uint32) for k, n in zip(keys, sizes)]
            tabs = [dlsm_amd.Keys(h, n, 4) for h, n in zip(hs, sizes)]
            fn = dlsm_amd.lib().dlsm_bloom_full_build_hashed
        else:
            tabs = [dlsm_amd.Keys(k if n else np.zeros(20, np.uint8), n, 20) for k, n in zip(keys, sizes)]
            fn = dlsm_amd.lib().dlsm_bloom_full_build
        for layout in range(2):
            if layout == 0:  # aligned pinned, pageable, unaligned pinned, aligned pinned
                outs = [pins[0].array, np.zeros(len(want[1]) + 16, np.uint8), pins[2].array[4:], pins[3].array]
            else:  # the other way round
                outs = [pins[0].array[4:], pins[1].array, np.zeros(len(want[2]) + 16, np.uint8), pins[3].array[8:]]
            for o in outs:
                o[:] = 0xA5
            jobs = gpu._jobs(tabs, outs, [len(w) for w in want])
            lens = (C.c_uint64 * len(sizes))()
            dlsm_amd.check(fn(gpu.h, jobs, len(sizes), 10, lens), "full_build")
            for o, w, ln in zip(outs, want, lens):
                assert ln == len(w) and o[:ln].tobytes() == w, layout
                assert np.all(o[ln:ln + 4] == 0xA5), layout  # nothing written past the filter
    finally:
        for p in pins:
            p.close()
