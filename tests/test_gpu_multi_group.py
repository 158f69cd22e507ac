"""One-pass probe of a multi-group filter set (round 6; bloom_internal.h
MGroupDev, probe_mpartition_kernel / probe_slice_kernel<..., MG> /
probe_munpermute_kernel): the filters Version::Get walks differ in line count
(db/version_set.cc:273-321; flush outputs whose dedup shifts L,
full_filter_block.cc:95-96), so the set splits into (L, k) groups, and one
partition pass buckets every lookup by every group's slice.

Every case is compared with the oracle (oracle/bloom_oracle.c, the CPU
restatement of FullFilterBlockReader::KeyMayMatch) and with the per-group
passes (DLSM_OPT_PROBE_MULTI = 0):

* the bench's realistic shapes: mixed sizes (4 packed pairs), dedup-shifted
  (8 groups of one), L0 + levels (16 filters, 2 mask bytes, byte-wide and
  packed groups in one set);
* 9..16 groups (the 2,048-key chunk), more than 16 groups (falls back to the
  per-group passes), 3 mask bytes, a k != 6 set (bits_per_key 16);
* ragged batches (1, 7, 8, 4,095 .. 8,193 lookups), an unaligned mask, hashed
  lookups, internal keys (ExtractUserKey) and variable-length keys."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

OPT_PROBE_MULTI = 10  # dlsm_amd.OPT_PROBE_MULTI


def _filters(orc, sizes, bpk=10):
    F = len(sizes)
    return [orc.full_build(orc.dbbench_keys(f, F, n), n, bpk=bpk) for f, n in enumerate(sizes)]


def _probe(gpu, fs, keys, nq, multi, offset=0, fill=0xEE):
    import torch

    mb = fs.mask_bytes
    buf = torch.full((nq * mb + offset + 16,), fill, dtype=torch.uint8, device="cuda")
    mask = buf[offset: offset + nq * mb]
    gpu.set_option(OPT_PROBE_MULTI, 1 if multi else 0)
    try:
        gpu.full_probe_dev(fs, keys, mask)
        gpu.sync()
    finally:
        gpu.set_option(OPT_PROBE_MULTI, 1)
    out = buf.cpu().numpy()
    # nothing written before or past the batch's mask bytes
    assert (out[:offset] == fill).all() and (out[offset + nq * mb:] == fill).all()
    return out[offset: offset + nq * mb]


def _check(gpu, orc, filters, nq, seed, check=None, offset=0):
    import torch

    import dlsm_amd

    span = 2 * len(filters) * 3_000_000
    q = orc.keys_from_values(orc.mt_values(seed, span, nq))
    fs = gpu.filterset(filters)
    try:
        keys = dlsm_amd.Keys(torch.from_numpy(q).cuda(), nq, 20)
        one = _probe(gpu, fs, keys, nq, True, offset)
        per = _probe(gpu, fs, keys, nq, False, offset)
        assert np.array_equal(one, per)
        nc = nq if check is None else min(check, nq)
        want = orc.full_probe(filters, q[: nc * 20], nc, nthreads=8)
        assert np.array_equal(one[: nc * fs.mask_bytes], want)
        return one
    finally:
        fs.close()


SHAPES = {
    "mixed_8": [153_846, 153_846, 600_000, 600_000, 1_600_000, 1_600_000, 3_000_000, 3_000_000],
    "dedup_shifted_8": [1_600_000 - 97 * f for f in range(8)],
    "l0_plus_levels_16": [153_846] * 10 + [600_000, 1_600_000, 3_000_000, 153_846 * 4, 153_846 * 40, 2_000_000],
}


@pytest.mark.parametrize("shape", list(SHAPES))
def test_bench_shapes(gpu, orc, shape):
    _check(gpu, orc, _filters(orc, SHAPES[shape]), 2_000_003, 11, check=1_000_000)


def test_twelve_groups_small_chunks(gpu, orc):
    # 12 distinct line counts: 9..16 groups take 2,048-key chunks
    sizes = [40_000 + 9_000 * f for f in range(12)]
    _check(gpu, orc, _filters(orc, sizes), 700_001, 12)


def test_sixteen_groups_three_mask_bytes(gpu, orc):
    # 24 filters: 3 mask bytes; 16 groups (8 singles, 4 pairs, one of 4... by size)
    base = [50_000, 70_000, 90_000, 110_000, 130_000, 150_000, 170_000, 190_000]
    sizes = base + [210_000, 210_000, 230_000, 230_000, 250_000, 250_000, 270_000, 270_000] + [290_000] * 4 + [310_000] * 4
    filters = _filters(orc, sizes)
    _check(gpu, orc, filters, 500_003, 13)


def test_more_than_sixteen_groups_falls_back(gpu, orc):
    sizes = [30_000 + 5_000 * f for f in range(20)]
    _check(gpu, orc, _filters(orc, sizes), 300_007, 14)


def test_k_not_six(gpu, orc):
    # bits_per_key 16 -> k = 11 (ChooseNumProbes): the slice pass's run-time k
    sizes = [100_000, 250_000, 250_000, 400_000, 777_777]
    _check(gpu, orc, _filters(orc, sizes, bpk=16), 600_001, 15)


def test_one_filter_per_size_with_tiny_filters(gpu, orc):
    # a 7-key filter (one line) and a 1-key filter next to large ones
    sizes = [7, 1, 153_846, 1_600_000, 600_000]
    _check(gpu, orc, _filters(orc, sizes), 400_009, 16)


@pytest.mark.parametrize("nq", [1, 7, 8, 9, 2047, 2048, 2049, 4095, 4096, 4097, 8193])
def test_ragged_batches(gpu, orc, nq):
    _check(gpu, orc, _filters(orc, [20_000, 35_000, 35_000, 60_000]), nq, 100 + nq)


def test_ragged_batches_two_mask_bytes_small_chunks(gpu, orc):
    sizes = [10_000 + 3_000 * f for f in range(10)]
    filters = _filters(orc, sizes)
    for nq in (1, 5, 2047, 2049, 6001):
        _check(gpu, orc, filters, nq, 200 + nq)


@pytest.mark.parametrize("offset", [1, 3, 8])
def test_unaligned_mask(gpu, orc, offset):
    _check(gpu, orc, _filters(orc, SHAPES["mixed_8"]), 100_003, 17, offset=offset)
    _check(gpu, orc, _filters(orc, [20_000 + 1_000 * f for f in range(10)]), 50_001, 18, offset=offset)


def test_hashed_lookups(gpu, orc):
    import torch

    import dlsm_amd

    filters = _filters(orc, SHAPES["dedup_shifted_8"])
    nq = 1_000_003
    q = orc.keys_from_values(orc.mt_values(19, 16 * 1_600_000, nq))
    h = torch.from_numpy(dlsm_amd.hash_batch(dlsm_amd.Keys(q, nq, 20)).view(np.int32).copy()).cuda()
    fs = gpu.filterset(filters)
    try:
        m = torch.full((nq,), 0x5A, dtype=torch.uint8, device="cuda")
        gpu.full_probe_hashed_dev(fs, h, m, nq)
        gpu.sync()
        assert np.array_equal(m.cpu().numpy(), orc.full_probe(filters, q, nq, nthreads=8))
    finally:
        fs.close()


def test_internal_keys(gpu, orc):
    import torch

    import dlsm_amd

    filters = _filters(orc, SHAPES["mixed_8"])
    nq = 500_001
    q = orc.keys_from_values(orc.mt_values(20, 16 * 3_000_000, nq))
    ik = np.concatenate([q.reshape(nq, 20), np.full((nq, 8), 0x37, dtype=np.uint8)], axis=1).reshape(-1)
    fs = gpu.filterset(filters)
    try:
        m = torch.full((nq,), 0x5A, dtype=torch.uint8, device="cuda")
        keys = dlsm_amd.Keys(torch.from_numpy(ik).cuda(), nq, 28, suffix_len=dlsm_amd.INTERNAL_KEY_TRAILER)
        gpu.full_probe_dev(fs, keys, m)
        gpu.sync()
        assert np.array_equal(m.cpu().numpy(), orc.full_probe(filters, q, nq, nthreads=8))
    finally:
        fs.close()


def test_variable_length_keys(gpu, orc):
    import dlsm_amd

    filters = _filters(orc, SHAPES["mixed_8"])
    rng = np.random.default_rng(21)
    nq = 200_003
    keys = [bytes(rng.integers(0, 256, size=int(rng.integers(0, 40)), dtype=np.uint8)) for _ in range(nq)]
    # some lookups that are real members of the filters
    for i in range(0, nq, 97):
        keys[i] = orc.dbbench_keys(i % 8 + 8 * (i % 1000), 8, 1).tobytes()
    data, offs = orc.pack_var(keys)
    want = orc.full_probe(filters, data, nq, stride=0, offsets=offs)
    fs = gpu.filterset(filters)
    try:
        got = gpu.full_probe(fs, dlsm_amd.Keys(np.concatenate([data, np.zeros(16, np.uint8)]), nq, 0, offs))
        assert np.array_equal(got, want)
        assert want[::97].any()
    finally:
        fs.close()


def test_group_with_256_slices(gpu, orc):
    # 8 filters of 3.35 M keys: one byte-wide group of 65,430 lines = 256
    # slices of 256 lines (the most a group may have), beside a packed single
    sizes = [3_350_000] * 8 + [100_000]
    _check(gpu, orc, _filters(orc, sizes), 400_001, 22)


@pytest.mark.parametrize("serial", [False, True])
def test_rounds(gpu, orc, serial):
    """DLSM_OPT_PROBE_ROUND_KEYS: the batch in rounds (the last one ragged),
    pipelined over two streams or one after another; 20-byte, hashed and
    variable-length lookups, against the oracle."""
    import torch

    import dlsm_amd

    filters = _filters(orc, SHAPES["mixed_8"])
    gpu.set_probe_round(300_000)
    gpu.set_probe_serial(serial)
    try:
        _check(gpu, orc, filters, 1_000_003, 23)
        nq = 700_001
        q = orc.keys_from_values(orc.mt_values(24, 16 * 3_000_000, nq))
        want = orc.full_probe(filters, q, nq, nthreads=8)
        h = torch.from_numpy(dlsm_amd.hash_batch(dlsm_amd.Keys(q, nq, 20)).view(np.int32).copy()).cuda()
        fs = gpu.filterset(filters)
        try:
            m = torch.full((nq,), 0x5A, dtype=torch.uint8, device="cuda")
            gpu.full_probe_hashed_dev(fs, h, m, nq)
            gpu.sync()
            assert np.array_equal(m.cpu().numpy(), want)
            rng = np.random.default_rng(25)
            keys = [bytes(rng.integers(0, 256, size=int(rng.integers(0, 40)), dtype=np.uint8))
                    for _ in range(400_001)]
            data, offs = orc.pack_var(keys)
            got = gpu.full_probe(fs, dlsm_amd.Keys(np.concatenate([data, np.zeros(16, np.uint8)]), len(keys), 0,
                                                   offs))
            assert np.array_equal(got, orc.full_probe(filters, data, len(keys), stride=0, offsets=offs))
        finally:
            fs.close()
    finally:
        gpu.set_probe_round(0)
        gpu.set_probe_serial(False)
