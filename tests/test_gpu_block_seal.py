"""Sealed filter blocks with the crc32c fused into the build's slice pass
(round 6; bloom_kernels.hip crc_slice_partial / full_block_seal_kernel):
`[filter][type 0][crc32c::Mask(crc32c::Value(filter || type))]`
(table/table_builder_computeside.cc:418-428, util/crc32c.h:17-37), compared
with the oracle (filter bytes + the reference crc32c.cc restated in
oracle/bloom_oracle.c, pinned by tests/golden) and with the direct path,
whose blocks take the separate crc passes (block_crc.hip).

Covers batches whose slices are 2^7 .. 2^11 lines (choose_build_lgR), single
short slices (front zero padding of the crc), filters whose last slice is
short, a duplicate-lowered line count (slices past the new L hold no
bytes), bits_per_key other than 10, internal keys, and a failed job beside
sealed ones."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _blocks(gpu, tables, caps, bpk, path):
    import torch

    import dlsm_amd

    outs = [torch.full((c,), 0xEE, dtype=torch.uint8, device="cuda") for c in caps]
    lens = torch.zeros(len(tables), dtype=torch.uint64, device="cuda")
    gpu.set_path(path)
    try:
        gpu.full_build_block_dev(tables, outs, lens, bpk)
        gpu.sync()
    finally:
        gpu.set_path(0)
    L = lens.cpu().numpy()
    return [o.cpu().numpy()[: int(n)].tobytes() for o, n in zip(outs, L)], [o.cpu().numpy() for o in outs], L


def _check(gpu, orc, keysets, bpk=10, extra=64):
    import torch

    import dlsm_amd

    tables, want, caps = [], [], []
    for k, n, stride in keysets:
        filt = orc.full_build(k, n, stride=stride, bpk=bpk)
        want.append(orc.filter_block(filt))
        tables.append(dlsm_amd.Keys(torch.from_numpy(k).cuda(), n, stride,
                                    suffix_len=8 if stride == 28 else 0))
        caps.append(dlsm_amd.full_size(n, bpk)[0] + 5 + extra)
    for path in (0, 2, 1):  # auto, sliced (fused seal), direct (separate crc passes)
        got, raw, L = _blocks(gpu, tables, caps, bpk, path)
        for j, w in enumerate(want):
            assert got[j] == w, (path, j, len(got[j]), len(w))
            assert (raw[j][len(w):] == 0xEE).all(), (path, j)  # nothing written past the block


@pytest.mark.parametrize("n", [0, 1, 7, 5_000, 20_000, 153_846])
def test_single_filter_sizes(gpu, orc, n):
    k = orc.dbbench_keys(3, 5, n) if n else np.zeros(20, np.uint8)
    _check(gpu, orc, [(k, n, 20)])


def test_empty_filters_beside_full_ones(gpu, orc):
    z = np.zeros(20, np.uint8)
    _check(gpu, orc, [(z, 0, 20), (orc.dbbench_keys(1, 2, 70_000), 70_000, 20), (z, 0, 20)])


def test_bench_batch_and_mixed_sizes(gpu, orc):
    sizes = [1_600_000] * 4 + [153_846, 600_000, 31, 2_000_001, 99_999]
    _check(gpu, orc, [(orc.dbbench_keys(f, 16, n), n, 20) for f, n in enumerate(sizes)])


@pytest.mark.parametrize("bpk", [1, 5, 16, 23])
def test_bits_per_key(gpu, orc, bpk):
    sizes = [50_000, 333_333, 1_000_000]
    _check(gpu, orc, [(orc.dbbench_keys(f, 3, n), n, 20) for f, n in enumerate(sizes)], bpk=bpk)


def test_duplicates_lower_line_count(gpu, orc):
    # every key twice in a row: AddKey's dedup halves the line count, so the
    # slices past the new L carry no bytes
    n = 400_000
    k = orc.dbbench_keys(0, 1, n // 2).reshape(-1, 20)
    k = np.repeat(k, 2, axis=0).reshape(-1)
    _check(gpu, orc, [(k, n, 20), (orc.dbbench_keys(9, 2, 300_000), 300_000, 20)])


def test_internal_keys(gpu, orc):
    n = 250_000
    uk = orc.dbbench_keys(0, 1, n).reshape(n, 20)
    ik = np.concatenate([uk, np.full((n, 8), 0x11, dtype=np.uint8)], axis=1).reshape(-1)
    # the oracle hashes ExtractUserKey: build its filter from the user keys
    import torch

    import dlsm_amd

    want = orc.filter_block(orc.full_build(uk.reshape(-1), n))
    cap = dlsm_amd.full_size(n)[0] + 5 + 64
    for path in (0, 1):
        got, raw, L = _blocks(gpu, [dlsm_amd.Keys(torch.from_numpy(ik).cuda(), n, 28, suffix_len=8)], [cap], 10,
                              path)
        assert got[0] == want, path


def test_failed_job_beside_sealed_ones(gpu, orc):
    import torch

    import dlsm_amd

    sizes = [100_000, 200_000, 50_000]
    tables = [dlsm_amd.Keys(torch.from_numpy(orc.dbbench_keys(f, 3, n)).cuda(), n, 20) for f, n in enumerate(sizes)]
    caps = [dlsm_amd.full_size(n)[0] + 5 for n in sizes]
    caps[1] -= 1  # one byte short of the sealed block
    for path in (0, 1):
        got, raw, L = _blocks(gpu, tables, caps, 10, path)
        assert int(L[1]) == 0, path  # the device entry point reports the failed job by length 0
        for j in (0, 2):
            w = orc.filter_block(orc.full_build(orc.dbbench_keys(j, 3, sizes[j]), sizes[j]))
            assert got[j] == w, (path, j)
