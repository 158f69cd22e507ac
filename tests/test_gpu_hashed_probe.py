"""The probe from host-computed BloomHash values
(dlsm_bloom_full_probe_hashed_dev, hashes from dlsm_bloom_hash_batch) equals
the probe from the keys and the oracle: one stacked group (the bench's set),
several groups (mixed filter sizes: the grouped path), and the direct path."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _probe_both(gpu, filters, q, nq, path):
    import torch

    import dlsm_amd

    fs = gpu.filterset(filters)
    try:
        mb = fs.mask_bytes
        qd = torch.from_numpy(q).cuda()
        h = torch.from_numpy(dlsm_amd.hash_batch(dlsm_amd.Keys(q, nq, 20)).view(np.int32).copy()).cuda()
        m1 = torch.zeros(nq * mb, dtype=torch.uint8, device="cuda")
        m2 = torch.full((nq * mb,), 0x5A, dtype=torch.uint8, device="cuda")
        gpu.set_path(path)
        try:
            gpu.full_probe_dev(fs, dlsm_amd.Keys(qd, nq, 20), m1)
            gpu.full_probe_hashed_dev(fs, h, m2, nq)
            gpu.sync()
        finally:
            gpu.set_path(0)
        return m1.cpu().numpy(), m2.cpu().numpy()
    finally:
        fs.close()


@pytest.mark.parametrize("path", [0, 1, 2])
def test_hashed_probe_one_group(gpu, orc, path):
    n, nq = 200_000, 1_000_003
    filters = [orc.full_build(orc.dbbench_keys(f, 8, n), n) for f in range(8)]
    q = orc.keys_from_values(orc.mt_values(1000, 16 * n, nq))
    a, b = _probe_both(gpu, filters, q, nq, path)
    assert np.array_equal(a, b)
    assert np.array_equal(b[:200_000], orc.full_probe(filters, q[: 200_000 * 20], 200_000, nthreads=8))


def test_hashed_probe_mixed_groups(gpu, orc):
    sizes = [153_846, 153_846, 400_000, 60_000, 153_846, 1_000_000, 7, 153_846, 33_333, 250_000]
    filters = [orc.full_build(orc.dbbench_keys(f, 11, n), n) for f, n in enumerate(sizes)]
    nq = 300_001
    q = orc.keys_from_values(orc.mt_values(77, 11 * 1_000_000, nq))
    a, b = _probe_both(gpu, filters, q, nq, 0)
    assert np.array_equal(a, b)
    assert np.array_equal(b.reshape(nq, -1)[:50_000].reshape(-1),
                          orc.full_probe(filters, q[: 50_000 * 20], 50_000, nthreads=8))


@pytest.mark.parametrize("path", [0, 1, 2])
def test_hashed_probe_ragged_sizes(gpu, orc, path):
    """Batches of 1 .. 8,193 hashed lookups (empty, one key, below / at /
    past one 8,192-key partition chunk) on every path: the same answers as
    the probe from the keys and the oracle, nothing written past the batch."""
    import torch

    import dlsm_amd

    n = 100_000
    filters = [orc.full_build(orc.dbbench_keys(f, 8, n), n) for f in range(8)]
    fs = gpu.filterset(filters)
    try:
        for nq in (1, 7, 64, 8_191, 8_192, 8_193):
            q = orc.keys_from_values(orc.mt_values(500 + nq, 16 * n, nq))
            h = torch.from_numpy(dlsm_amd.hash_batch(dlsm_amd.Keys(q, nq, 20)).view(np.int32).copy()).cuda()
            m = torch.full((nq + 64,), 0x5A, dtype=torch.uint8, device="cuda")
            gpu.set_path(path)
            try:
                gpu.full_probe_hashed_dev(fs, h, m, nq)
                gpu.sync()
            finally:
                gpu.set_path(0)
            got = m.cpu().numpy()
            assert np.array_equal(got[:nq], orc.full_probe(filters, q, nq)), (nq, path)
            assert (got[nq:] == 0x5A).all(), (nq, path)
        empty = torch.zeros(1, dtype=torch.int32, device="cuda")
        m0 = torch.full((8,), 0x5A, dtype=torch.uint8, device="cuda")
        gpu.full_probe_hashed_dev(fs, empty, m0, 0)
        gpu.sync()
        assert (m0.cpu().numpy() == 0x5A).all()
    finally:
        fs.close()
