"""GPU parity of the workspace / scheduling corners of the C ABI: the job-table
upload cache across dlsm_ctx_reserve, the exact (count-first) build for
batches whose duplicate user keys lower the line count, and probe masks that
start at any byte.  Everything is compared with the oracle byte for byte."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _dev_tables(orc, n, T, first=0):
    import torch

    import dlsm_amd

    tabs, want = [], []
    for s in range(T):
        k = orc.dbbench_keys(first + s, T, n)
        want.append(orc.full_build(k, n))
        tabs.append(dlsm_amd.Keys(torch.from_numpy(k).cuda(), n, 20))
    return tabs, want


def test_reserve_between_identical_builds(gpu, orc):
    """build A; reserve(bigger) reallocates the job table; build A again must
    re-upload it (the cache compared host vectors only)."""
    import torch

    import dlsm_amd

    n, T = 20_000, 3
    tabs, want = _dev_tables(orc, n, T)
    outs = [torch.zeros(dlsm_amd.full_size(n)[0] + 16, dtype=torch.uint8, device="cuda") for _ in range(T)]
    lens = torch.zeros(T, dtype=torch.uint64, device="cuda")
    for rep in range(3):
        for o in outs:
            o.fill_(0xAB)
        torch.cuda.synchronize()  # torch's stream vs the context's own stream
        gpu.full_build_dev(tabs, outs, lens, 10)
        gpu.sync()
        L = lens.cpu().numpy()
        for s in range(T):
            assert outs[s][: int(L[s])].cpu().numpy().tobytes() == want[s], (rep, s)
        gpu.reserve(1_000_000 * (rep + 2), 64 * (rep + 2))  # grows jobs / starts every time


def _dup_batch(orc, n, every=3):
    v = np.arange(n, dtype=np.uint64)
    v[1::every] = v[0::every][: v[1::every].size]
    return orc.keys_from_values(v)


@pytest.mark.parametrize("exact", [0, 1, 2])
def test_build_duplicates_exact_modes(gpu, orc, exact):
    """Duplicates that lower L, through every DLSM_OPT_BUILD_EXACT mode, for
    user keys (K20) and internal keys (K28 + suffix 8) and offsets."""
    import dlsm_amd

    n = 300_000
    keys = _dup_batch(orc, n)
    want = orc.full_build(keys, n)
    assert len(want) < dlsm_amd.full_size(n)[0]
    # internal keys: user key || Fixed64(seq << 8 | type)
    ik = np.zeros((n, 28), np.uint8)
    ik[:, :20] = keys.reshape(n, 20)
    ik[:, 20:] = np.frombuffer(((np.arange(n, dtype=np.uint64) << 8) | 1).tobytes(), np.uint8).reshape(n, 8)
    offs = np.arange(n + 1, dtype=np.uint64) * 20
    gpu.set_build_exact(exact)
    try:
        got20 = gpu.full_build([dlsm_amd.Keys(keys, n, 20)], 10)[0]
        got28 = gpu.full_build([dlsm_amd.Keys(ik.reshape(-1), n, 28, None, 8)], 10)[0]
        gotv = gpu.full_build([dlsm_amd.Keys(np.concatenate([keys, np.zeros(16, np.uint8)]), n, 0, offs)], 10)[0]
    finally:
        gpu.set_build_exact(0)
    assert got20 == want and got28 == want and gotv == want


def test_build_multiversion_internal_batch(gpu, orc):
    """A compaction-shaped batch: 3 versions per user key (newest first), 16
    tables in one device call, exact mode chosen automatically."""
    import torch

    import dlsm_amd

    n_user, ver, T = 50_000, 3, 16
    tabs, outs, want = [], [], []
    for s in range(T):
        uk = orc.dbbench_keys(s, T, n_user).reshape(n_user, 20)
        ik = np.zeros((n_user, ver, 28), np.uint8)
        ik[:, :, :20] = uk[:, None, :]
        seq = (np.arange(n_user * ver, dtype=np.uint64)[::-1].reshape(n_user, ver) << 8) | 1
        ik[:, :, 20:] = np.frombuffer(seq.tobytes(), np.uint8).reshape(n_user, ver, 8)
        flat = ik.reshape(-1)
        n = n_user * ver
        want.append(orc.full_build(np.repeat(uk, ver, axis=0).reshape(-1), n))
        tabs.append(dlsm_amd.Keys(torch.from_numpy(flat).cuda(), n, 28, None, 8))
        outs.append(torch.zeros(dlsm_amd.full_size(n)[0], dtype=torch.uint8, device="cuda"))
    lens = torch.zeros(T, dtype=torch.uint64, device="cuda")
    torch.cuda.synchronize()
    gpu.full_build_dev(tabs, outs, lens, 10)
    gpu.sync()
    L = lens.cpu().numpy()
    for s in range(T):
        assert int(L[s]) == len(want[s]) < dlsm_amd.full_size(n_user * ver)[0]
        assert outs[s][: int(L[s])].cpu().numpy().tobytes() == want[s], s


@pytest.mark.parametrize("off", [1, 3, 5, 7])
def test_probe_mask_at_any_byte(gpu, orc, off):
    """The sliced probe's 8-byte answer stores fall back to byte stores when the
    caller's mask starts at an odd address."""
    import torch

    import dlsm_amd

    n = 100_000
    filters = [orc.full_build(orc.dbbench_keys(f, 4, n), n) for f in range(4)]
    q = orc.keys_from_values(orc.mt_values(7 + off, 8 * n, 70_001))
    want = orc.full_probe(filters, q, 70_001)
    fs = gpu.filterset(filters)
    buf = torch.full((70_001 + 16,), 0x5A, dtype=torch.uint8, device="cuda")
    qd = torch.from_numpy(q).cuda()
    torch.cuda.synchronize()
    gpu.set_path(2)
    try:
        gpu.full_probe_dev(fs, dlsm_amd.Keys(qd, 70_001, 20), buf[off:])
        gpu.sync()
    finally:
        gpu.set_path(0)
    got = buf.cpu().numpy()
    assert np.array_equal(got[off:off + 70_001], want)
    assert (got[:off] == 0x5A).all() and (got[off + 70_001:] == 0x5A).all()
    fs.close()
