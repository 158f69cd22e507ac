"""Internal keys: ExtractUserKey stripping in build /
probe, and the flush / compaction selection + user-key gather on the GPU.

The oracle (``orc_internal_keys_select``) restates the two reference loops
statement by statement -- db/memtable_list.cc:855-886 (FlushJob::BuildTable)
and db/db_impl.cc:3500-3562 (DoCompactionWork) -- as a sequential state
machine; the GPU decides every key from its predecessor in one parallel pass.
The reference loops cannot run here (they need the RDMA Env), so the CPU
cases below are hand-derived from those lines; parity for this row is
anchored on them and on the oracle ("parity unpinned" by reference outputs).
"""
import numpy as np
import pytest

import oracle

IK = oracle.internal_key


def pack(keys):
    return np.frombuffer(b"".join(keys) + b"\0" * 16, dtype=np.uint8).copy()


def pack_var(keys):
    offs = np.zeros(len(keys) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(k) for k in keys])
    return pack(keys), offs


U = lambda c: bytes([c]) * 20  # noqa: E731


# (internal keys, policy, snapshot, expected keep, expected n_kept, first_corrupt)
CASES = [
    # flush keeps the newest entry of each user key (iterator order: seq descending)
    ([IK(U(1), 9), IK(U(1), 7), IK(U(1), 2), IK(U(2), 5), IK(U(3), 4), IK(U(3), 1, 0)],
     0, 0, [1, 0, 0, 1, 1, 0], 3, None),
    # compaction rule (A): an entry is dropped when the previous entry of its
    # user key has sequence <= smallest_snapshot
    ([IK(U(1), 9), IK(U(1), 7), IK(U(1), 2), IK(U(2), 5)], 1, 9, [1, 0, 0, 1], 2, None),
    ([IK(U(1), 9), IK(U(1), 7), IK(U(1), 2), IK(U(2), 5)], 1, 8, [1, 1, 0, 1], 3, None),
    ([IK(U(1), 9), IK(U(1), 7), IK(U(1), 2), IK(U(2), 5)], 1, 7, [1, 1, 0, 1], 3, None),
    ([IK(U(1), 9), IK(U(1), 7), IK(U(1), 2), IK(U(2), 5)], 1, 6, [1, 1, 1, 1], 4, None),
    # deletion markers (type 0) parse fine and follow the same rule
    ([IK(U(4), 9, 0), IK(U(4), 3, 1)], 1, 100, [1, 0], 1, None),
    # a corrupt key (type 2) is kept by a compaction and restarts the user key
    ([IK(U(1), 9), IK(U(1), 8, 2), IK(U(1), 7), IK(U(1), 6)], 1, 100, [1, 1, 1, 0], 3, 1),
    # ... and aborts a flush
    ([IK(U(1), 9), IK(U(1), 8, 2), IK(U(2), 7)], 0, 0, None, -1, 1),
    # same user-key bytes, different length: different user keys
    ([IK(b"ab", 5), IK(b"abc", 5)], 0, 0, [1, 1], 2, None),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_oracle_select_cases(case):
    keys, policy, snap, want_keep, want_n, want_bad = CASES[case]
    data, offs = pack_var(keys)
    keep, n, bad = oracle.internal_keys_select(data, len(keys), policy, snap, offsets=offs)
    assert n == want_n
    assert (bad if bad != 2**64 - 1 else None) == want_bad
    if want_keep is not None:
        assert keep.tolist() == want_keep


def test_oracle_short_key_is_corrupt():
    data, offs = pack_var([IK(U(1), 3), b"\x01\x02\x03", IK(U(1), 2)])
    keep, n, bad = oracle.internal_keys_select(data, 3, 1, 100, offsets=offs)
    assert bad == 1 and keep.tolist() == [1, 1, 1]


def memtable_stream(seed, n_users, max_versions, corrupt_frac=0.0, ulen=20):
    """Sorted internal keys the way a memtable iterator yields them: user keys
    ascending, versions of one user key by descending sequence."""
    rng = np.random.default_rng(seed)
    users = sorted(set(int(x) for x in rng.integers(0, 1 << 40, n_users)))
    out, seq = [], 1 << 30
    for u in users:
        uk = u.to_bytes(8, "big") + b"0" * (ulen - 8)
        for _ in range(int(rng.integers(1, max_versions + 1))):
            vtype = int(rng.integers(0, 2))
            if corrupt_frac and rng.random() < corrupt_frac:
                vtype = int(rng.integers(2, 256))
            out.append(IK(uk, seq, vtype))
            seq -= int(rng.integers(1, 5))
    return out


def test_oracle_filter_invariant_under_selection():
    """The full filter of the kept user keys equals the full filter of every
    key's ExtractUserKey: each dropped entry repeats the previous entry's user
    key, which AddKey's consecutive dedup (full_filter_block.cc:45-48) drops."""
    keys = memtable_stream(5, 3000, 4, corrupt_frac=0.01)
    data = pack(keys)
    n = len(keys)
    users = np.frombuffer(b"".join(k[:-8] for k in keys), dtype=np.uint8).copy()
    all_filter = oracle.full_build(users, n, 20)
    for policy, snap in ((1, 0), (1, 1 << 29), (1, 1 << 31)):
        keep, nk, _ = oracle.internal_keys_select(data, n, policy, snap, stride=28)
        kept = np.frombuffer(b"".join(k[:-8] for k, f in zip(keys, keep) if f), dtype=np.uint8).copy()
        assert oracle.full_build(kept, nk, 20) == all_filter


# ---------------------------------------------------------------------------
# GPU: select / gather / build / probe with suffix_len = 8, against the oracle
# ---------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("policy,snap", [(0, 0), (1, 0), (1, 1 << 29), (1, 1 << 31)])
@pytest.mark.parametrize("var", [False, True])
def test_gpu_select_and_gather(gpu, policy, snap, var):
    import torch

    import dlsm_amd

    keys = memtable_stream(11 + policy, 40_000, 5, corrupt_frac=0.0 if policy == 0 else 0.002)
    if var:  # variable-length user keys 0..30 bytes (plus the trailer)
        rng = np.random.default_rng(3)
        keys = [k[: int(rng.integers(0, 21))] + k[-8:] for k in keys]
    n = len(keys)
    if var:
        data, offs = pack_var(keys)
        ks = dlsm_amd.Keys(torch.from_numpy(data).cuda(), n, 0, torch.from_numpy(offs).cuda())
        want_keep, want_n, want_bad = oracle.internal_keys_select(data, n, policy, snap, offsets=offs)
    else:
        data = pack(keys)
        ks = dlsm_amd.Keys(torch.from_numpy(data).cuda(), n, 28)
        want_keep, want_n, want_bad = oracle.internal_keys_select(data, n, policy, snap, stride=28)
    keep = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    nk, nbytes, bad = gpu.internal_keys_select_dev(ks, policy, snap, keep)
    assert nk == want_n
    assert (bad if bad is not None else 2**64 - 1) == want_bad
    if policy == 1:
        assert bad is not None  # the stream carries corrupt keys
    assert np.array_equal(keep.cpu().numpy(), want_keep)
    kept = [k[:-8] for k, f in zip(keys, want_keep) if f]
    assert nbytes == sum(len(k) for k in kept)
    out = torch.full((nbytes + 16,), 0xEE, dtype=torch.uint8, device="cuda")
    offs_out = torch.zeros(nk + 1, dtype=torch.uint64, device="cuda") if var else None
    gpu.user_keys_gather_dev(ks, keep, out, offs_out)
    gpu.sync()
    assert out[:nbytes].cpu().numpy().tobytes() == b"".join(kept)
    if var:
        want_offs = np.concatenate([[0], np.cumsum([len(k) for k in kept])]).astype(np.uint64)
        assert np.array_equal(offs_out.cpu().numpy(), want_offs)


@pytest.mark.gpu
def test_gpu_flush_select_reports_corrupt_key(gpu):
    import torch

    import dlsm_amd

    keys = [IK(U(1), 9), IK(U(1), 8), IK(U(2), 7, 5), IK(U(3), 6)]
    data = pack(keys)
    ks = dlsm_amd.Keys(torch.from_numpy(data).cuda(), 4, 28)
    keep = torch.zeros(4, dtype=torch.uint8, device="cuda")
    with pytest.raises(dlsm_amd.DlsmError):
        gpu.internal_keys_select_dev(ks, dlsm_amd.SELECT_FLUSH, 0, keep)
    _, _, bad = gpu.internal_keys_select_dev(ks, dlsm_amd.SELECT_COMPACTION, 0, keep)
    assert bad == 2
    assert keep.cpu().numpy().tolist() == [1, 1, 1, 1]  # 2 restarts the user key, 3 is new


@pytest.mark.gpu
@pytest.mark.parametrize("var", [False, True])
def test_gpu_build_probe_internal_keys(gpu, var):
    """suffix_len = 8: build and probe hash ExtractUserKey(key); the filter
    equals the oracle's over the stripped user keys (and over the kept ones)."""
    import torch

    import dlsm_amd

    keys = memtable_stream(21, 60_000, 3)
    if var:
        rng = np.random.default_rng(4)
        keys = [k[: int(rng.integers(8, 21))] + k[-8:] for k in keys]
    n = len(keys)
    users = [k[:-8] for k in keys]
    udata, uoffs = pack_var(users)
    want = oracle.full_build(udata, n, 0, offsets=uoffs)
    if var:
        data, offs = pack_var(keys)
        ks = dlsm_amd.Keys(data, n, 0, offs, suffix_len=dlsm_amd.INTERNAL_KEY_TRAILER)
        dks = dlsm_amd.Keys(torch.from_numpy(data).cuda(), n, 0, torch.from_numpy(offs).cuda(),
                            suffix_len=8)
    else:
        data = pack(keys)
        ks = dlsm_amd.Keys(data, n, 28, suffix_len=8)
        dks = dlsm_amd.Keys(torch.from_numpy(data).cuda(), n, 28, suffix_len=8)
    assert gpu.full_build([ks], 10)[0] == want
    assert gpu.legacy_build([ks], 10)[0] == oracle.legacy_build(udata, n, 0, offsets=uoffs)
    fs = gpu.filterset([want])
    mask = torch.zeros(n, dtype=torch.uint8, device="cuda")
    gpu.full_probe_dev(fs, dks, mask)
    gpu.sync()
    assert np.array_equal(mask.cpu().numpy(), oracle.full_probe([want], udata, n, 0, offsets=uoffs))
    fs.close()


@pytest.mark.gpu
def test_gpu_rejects_fixed_keys_shorter_than_suffix(gpu):
    import dlsm_amd

    with pytest.raises(dlsm_amd.DlsmError):
        gpu.full_build([dlsm_amd.Keys(np.zeros(64, np.uint8), 4, 4, suffix_len=8)], 10)


def _internal28(user20: np.ndarray, n: int, seed: int) -> np.ndarray:
    """Packed 28-byte internal keys: each 20-byte user key + an 8-byte trailer
    (random seq/type bytes: the trailer must never reach the hash)."""
    trl = np.random.default_rng(seed).integers(0, 256, size=(n, 8), dtype=np.uint8)
    return np.ascontiguousarray(np.hstack([user20.reshape(n, 20), trl]).reshape(-1))


@pytest.mark.gpu
def test_gpu_k28_tiled_build_and_probe(gpu):
    """Fixed-stride 28-byte internal keys (suffix_len 8) take the LDS-tiled K28
    partition loaders in the build and the sliced probe: filters and 8-filter
    masks must equal the oracle's over the stripped 20-byte user keys.  Sizes
    cross the build's 4,096-key and the probe's 8,192-key chunk boundaries
    with ragged tails; device (torch) and host (staged) buffers both go in."""
    import torch

    import dlsm_amd

    sizes = [1, 4095, 4097, 8193, 100_003, 153_846]
    users = [oracle.dbbench_keys(s, 7, n) for s, n in enumerate(sizes)]
    ints = [_internal28(u, n, 10 + s) for s, (u, n) in enumerate(zip(users, sizes))]
    want = [oracle.full_build(u, n) for u, n in zip(users, sizes)]
    got = gpu.full_build([dlsm_amd.Keys(d, n, 28, suffix_len=8) for d, n in zip(ints, sizes)], 10)
    assert got == want
    dev = [torch.from_numpy(d).cuda() for d in ints]
    outs = [torch.zeros(len(w) + 64, dtype=torch.uint8, device="cuda") for w in want]
    lens = torch.zeros(len(sizes), dtype=torch.uint64, device="cuda")
    gpu.full_build_dev([dlsm_amd.Keys(d, n, 28, suffix_len=8) for d, n in zip(dev, sizes)], outs, lens, 10)
    gpu.sync()
    for o, w, ln in zip(outs, want, lens.cpu().tolist()):
        assert ln == len(w) and bytes(o[:ln].cpu().numpy()) == w

    # 8 stacked filters of one line count (sliced probe), ~50 % absent lookups
    nf = 60_000
    fkeys = [oracle.dbbench_keys(f, 8, nf) for f in range(8)]
    filters = [oracle.full_build(k, nf) for k in fkeys]
    nq = 8192 * 9 + 1234
    qu = oracle.keys_from_values(oracle.mt_values(7, 16 * nf, nq))
    want_mask = oracle.full_probe(filters, qu, nq, nthreads=4)
    fs = gpu.filterset(filters)
    q28 = _internal28(qu, nq, 99)
    assert np.array_equal(gpu.full_probe(fs, dlsm_amd.Keys(q28, nq, 28, suffix_len=8)), want_mask)
    mask = torch.zeros(nq, dtype=torch.uint8, device="cuda")
    gpu.full_probe_dev(fs, dlsm_amd.Keys(torch.from_numpy(q28).cuda(), nq, 28, suffix_len=8), mask)
    gpu.sync()
    assert np.array_equal(mask.cpu().numpy(), want_mask)
    assert 0.2 < (want_mask != 0).mean() < 0.8
    fs.close()
