"""MultiGet-style probe of a version's files.

For each lookup key the GPU returns the files Version::Get would visit --
Version::ForEachOverlapping (db/version_set.cc:273-321: level-0 files holding
the key newest first, then per level the file FindFile picks, :95-118) --
whose filter passes the key (Table::InternalGet, table/table.cc:350-358).
The oracle (``orc_version_probe``) restates those lines; the cases below are
hand-derived from them, including the reference's FindFile quirk (right
starts at files.size()-1, so a key past a level's last file still visits that
file when it is >= its smallest key).  Parity unpinned by reference outputs
(Version needs the RDMA Env to run).
"""
import numpy as np
import pytest

import oracle
from dlsm_amd import VersionFile

K = lambda v: oracle.keys_from_values(np.array([v], dtype=np.uint64)).tobytes()  # noqa: E731


def build_filter(values):
    keys = oracle.keys_from_values(np.asarray(values, dtype=np.uint64))
    return oracle.full_build(keys, len(values))


def make_version(seed=0, with_nofilter=True):
    """L0: 4 overlapping files; L1: 8 range-partitioned files; L2: 16; L3 empty;
    L4: 2; L5: 1 file (without a filter when with_nofilter)."""
    rng = np.random.default_rng(seed)
    files = []
    span = 1_000_000
    for j in range(4):  # level 0: overlapping ranges, numbers out of order
        a = int(rng.integers(0, span // 2))
        b = a + int(rng.integers(span // 10, span // 2))
        vals = np.arange(a, b, 7 + j)
        files.append(VersionFile(0, int(rng.integers(100, 200)) * 10 + j, K(vals[0]), K(vals[-1]),
                                 (int(rng.integers(1, 1 << 40)) << 8) | 1, build_filter(vals)))
    for level, nf, step in ((1, 8, 3), (2, 16, 5), (4, 2, 11)):
        edges = np.linspace(0, span, nf + 1).astype(np.int64)
        for q in range(nf):
            vals = np.arange(edges[q] + q % 3, edges[q + 1] - 1, step)
            files.append(VersionFile(level, 1000 + level * 100 + q, K(vals[0]), K(vals[-1]),
                                     (int(rng.integers(1, 1 << 40)) << 8) | 1, build_filter(vals)))
    vals = np.arange(100, span // 2, 13)
    files.append(VersionFile(5, 7, K(vals[0]), K(vals[-1]), (5 << 8) | 1,
                             None if with_nofilter else build_filter(vals)))
    return files


def lookups(n, seed=1):
    rng = np.random.default_rng(seed)
    v = np.concatenate([rng.integers(0, 1_300_000, n - 4), [0, 999_999, 1_000_000, 2_000_000]])
    return oracle.keys_from_values(v.astype(np.uint64))


def test_oracle_hand_cases():
    """Level 1 has files [10..20] and [30..40]; level 0 files [15..35] (#9) and
    [0..50] (#12).  Key 25: both L0 files (newest first: #12, #9), level 1
    picks file 1 ([30..40], largest >= 25) and skips it (25 < 30).  Key 45:
    L0 #12 only; level 1 FindFile returns the last file (the quirk) and it is
    visited (45 >= 30).  Key 5: L0 #12 only; level 1 picks file 0 and skips it
    (5 < 10).  No filters: every candidate passes."""
    t = (1 << 8) | 1
    files = [VersionFile(1, 1, K(10), K(20), t), VersionFile(1, 2, K(30), K(40), t),
             VersionFile(0, 9, K(15), K(35), t), VersionFile(0, 12, K(0), K(50), t)]
    keys = np.frombuffer(K(25) + K(45) + K(5), dtype=np.uint8).copy()
    mask, lf = oracle.version_probe(files, keys, 3, snapshot=100)
    # slots: 0 = L0 #12, 1 = L0 #9, 2 = level 1, 3.. = levels 2..5
    assert mask.tolist() == [0b011, 0b101, 0b001]
    assert lf[:, 0].tolist() == [0xFFFFFFFF, 1, 0xFFFFFFFF]


def test_oracle_findfile_snapshot_tiebreak():
    """Key == a file's largest user key: FindFile compares internal keys; with
    the lookup snapshot below the file's largest sequence the file's largest
    sorts before the lookup key, so FindFile moves on to the next file."""
    files = [VersionFile(1, 1, K(10), K(20), (50 << 8) | 1), VersionFile(1, 2, K(30), K(40), (9 << 8) | 1)]
    keys = np.frombuffer(K(20), dtype=np.uint8).copy()
    _, lf = oracle.version_probe(files, keys, 1, snapshot=60)
    assert lf[0, 0] == 0
    _, lf = oracle.version_probe(files, keys, 1, snapshot=40)
    assert lf[0, 0] == 0xFFFFFFFF  # picks file 1 ([30..40]) and 20 < 30 skips it


def test_oracle_filter_gates_candidates():
    files = make_version(3, with_nofilter=False)
    q = lookups(5000, 4)
    mask, lf = oracle.version_probe(files, q, 5000, snapshot=1 << 45)
    nofilt = [VersionFile(f.level, f.number, f.smallest, f.largest, f.largest_trailer, None) for f in files]
    cand, lf2 = oracle.version_probe(nofilt, q, 5000, snapshot=1 << 45)
    assert np.array_equal(lf, lf2)
    assert np.all((mask & ~cand) == 0)       # the filter only removes candidates
    assert (mask != cand).any() and mask.any()


@pytest.mark.gpu
@pytest.mark.parametrize("snapshot", [1 << 45, 1 << 20])
@pytest.mark.parametrize("on_device", [False, True])
def test_gpu_version_probe(gpu, snapshot, on_device):
    import torch

    import dlsm_amd

    files = make_version(0)
    if on_device:
        files = [VersionFile(f.level, f.number, f.smallest, f.largest, f.largest_trailer,
                             None if f.filter is None else torch.frombuffer(bytearray(f.filter), dtype=torch.uint8).cuda())
                 for f in files]
    n = 200_003
    q = lookups(n, 9)
    want, want_lf = oracle.version_probe(make_version(0), q, n, snapshot)
    v = gpu.version(files, on_device=on_device)
    assert v.n_l0 == 4 and v.n_slots == 9
    mask = torch.zeros(n, dtype=torch.uint64, device="cuda")
    lf = torch.zeros((n, 5), dtype=torch.int32, device="cuda")
    gpu.version_probe_dev(v, dlsm_amd.Keys(torch.from_numpy(q).cuda(), n, 20), snapshot, mask, lf)
    gpu.sync()
    assert np.array_equal(mask.cpu().numpy().view(np.uint64), want)
    assert np.array_equal(lf.cpu().numpy().view(np.uint32), want_lf)
    v.close()


@pytest.mark.gpu
def test_gpu_version_probe_internal_var_keys(gpu):
    """Variable-length internal keys (suffix_len 8) against the same version."""
    import torch

    import dlsm_amd

    files = make_version(2)
    n = 30_000
    q = lookups(n, 5)
    ikeys = [q[20 * i: 20 * i + 20].tobytes() + ((77 << 8) | 1).to_bytes(8, "little") for i in range(n)]
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(k) for k in ikeys])
    data = np.frombuffer(b"".join(ikeys) + b"\0" * 16, dtype=np.uint8).copy()
    want, _ = oracle.version_probe(files, data, n, 1 << 30, offsets=offs, suffix=8)
    v = gpu.version(files)
    mask = torch.zeros(n, dtype=torch.uint64, device="cuda")
    ks = dlsm_amd.Keys(torch.from_numpy(data).cuda(), n, 0, torch.from_numpy(offs).cuda(), suffix_len=8)
    gpu.version_probe_dev(v, ks, 1 << 30, mask)
    gpu.sync()
    assert np.array_equal(mask.cpu().numpy().view(np.uint64), want)
    v.close()


@pytest.mark.gpu
def test_gpu_version_rejects_bad_input(gpu):
    import dlsm_amd

    t = (1 << 8) | 1
    with pytest.raises(dlsm_amd.DlsmError):  # too many level-0 files for 64 slots
        gpu.version([VersionFile(0, j, K(0), K(9), t) for j in range(60)])
    with pytest.raises(dlsm_amd.DlsmError):  # corrupt filter
        gpu.version([VersionFile(1, 1, K(0), K(9), t, b"\x01\x02")])
    with pytest.raises(dlsm_amd.DlsmError):  # level out of range
        gpu.version([VersionFile(6, 1, K(0), K(9), t)])


@pytest.mark.gpu
def test_gpu_version_probe_prefix_ties(gpu):
    """Keys that the 16-byte prefix comparison cannot order on its own: user
    keys sharing their first 16 bytes, keys with embedded and trailing zero
    bytes (b"ab" < b"ab\\0" < b"ab\\0\\0c"), keys shorter than 16 bytes and
    exact boundary hits, as files' smallest / largest keys and as lookups
    (no filters: the candidates alone are compared with the oracle)."""
    import torch

    import dlsm_amd

    t = (1 << 8) | 1
    P = b"0123456789abcdef"  # a shared 16-byte prefix
    bounds = [b"", b"\0", b"ab", b"ab\0", b"ab\0\0c", b"ab\x01", P, P + b"\0", P + b"0", P + b"5",
              P + b"5\0", P + b"9zz", b"0123456789abcdeg", b"\xff" * 3, b"\xff" * 17]
    bounds = sorted(set(bounds))
    files = [VersionFile(0, 3, bounds[2], bounds[9], t), VersionFile(0, 7, bounds[5], bounds[12], t)]
    for q in range(0, len(bounds) - 1, 2):  # level 1: [b_q, b_q+1] ranges, disjoint and ordered
        files.append(VersionFile(1, 100 + q, bounds[q], bounds[q + 1], ((50 + q) << 8) | 1))
    files.append(VersionFile(2, 200, bounds[1], bounds[-2], (9 << 8) | 1))
    probes = set(bounds)
    for b in bounds:
        probes |= {b + b"\0", b[:-1], b + b"\xff"}
    probes = sorted(probes)
    n = len(probes)
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(k) for k in probes])
    data = np.frombuffer(b"".join(probes) + b"\0" * 16, dtype=np.uint8).copy()
    for snap in (1 << 40, 60):
        want, want_lf = oracle.version_probe(files, data, n, snap, offsets=offs)
        v = gpu.version(files)
        mask = torch.zeros(n, dtype=torch.uint64, device="cuda")
        lf = torch.zeros((n, 5), dtype=torch.int32, device="cuda")
        ks = dlsm_amd.Keys(torch.from_numpy(data).cuda(), n, 0, torch.from_numpy(offs).cuda())
        gpu.version_probe_dev(v, ks, snap, mask, lf)
        gpu.sync()
        assert np.array_equal(mask.cpu().numpy().view(np.uint64), want), snap
        assert np.array_equal(lf.cpu().numpy().view(np.uint32), want_lf), snap
        v.close()


@pytest.mark.gpu
@pytest.mark.parametrize("pass_slices", [1024, 3, 1])
def test_gpu_version_probe_sliced(gpu, pass_slices):
    """The sliced version probe (route pass; per sliced level a partition /
    LDS slice / unpermute round) against the oracle: every level with filters
    forced onto it (DLSM_OPT_VERSION_SLICE_BYTES = 1), one level with a
    different probe count left on the direct path, a level with a file
    without a filter, and groups of 1024, 3 or 1 slices per pass (several
    passes per level: answer bits OR-ed across passes before the last one
    folds them into the slot mask).  Level files and masks must equal the
    oracle's and the direct path's."""
    import torch

    import dlsm_amd

    files = make_version(6)
    # level 4's two files at 14 bits/key (k = 9): a level of mixed k stays direct
    rebuilt = []
    for f in files:
        if f.level == 4 and f.number % 2 == 0:
            lo = int.from_bytes(f.smallest[:8], "big")
            hi = int.from_bytes(f.largest[:8], "big")
            vals = np.arange(lo, hi + 1, 11, dtype=np.uint64)
            keys = oracle.keys_from_values(vals)
            f = VersionFile(f.level, f.number, f.smallest, f.largest, f.largest_trailer,
                            oracle.full_build(keys, len(vals), bpk=14))
        rebuilt.append(f)
    files = rebuilt
    n = 300_007
    q = lookups(n, 17)
    snap = 1 << 44
    want, want_lf = oracle.version_probe(files, q, n, snap)
    qk = dlsm_amd.Keys(torch.from_numpy(q).cuda(), n, 20)
    old = gpu.get_option(dlsm_amd.OPT_VERSION_SLICE_BYTES)
    try:
        gpu.set_option(dlsm_amd.OPT_VERSION_SLICE_BYTES, 1)
        gpu.set_option(dlsm_amd.OPT_VERSION_PASS_SLICES, pass_slices)
        v = gpu.version(files)
        for path in (0, 1):  # sliced, then the direct kernel on the same version
            gpu.set_path(path)
            mask = torch.zeros(n, dtype=torch.uint64, device="cuda")
            lf = torch.zeros((n, 5), dtype=torch.int32, device="cuda")
            gpu.version_probe_dev(v, qk, snap, mask, lf)
            gpu.sync()
            assert np.array_equal(mask.cpu().numpy().view(np.uint64), want), (pass_slices, path)
            assert np.array_equal(lf.cpu().numpy().view(np.uint32), want_lf), (pass_slices, path)
        v.close()
    finally:
        gpu.set_path(0)
        gpu.set_option(dlsm_amd.OPT_VERSION_SLICE_BYTES, old)
        gpu.set_option(dlsm_amd.OPT_VERSION_PASS_SLICES, 1024)


@pytest.mark.gpu
def test_gpu_version_probe_sliced_internal_var_keys(gpu):
    """Variable-length internal keys (suffix 8, generic route loader) through
    the sliced probe."""
    import torch

    import dlsm_amd

    files = make_version(8, with_nofilter=False)
    n = 40_000
    q = lookups(n, 3)
    ikeys = [q[20 * i: 20 * i + 20].tobytes()[: 12 + i % 9] + ((77 << 8) | 1).to_bytes(8, "little")
             for i in range(n)]
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(k) for k in ikeys])
    data = np.frombuffer(b"".join(ikeys) + b"\0" * 16, dtype=np.uint8).copy()
    want, want_lf = oracle.version_probe(files, data, n, 1 << 30, offsets=offs, suffix=8)
    old = gpu.get_option(dlsm_amd.OPT_VERSION_SLICE_BYTES)
    try:
        gpu.set_option(dlsm_amd.OPT_VERSION_SLICE_BYTES, 1)
        gpu.set_option(dlsm_amd.OPT_VERSION_PASS_SLICES, 2)
        v = gpu.version(files)
        mask = torch.zeros(n, dtype=torch.uint64, device="cuda")
        lf = torch.zeros((n, 5), dtype=torch.int32, device="cuda")
        ks = dlsm_amd.Keys(torch.from_numpy(data).cuda(), n, 0, torch.from_numpy(offs).cuda(), suffix_len=8)
        gpu.version_probe_dev(v, ks, 1 << 30, mask, lf)
        gpu.sync()
        assert np.array_equal(mask.cpu().numpy().view(np.uint64), want)
        assert np.array_equal(lf.cpu().numpy().view(np.uint32), want_lf)
        v.close()
    finally:
        gpu.set_option(dlsm_amd.OPT_VERSION_SLICE_BYTES, old)
        gpu.set_option(dlsm_amd.OPT_VERSION_PASS_SLICES, 1024)


@pytest.mark.gpu
@pytest.mark.parametrize("l1_files", [600, 900, 2400])
def test_gpu_version_probe_many_files(gpu, l1_files):
    """Versions whose tables do not all fit the LDS beside the wave queues:
    4 + 600 + 60 files (file metadata and bound prefixes in LDS, interval
    records from global memory), 4 + 900 + 60 (the metadata and the sparse
    bound index in LDS) and 4 + 2,400 + 60 (the sparse bound index alone).  Slot masks and picked
    files equal the oracle's, for 20-byte keys and for 28-byte internal keys."""
    import torch

    import dlsm_amd

    rng = np.random.default_rng(9)
    span = 3_000_000
    files = []
    for j in range(4):
        a = int(rng.integers(0, span // 2))
        vals = np.arange(a, a + 400_000, 97 + j)
        files.append(VersionFile(0, 9000 + j, K(vals[0]), K(vals[-1]), (((1 << 40) + j) << 8) | 1,
                                 build_filter(vals)))
    for level, nf, step in ((1, l1_files, 29), (2, 60, 13)):
        edges = np.linspace(0, span, nf + 1).astype(np.int64)
        for q in range(nf):
            vals = np.arange(edges[q] + q % 5, edges[q + 1] - 1, step)
            files.append(VersionFile(level, 1000 * level + q, K(vals[0]), K(vals[-1]),
                                     (int(rng.integers(1, 1 << 40)) << 8) | 1, build_filter(vals)))
    n = 300_000
    v_ = np.concatenate([rng.integers(0, span + span // 10, n - 3), [0, span - 1, 5 * span]]).astype(np.uint64)
    q = oracle.keys_from_values(v_)
    snap = (1 << 56) - 1
    want, want_lf = oracle.version_probe(files, q, n, snapshot=snap)
    v = gpu.version(files)
    mask = torch.zeros(n, dtype=torch.uint64, device="cuda")
    lf = torch.zeros((n, 5), dtype=torch.int32, device="cuda")
    gpu.version_probe_dev(v, dlsm_amd.Keys(torch.from_numpy(q).cuda(), n, 20), snap, mask, lf)
    gpu.sync()
    assert np.array_equal(mask.cpu().numpy().view(np.uint64), want)
    assert np.array_equal(lf.cpu().numpy().view(np.uint32), want_lf)
    # the same lookups as 28-byte internal keys (K28 key mode)
    ik = np.concatenate([q.reshape(n, 20), np.frombuffer(((5 << 8) | 1).to_bytes(8, "little") * n,
                                                         dtype=np.uint8).reshape(n, 8)], axis=1).reshape(-1)
    want28, _ = oracle.version_probe(files, ik, n, snapshot=snap, stride=28, suffix=8)
    assert np.array_equal(want28, want)  # the trailer never changes a user-key comparison
    mask.zero_()
    gpu.version_probe_dev(v, dlsm_amd.Keys(torch.from_numpy(np.ascontiguousarray(ik)).cuda(), n, 28, suffix_len=8),
                          snap, mask)
    gpu.sync()
    assert np.array_equal(mask.cpu().numpy().view(np.uint64), want28)
    v.close()


@pytest.mark.gpu
@pytest.mark.parametrize("nf", [5_000, 20_000, 60_000, 70_000])
def test_gpu_version_probe_more_files_than_task_bits(gpu, nf):
    """Versions past the LDS tables: 5,001 files keep only the sparse bound
    index in LDS (windows of 8 prefixes read from global memory), 20,001 keep
    nothing there, and more than 65,535 files -- a queued probe task names its
    file in 16 bits -- take the lane-per-lookup kernel; their answers equal
    the oracle's like every other version's.  Creating the version stays
    linear in its files (the interval index's FindFile picks are a two-pointer
    sweep per level: a 60,000-file level took seconds when every interval
    re-walked the level)."""
    import time

    import torch

    import dlsm_amd

    files = [VersionFile(1, 10 + q, K(10 * q), K(10 * q + 5), ((q + 1) << 8) | 1,
                         build_filter(np.array([10 * q, 10 * q + 3]))) for q in range(nf)]
    files.append(VersionFile(0, 5, K(0), K(10 * nf), (1 << 40 << 8) | 1, build_filter(np.arange(0, 10 * nf, 7))))
    n = 200_000
    v_ = np.random.default_rng(3).integers(0, 10 * nf + 100, n).astype(np.uint64)
    q = oracle.keys_from_values(v_)
    snap = (1 << 56) - 1
    want, want_lf = oracle.version_probe(files, q, n, snapshot=snap)
    t0 = time.perf_counter()
    v = gpu.version(files)
    t_create = time.perf_counter() - t0
    mask = torch.zeros(n, dtype=torch.uint64, device="cuda")
    lf = torch.zeros((n, 5), dtype=torch.int32, device="cuda")
    gpu.version_probe_dev(v, dlsm_amd.Keys(torch.from_numpy(q).cuda(), n, 20), snap, mask, lf)
    gpu.sync()
    assert t_create < 3.0, (nf, t_create)
    assert np.array_equal(mask.cpu().numpy().view(np.uint64), want), nf
    assert np.array_equal(lf.cpu().numpy().view(np.uint32), want_lf), nf
    v.close()


def random_version(rng, n_l0, span):
    """A version of random shape: n_l0 overlapping level-0 files, levels 1-5
    with 0-80 range-partitioned files each (some levels empty), filters of
    bits_per_key 2-20 (k 1-13; the kernels' k = 6 specialisation and the
    generic loop), a fifth of the files without a filter, one-key files."""
    files = []
    num = 1
    for j in range(n_l0):
        a = int(rng.integers(0, span))
        b = min(span, a + int(rng.integers(1, span // 2)))
        vals = np.unique(rng.integers(a, b + 1, int(rng.integers(1, 3000))))
        filt = None if rng.random() < 0.2 else build_filter_bpk(vals, int(rng.integers(2, 21)))
        files.append(VersionFile(0, num, K(vals[0]), K(vals[-1]), (int(rng.integers(1, 1 << 50)) << 8) | 1, filt))
        num += 1
    for level in range(1, 6):
        nf = int(rng.integers(0, 81)) if rng.random() < 0.85 else 0
        if nf == 0:
            continue
        edges = np.sort(rng.choice(np.arange(1, span), size=2 * nf, replace=False))
        for q in range(nf):
            lo, hi = int(edges[2 * q]), int(edges[2 * q + 1])
            vals = np.unique(rng.integers(lo, hi + 1, int(rng.integers(1, 2000))))
            vals = np.unique(np.concatenate([[lo, hi], vals]))  # the file's bounds are keys of the file
            filt = None if rng.random() < 0.2 else build_filter_bpk(vals, int(rng.integers(2, 21)))
            files.append(VersionFile(level, num, K(lo), K(hi), (int(rng.integers(1, 1 << 50)) << 8) | 1, filt))
            num += 1
    return files


def build_filter_bpk(values, bpk):
    keys = oracle.keys_from_values(np.asarray(values, dtype=np.uint64))
    return oracle.full_build(keys, len(values), bpk=bpk)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_gpu_version_probe_random_shapes(gpu, seed):
    """Random versions (level-0 counts 0-50, levels of 0-80 files, empty levels,
    filters of k 1-13 and none, one-key files) against lookups that are half
    keys of the files (filters pass: long probe queues) and half uniform, at
    random snapshots: slot masks and picked files equal the oracle's, for
    20-byte keys and as 28-byte internal keys."""
    import torch

    import dlsm_amd

    rng = np.random.default_rng(100 + seed)
    span = 2_000_000
    n_l0 = [0, 1, 7, 23, 50, 12, 3, 40][seed]
    files = random_version(rng, n_l0, span)
    n = 150_001
    hits = rng.integers(0, span + 1, n // 2)
    v_ = np.concatenate([hits, rng.integers(0, span + span // 5, n - n // 2)]).astype(np.uint64)
    q = oracle.keys_from_values(v_)
    snap = int(rng.integers(1, 1 << 52))
    want, want_lf = oracle.version_probe(files, q, n, snapshot=snap)
    v = gpu.version(files)
    mask = torch.zeros(n, dtype=torch.uint64, device="cuda")
    lf = torch.zeros((n, 5), dtype=torch.int32, device="cuda")
    gpu.version_probe_dev(v, dlsm_amd.Keys(torch.from_numpy(q).cuda(), n, 20), snap, mask, lf)
    gpu.sync()
    assert np.array_equal(mask.cpu().numpy().view(np.uint64), want)
    assert np.array_equal(lf.cpu().numpy().view(np.uint32), want_lf)
    ik = np.concatenate([q.reshape(n, 20), np.frombuffer(((snap & 0xffff) << 8 | 1).to_bytes(8, "little") * n,
                                                         dtype=np.uint8).reshape(n, 8)], axis=1).reshape(-1)
    want28, _ = oracle.version_probe(files, ik, n, snapshot=snap, stride=28, suffix=8)
    mask.zero_()
    gpu.version_probe_dev(v, dlsm_amd.Keys(torch.from_numpy(np.ascontiguousarray(ik)).cuda(), n, 28, suffix_len=8),
                          snap, mask)
    gpu.sync()
    assert np.array_equal(mask.cpu().numpy().view(np.uint64), want28)
    v.close()


def test_oracle_random_shapes_consistent():
    """CPU check of the random-shape generator and the oracle: the filter only
    removes candidates, and every lookup that is a key of a file with a filter
    keeps that file when it is the file Version::Get visits."""
    rng = np.random.default_rng(7)
    files = random_version(rng, 9, 200_000)
    n = 20_000
    q = oracle.keys_from_values(rng.integers(0, 220_000, n).astype(np.uint64))
    mask, lf = oracle.version_probe(files, q, n, snapshot=1 << 51)
    nofilt = [VersionFile(f.level, f.number, f.smallest, f.largest, f.largest_trailer, None) for f in files]
    cand, lf2 = oracle.version_probe(nofilt, q, n, snapshot=1 << 51)
    assert np.array_equal(lf, lf2)
    assert np.all((mask & ~cand) == 0) and cand.any()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [2, 3, 4, 5])
def test_gpu_version_tiers_forced(mode):
    """Every table tier on small and random versions (one file, three, up to a
    few hundred, no level-0 files, empty levels): DLSM_VERSION_LDS=2..5 forces
    the metadata + prefixes, metadata + sparse index, sparse index only and
    nothing-in-LDS tiers (the variable is read once per process, so each tier
    runs in a child process of its own, one after another)."""
    import os
    import subprocess
    import sys

    env = dict(os.environ, DLSM_VERSION_LDS=str(mode))
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "_version_tier_check.py")],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.strip().splitlines()[-1] == "ok 5"
