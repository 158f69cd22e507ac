"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference-generated golden fixtures.  Bit-exact for every byte and every
probe answer; both kernel families (direct, sliced) are checked."""
import numpy as np
import pytest

from tests._util import case_keys

pytestmark = pytest.mark.gpu

PATHS = [0, 1, 2]  # auto, direct, sliced


def keys_of(case):
    import dlsm_amd

    data, offs, stride, n = case_keys(case)
    if offs is None:
        return dlsm_amd.Keys(data, n, stride, None)
    return dlsm_amd.Keys(np.concatenate([data, np.zeros(16, np.uint8)]), n, 0, offs)


@pytest.mark.parametrize("path", [1, 2])
def test_full_build_golden_cases(gpu, golden, path):
    gpu.set_path(path)
    try:
        for c in golden["full"]["cases"]:
            got = gpu.full_build([keys_of(c)], c["bpk"])[0]
            assert got.hex() == c["filter"], (c["name"], path)
    finally:
        gpu.set_path(0)


@pytest.mark.parametrize("path", [1, 2])
def test_full_build_golden_batch(gpu, golden, path):
    """All golden cases with bpk 10 as ONE batched call (mixed shapes -> generic keys)."""
    cases = [c for c in golden["full"]["cases"] if c["bpk"] == 10]
    gpu.set_path(path)
    try:
        got = gpu.full_build([keys_of(c) for c in cases], 10)
    finally:
        gpu.set_path(0)
    for c, g in zip(cases, got):
        assert g.hex() == c["filter"], c["name"]


@pytest.mark.parametrize("path", [1, 2])
def test_full_build_digests(gpu, golden, orc, path):
    import dlsm_amd

    gpu.set_path(path)
    try:
        for d in golden["full"]["digests"]:
            if d.get("format") == "legacy":
                continue
            keys = orc.dbbench_keys(d["first"], d["step"], d["n"])
            f = gpu.full_build([dlsm_amd.Keys(keys, d["n"], 20)], d["bpk"])[0]
            assert len(f) == d["len"] and orc.fnv1a64(f) == d["fnv1a64"], (d["name"], path)
    finally:
        gpu.set_path(0)


def test_full_build_dev_config4_batch(gpu, orc):
    """16 SSTables (12 subcompaction + 4 flush) in one device-resident call."""
    import torch

    import dlsm_amd

    n = 153_846
    tables, outs, want = [], [], []
    for s in range(16):
        k = orc.dbbench_keys(s, 16, n)
        want.append(orc.full_build(k, n))
        tables.append(dlsm_amd.Keys(torch.from_numpy(k).cuda(), n, 20))
        outs.append(torch.zeros(dlsm_amd.full_size(n)[0] + 64, dtype=torch.uint8, device="cuda"))
    lens = torch.zeros(16, dtype=torch.uint64, device="cuda")
    for path in (1, 2):
        for o in outs:
            o.fill_(0xEE)  # garbage: the library must write every filter byte
        torch.cuda.synchronize()  # torch's stream vs the context's own stream
        gpu.set_path(path)
        gpu.full_build_dev(tables, outs, lens, 10)
        gpu.sync()
        gpu.set_path(0)
        L = lens.cpu().numpy()
        for s in range(16):
            assert int(L[s]) == len(want[s])
            got = outs[s][: int(L[s])].cpu().numpy().tobytes()
            assert got == want[s], (s, path)
            assert (outs[s][int(L[s]):].cpu().numpy() == 0xEE).all()  # nothing past the filter


@pytest.mark.parametrize("path", [1, 2])
def test_full_build_random_varlen_and_unaligned(gpu, orc, path):
    import dlsm_amd

    rng = np.random.default_rng(99)
    tables, want = [], []
    for t in range(12):
        n = int(rng.choice([0, 1, 2, 3, 50, 51, 52, 4095, 4096, 4097, 9000, 20000]))
        keys = [bytes(rng.integers(0, 256, int(rng.integers(0, 45)), dtype=np.uint8)) for _ in range(n)]
        # inject adjacent duplicates and repeats
        if n > 10:
            for q in rng.integers(1, n, 5):
                keys[int(q)] = keys[int(q) - 1]
        data, offs = orc.pack_var(keys)
        want.append(orc.full_build(data, n, stride=0, offsets=offs))
        pad = np.concatenate([np.zeros(3, np.uint8), data, np.zeros(16, np.uint8)])
        tables.append(dlsm_amd.Keys(pad, n, 0, offs + 3))  # unaligned start via offsets
    gpu.set_path(path)
    try:
        got = gpu.full_build(tables, 10)
    finally:
        gpu.set_path(0)
    for t in range(len(want)):
        assert got[t] == want[t], (t, path)


@pytest.mark.parametrize("path", [1, 2])
def test_full_build_fixed_nonaligned_lengths(gpu, orc, path):
    import dlsm_amd

    for klen in (1, 3, 7, 8, 16, 21, 24, 29):
        n = 7000
        raw = np.random.default_rng(klen).integers(0, 256, n * klen + 16, dtype=np.uint8)
        want = orc.full_build(raw, n, stride=klen)
        gpu.set_path(path)
        try:
            got = gpu.full_build([dlsm_amd.Keys(raw, n, klen)], 10)[0]
        finally:
            gpu.set_path(0)
        assert got == want, (klen, path)


def test_full_build_dedup_changes_line_count_large(gpu, orc):
    """Enough adjacent duplicates to lower L below the speculative count, at a
    size where the sliced path has many slices (slow-path re-scan)."""
    import dlsm_amd

    n = 300_000
    v = np.arange(n, dtype=np.uint64)
    v[1::3] = v[0::3][: v[1::3].size]  # every third key repeats its predecessor
    keys = orc.keys_from_values(v)
    want = orc.full_build(keys, n)
    assert orc.full_dedup_count(keys, n) < n
    assert len(want) < dlsm_amd.full_size(n)[0]
    for path in (1, 2):
        gpu.set_path(path)
        got = gpu.full_build([dlsm_amd.Keys(keys, n, 20)], 10)[0]
        gpu.set_path(0)
        assert got == want, path


def test_full_build_capacity_error(gpu, orc):
    import dlsm_amd

    keys = orc.dbbench_keys(0, 1, 1000)
    need = dlsm_amd.full_size(1000)[0]
    with pytest.raises(dlsm_amd.DlsmError) as e:
        gpu.full_build([dlsm_amd.Keys(keys, 1000, 20)], 10, caps=[need - 1])
    assert e.value.status == -2


def test_full_build_bits_per_key_sweep(gpu, orc):
    import dlsm_amd

    keys = orc.dbbench_keys(17, 5, 5000)
    for bpk in (0, 1, 2, 3, 7, 10, 15, 20, 33, 44, 64):
        want = orc.full_build(keys, 5000, bpk=bpk)
        for path in (1, 2):
            gpu.set_path(path)
            got = gpu.full_build([dlsm_amd.Keys(keys, 5000, 20)], bpk)[0]
            gpu.set_path(0)
            assert got == want, (bpk, path)


# ---------------------------------------------------------------------------
# probe
# ---------------------------------------------------------------------------

def test_full_probe_golden(gpu, golden, orc):
    import dlsm_amd

    g = golden["probe"]
    filters = [bytes.fromhex(f["filter"]) for f in g["filters"]]
    q = g["queries"]
    keys = orc.dbbench_keys(q["first"], q["step"], q["n"])
    fs = gpu.filterset(filters)
    mask = gpu.full_probe(fs, dlsm_amd.Keys(keys, q["n"], 20))
    for f, ans in enumerate(g["answers"]):
        want = np.frombuffer(bytes.fromhex(ans), dtype=np.uint8)
        assert np.array_equal((mask >> f) & 1, want), f


@pytest.mark.parametrize("F", [1, 3, 8])
def test_full_probe_stacked_vs_oracle(gpu, orc, F):
    """Equal-L filter sets take the sliced (LDS) probe; compare with direct + oracle."""
    import dlsm_amd

    n_per = 200_000
    filters = [orc.full_build(orc.dbbench_keys(f, 8, n_per), n_per) for f in range(F)]
    nq = 1_300_001  # > 256 chunks of 4096: every wave of a 1024-thread slice group works
    vals = orc.mt_values(1000, 8 * n_per * 2, nq)
    q = orc.keys_from_values(vals)
    want = orc.full_probe(filters, q, nq, nthreads=8)
    fs = gpu.filterset(filters)
    for path in PATHS:
        gpu.set_path(path)
        got = gpu.full_probe(fs, dlsm_amd.Keys(q, nq, 20))
        gpu.set_path(0)
        assert np.array_equal(got, want), path
    # keys that are in filter f must answer 1 for f
    assert ((want & 1)[vals % 8 == 0][vals[vals % 8 == 0] < 8 * n_per] == 1).all()


@pytest.mark.parametrize("round_keys", [0, 4096, 4096 * 37, 4096 * 100])
def test_full_probe_pipelined_rounds(gpu, orc, round_keys):
    """Probe rounds pipelined over two streams and three rotating buffers
    (round r's partition beside round r-1's slices): any round size gives the
    oracle's masks, including a ragged last round."""
    import torch

    import dlsm_amd

    n_per = 100_000
    filters = [orc.full_build(orc.dbbench_keys(f, 8, n_per), n_per) for f in range(8)]
    nq = 1_000_003 if round_keys != 4096 else 40_961
    q = orc.keys_from_values(orc.mt_values(77, 8 * n_per * 2, nq))
    want = orc.full_probe(filters, q, nq, nthreads=8)
    fs = gpu.filterset(filters)
    qd = torch.from_numpy(q).cuda()
    mask = torch.full((nq,), 0xEE, dtype=torch.uint8, device="cuda")
    gpu.set_probe_round(round_keys)
    try:
        gpu.full_probe_dev(fs, dlsm_amd.Keys(qd, nq, 20), mask)
        gpu.sync()
    finally:
        gpu.set_probe_round(0)
    assert np.array_equal(mask.cpu().numpy(), want)


@pytest.mark.parametrize("chunk_lg", [12, 13, 14])
@pytest.mark.parametrize("slice_lg", [7, 8])
@pytest.mark.parametrize("key_len", [20, 28])
def test_full_probe_shapes(gpu, orc, chunk_lg, slice_lg, key_len):
    """Every sliced-probe shape (chunk of 4096/8192/16384 keys -- the latter
    two bucketed in two units -- x 64/128 KiB LDS slices) gives the oracle's
    masks, for 20-byte user keys (K20 tiles) and 28-byte internal keys
    (suffix 8, K28 tiles): a ragged key count, filters whose line count is
    not a multiple of the slice, and a 60-line filter set (one partial
    slice)."""
    import torch

    import dlsm_amd

    for n_per, nq in ((100_000, 300_007), (3_000, 20_001)):
        filters = [orc.full_build(orc.dbbench_keys(f, 8, n_per), n_per) for f in range(8)]
        q = orc.keys_from_values(orc.mt_values(91 + chunk_lg, 8 * n_per * 2, nq))
        want = orc.full_probe(filters, q, nq, nthreads=8)
        fs = gpu.filterset(filters)
        if key_len == 28:  # + an 8-byte trailer the hash must skip
            trl = np.random.default_rng(chunk_lg).integers(0, 256, size=(nq, 8), dtype=np.uint8)
            q = np.ascontiguousarray(np.hstack([q.reshape(nq, 20), trl]).reshape(-1))
        qd = torch.from_numpy(q).cuda()
        mask = torch.full((nq,), 0xEE, dtype=torch.uint8, device="cuda")
        gpu.set_path(2)
        gpu.set_probe_shape(chunk_lg, slice_lg)
        try:
            gpu.full_probe_dev(fs, dlsm_amd.Keys(qd, nq, key_len, suffix_len=key_len - 20), mask)
            gpu.sync()
        finally:
            gpu.set_probe_shape(13, 8)
            gpu.set_path(0)
        fs.close()
        assert np.array_equal(mask.cpu().numpy(), want), (n_per, nq)


@pytest.mark.parametrize("groups", [1, 2, 3, 4])
def test_full_build_pipelined_groups(gpu, orc, groups):
    """Job groups pipelined over two streams (group g's partition beside group
    g-1's slices), uneven table sizes, dev and host entry points."""
    import torch

    import dlsm_amd

    sizes = [153_846, 1, 0, 600_000, 77_777, 153_846, 4096, 300_001, 12]
    tables, outs, want = [], [], []
    for s, n in enumerate(sizes):
        k = orc.dbbench_keys(s, len(sizes), n) if n else np.zeros(20, np.uint8)
        want.append(orc.full_build(k, n))
        tables.append(dlsm_amd.Keys(torch.from_numpy(k).cuda(), n, 20))
        outs.append(torch.full((dlsm_amd.full_size(n)[0] + 32,), 0xEE, dtype=torch.uint8, device="cuda"))
    lens = torch.zeros(len(sizes), dtype=torch.uint64, device="cuda")
    gpu.set_build_groups(groups)
    try:
        gpu.full_build_dev(tables, outs, lens, 10)
        gpu.sync()
        host = gpu.full_build([dlsm_amd.Keys(t.data.cpu().numpy(), t.n, 20) for t in tables], 10)
    finally:
        gpu.set_build_groups(0)
    L = lens.cpu().numpy()
    for j, w in enumerate(want):
        assert int(L[j]) == len(w), j
        assert outs[j][: int(L[j])].cpu().numpy().tobytes() == w, (j, groups)
        assert host[j] == w, (j, groups)


def test_set_option_rejects_bad_values(gpu):
    import dlsm_amd

    with pytest.raises(dlsm_amd.DlsmError):
        gpu.set_build_groups(5)
    with pytest.raises(dlsm_amd.DlsmError):
        gpu.set_option(99, 1)
    with pytest.raises(dlsm_amd.DlsmError):
        gpu.set_option(dlsm_amd.OPT_PATH, 3)
    for opt, bad in ((dlsm_amd.OPT_PROBE_CHUNK_LG, 11), (dlsm_amd.OPT_PROBE_CHUNK_LG, 15),
                     (dlsm_amd.OPT_PROBE_SLICE_LG, 6), (dlsm_amd.OPT_PROBE_SLICE_LG, 9)):
        with pytest.raises(dlsm_amd.DlsmError):
            gpu.set_option(opt, bad)


def test_full_probe_many_filters_and_varlen(gpu, orc):
    import dlsm_amd

    rng = np.random.default_rng(5)
    filters = []
    for f in range(13):  # > 8 -> 2 mask bytes, mixed L
        n = int(rng.integers(1, 5000))
        filters.append(orc.full_build(orc.dbbench_keys(int(rng.integers(0, 10000)), 1, n), n))
    keys = [bytes(rng.integers(0, 256, int(rng.integers(0, 30)), dtype=np.uint8)) for _ in range(3000)]
    keys += [orc.dbbench_keys(v, 1, 1).tobytes() for v in range(0, 12000, 7)]
    data, offs = orc.pack_var(keys)
    want = orc.full_probe(filters, data, len(keys), stride=0, offsets=offs)
    fs = gpu.filterset(filters)
    got = gpu.full_probe(fs, dlsm_amd.Keys(np.concatenate([data, np.zeros(16, np.uint8)]),
                                           len(keys), 0, offs))
    assert np.array_equal(got, want)


def test_full_probe_sixteen_mixed_filters_k20(gpu, orc):
    """The filter set Version::Get walks: 10 level-0 flushes (153,846 keys) +
    6 level files of other sizes (up to 6.15 M keys, a 7.7 MB filter): 2 mask
    bytes, 20-byte keys, every path, run twice (deterministic)."""
    import torch

    import dlsm_amd

    sizes = [153_846] * 10 + [600_000, 1_600_000, 3_000_000, 615_384, 6_153_840, 2_000_000]
    F = len(sizes)
    filters = [orc.full_build(orc.dbbench_keys(f, F, n), n) for f, n in enumerate(sizes)]
    nq = 2_000_003
    q = orc.keys_from_values(orc.mt_values(4242, 2 * F * max(sizes), nq))
    want = orc.full_probe(filters, q, nq, nthreads=8)
    fs = gpu.filterset(filters)
    qd = torch.from_numpy(q).cuda()
    mask = torch.empty(2 * nq, dtype=torch.uint8, device="cuda")
    for path in (0, 1, 0):
        mask.fill_(0xEE)
        gpu.set_path(path)
        try:
            gpu.full_probe_dev(fs, dlsm_amd.Keys(qd, nq, 20), mask)
            gpu.sync()
        finally:
            gpu.set_path(0)
        assert np.array_equal(mask.cpu().numpy(), want), path
    fs.close()


@pytest.mark.parametrize("shape", ["mixed8", "equal16", "mixed11_k28"])
def test_full_probe_grouped_sliced(gpu, orc, shape):
    """Filter sets of several (L, k) groups take the grouped sliced probe (one
    hash pass, one partition + slice + unpermute per group, OR-ed mask bytes):
    filters of different sizes, 16 equal filters (two mask bytes), 11 filters
    of 3 sizes probed with 28-byte internal keys.  Forced sliced and auto
    against direct and the oracle."""
    import torch

    import dlsm_amd

    sizes = {"mixed8": [153_846, 153_846, 600_000, 600_000, 1_600_000, 1_600_000, 3_000_000, 3_000_000],
             "equal16": [200_000] * 16,
             "mixed11_k28": [50_000, 90_000, 50_000, 120_000, 90_000, 50_000, 50_000, 120_000, 90_000,
                             50_000, 120_000]}[shape]
    F = len(sizes)
    filters = [orc.full_build(orc.dbbench_keys(f, F, n), n) for f, n in enumerate(sizes)]
    nq = 1_500_007
    q = orc.keys_from_values(orc.mt_values(17, 2 * F * max(sizes), nq))
    want = orc.full_probe(filters, q, nq, nthreads=8)
    klen = 20
    if shape.endswith("k28"):
        trl = np.random.default_rng(3).integers(0, 256, size=(nq, 8), dtype=np.uint8)
        q = np.ascontiguousarray(np.hstack([q.reshape(nq, 20), trl]).reshape(-1))
        klen = 28
    fs = gpu.filterset(filters)
    mb = (F + 7) // 8
    qd = torch.from_numpy(q).cuda()
    mask = torch.empty(mb * nq, dtype=torch.uint8, device="cuda")
    for path in (2, 0, 1):
        mask.fill_(0xEE)
        gpu.set_path(path)
        try:
            gpu.full_probe_dev(fs, dlsm_amd.Keys(qd, nq, klen, suffix_len=klen - 20), mask)
            gpu.sync()
        finally:
            gpu.set_path(0)
        assert np.array_equal(mask.cpu().numpy(), want), (shape, path)
    fs.close()


def test_full_probe_reader_branches_golden(gpu, golden, orc):
    """The reader ctor's two accepted layouts (log2 line 6 and the
    len % num_lines == 0 branch with log2 line 0), against answers of the
    compiled reference (tests/golden/probe.json), filter by filter and all six
    in one set (the set mixes line counts, so it is probed group by group)."""
    import dlsm_amd

    g = golden["probe"]["reader_branches"]
    q = g["queries"]
    keys = orc.dbbench_keys(q["first"], q["step"], q["n"])
    filters = [bytes.fromhex(c["filter"]) for c in g["cases"]]
    wants = [np.frombuffer(bytes.fromhex(c["answers"]), dtype=np.uint8) for c in g["cases"]]
    for fb, want in zip(filters, wants):
        got = gpu.full_probe(gpu.filterset([fb]), dlsm_amd.Keys(keys, q["n"], 20))
        assert np.array_equal(got & 1, want)
    got = gpu.full_probe(gpu.filterset(filters), dlsm_amd.Keys(keys, q["n"], 20))
    for f, want in enumerate(wants):
        assert np.array_equal((got >> f) & 1, want), f


def test_full_probe_log2_zero_branch(gpu, orc):
    """A filter whose num_lines*64 != len but len % num_lines == 0: the reference
    probes it with log2_cache_line_size_ == 0 (full_filter_block.h:85)."""
    import dlsm_amd

    rng = np.random.default_rng(3)
    body = rng.integers(0, 256, 96, dtype=np.uint8).tobytes()
    filt = body + bytes([6, 3, 0, 0, 0])  # L = 3, len 96 = 3 * 32
    st, k, L, lg = dlsm_amd.full_parse(filt)
    assert st == 0 and lg == 0
    q = orc.dbbench_keys(0, 1, 5000)
    want = orc.full_probe([filt], q, 5000)
    got = gpu.full_probe(gpu.filterset([filt]), dlsm_amd.Keys(q, 5000, 20))
    assert np.array_equal(got, want)


def test_full_probe_corrupt_filters(gpu):
    import dlsm_amd

    for bad in [b"", b"\x06", bytes([6, 0, 0, 0, 0]), bytes(64) + bytes([0, 1, 0, 0, 0]),
                bytes(64) + bytes([0x80, 1, 0, 0, 0]), bytes(100) + bytes([6, 3, 0, 0, 0])]:
        with pytest.raises(dlsm_amd.DlsmError) as e:
            gpu.filterset([bad])
        assert e.value.status == -3


def test_full_probe_dev_torch(gpu, orc):
    import torch

    import dlsm_amd

    filters = [orc.full_build(orc.dbbench_keys(f, 4, 50_000), 50_000) for f in range(4)]
    nq = 123_457
    q = orc.keys_from_values(orc.mt_values(7, 400_000, nq))
    want = orc.full_probe(filters, q, nq)
    fdev = [torch.from_numpy(np.frombuffer(f, np.uint8).copy()).cuda() for f in filters]
    fs = gpu.filterset(fdev, on_device=True)
    qd = torch.from_numpy(q).cuda()
    mask = torch.zeros(nq, dtype=torch.uint8, device="cuda")
    gpu.full_probe_dev(fs, dlsm_amd.Keys(qd, nq, 20), mask)
    gpu.sync()
    assert np.array_equal(mask.cpu().numpy(), want)


# ---------------------------------------------------------------------------
# legacy FilterPolicy format
# ---------------------------------------------------------------------------

def test_legacy_golden(gpu, golden, orc):
    import dlsm_amd

    g = golden["legacy"]
    for c in g["cases"]:
        got = gpu.legacy_build([keys_of(c)], c["bpk"])[0]
        assert got.hex() == c["filter"], c["name"]
    f = bytes.fromhex(g["small"]["filter"])
    for q, want in g["small"]["queries"].items():
        assert gpu.legacy_probe(f, dlsm_amd.Keys.pack([q.encode()]))[0] == want
    for e in g["edges"]:
        fb = bytes.fromhex(e["filter"])
        keys = orc.dbbench_keys(e["query_first"], 1, len(e["answers"]))
        got = gpu.legacy_probe(fb, dlsm_amd.Keys(keys, len(e["answers"]), 20))
        assert list(got) == e["answers"], e.get("k_byte")


def test_legacy_random_vs_oracle(gpu, orc):
    import dlsm_amd

    rng = np.random.default_rng(11)
    tables, want = [], []
    for n in (0, 1, 5, 6, 7, 64, 1000, 33333):
        keys = [bytes(rng.integers(0, 256, int(rng.integers(0, 25)), dtype=np.uint8)) for _ in range(n)]
        data, offs = orc.pack_var(keys)
        want.append(orc.legacy_build(data, n, stride=0, offsets=offs))
        tables.append(dlsm_amd.Keys(np.concatenate([data, np.zeros(16, np.uint8)]), n, 0, offs))
    got = gpu.legacy_build(tables, 10)
    assert got == want
    q = orc.dbbench_keys(0, 3, 20000)
    for f in want:
        assert np.array_equal(gpu.legacy_probe(f, dlsm_amd.Keys(q, 20000, 20)),
                              orc.legacy_probe(f, q, 20000))


def test_bloom_test_semantics_on_gpu(gpu):
    """util/bloom_test.cc:82-150 (EmptyFilter, Small, VaryingLengths) on the GPU policy."""
    import struct

    import dlsm_amd

    pol = dlsm_amd.BloomFilterPolicy(10, gpu)
    assert pol.Name() == "TimberSaw.BuiltinBloomFilter2"
    empty = bytearray()
    pol.CreateFilter([], 0, empty)
    assert not pol.KeyMayMatch(b"hello", bytes(empty))
    small = bytearray()
    pol.CreateFilter([b"hello", b"world"], 2, small)
    assert pol.KeyMayMatch(b"hello", bytes(small)) and pol.KeyMayMatch(b"world", bytes(small))
    assert not pol.KeyMayMatch(b"x", bytes(small)) and not pol.KeyMayMatch(b"foo", bytes(small))
    good = mediocre = 0
    length = 1
    while length <= 10000:
        keys = [struct.pack("<I", i) for i in range(length)]
        f = bytearray()
        pol.CreateFilter(keys, length, f)
        assert len(f) <= length * 10 // 8 + 40
        assert pol.KeysMayMatch(dlsm_amd.Keys.pack(keys), bytes(f)).all()
        qk = dlsm_amd.Keys.pack([struct.pack("<I", i + 1000000000) for i in range(10000)])
        rate = pol.KeysMayMatch(qk, bytes(f)).mean()
        assert rate <= 0.02
        good, mediocre = (good, mediocre + 1) if rate > 0.0125 else (good + 1, mediocre)
        length = length + 1 if length < 10 else length + 10 if length < 100 else \
            length + 100 if length < 1000 else length + 1000
    assert mediocre <= good / 5


# ---------------------------------------------------------------------------
# reference-shaped classes and full-size properties
# ---------------------------------------------------------------------------

def test_full_filter_block_builder_and_reader(gpu, orc):
    import dlsm_amd

    slot = np.zeros(256 * 1024, dtype=np.uint8)  # FILTER_BLOCK slot (options.h:28)
    b = dlsm_amd.FullFilterBlockBuilder(slot, 10, gpu)
    b.RestartBlock(0)
    keys = orc.dbbench_keys(0, 1, 20_000)
    for i in range(20_000):
        b.AddKey(keys[i * 20:(i + 1) * 20].tobytes())
    b.Finish()
    want = orc.full_build(keys, 20_000)
    assert bytes(b.result) == want
    r = dlsm_amd.FullFilterBlockReader(bytes(b.result), gpu)
    assert r.num_probes_ == 6 and r.num_lines_ == dlsm_amd.full_size(20_000)[1]
    assert r.KeyMayMatch(keys[:20].tobytes())
    q = orc.dbbench_keys(0, 1, 40_000)
    assert np.array_equal(r.KeysMayMatch(dlsm_amd.Keys(q, 40_000, 20)),
                          orc.full_probe([want], q, 40_000).astype(bool))
    b.Reset()
    assert len(b.result) == 0


def test_full_size_properties(gpu, orc):
    """At BASELINE size (1.6M keys): no false negatives, FP ~1.2 %, probe of
    a stacked set agrees with single-filter probes (size-independent checks)."""
    import dlsm_amd

    n = 1_600_000
    tabs = [dlsm_amd.Keys(orc.dbbench_keys(f, 8, n), n, 20) for f in range(8)]
    filters = gpu.full_build(tabs, 10)
    fs = gpu.filterset(filters)
    for f in range(8):
        m = gpu.full_probe(fs, tabs[f])
        assert ((m >> f) & 1).all(), f
    absent = dlsm_amd.Keys(orc.dbbench_keys(8 * n + 12345, 1, 1_000_000), 1_000_000, 20)
    m = gpu.full_probe(fs, absent)
    fp = np.unpackbits(m[:, None], axis=1).mean()
    assert 0.008 < fp < 0.016, fp
    single = gpu.filterset([filters[3]])
    m3 = gpu.full_probe(single, absent)
    assert np.array_equal(m3 & 1, (m >> 3) & 1)


# ---------------------------------------------------------------------------
# filter blocks (FinishFilterBlock trailer) and crc32c on the GPU
# ---------------------------------------------------------------------------

def test_filter_block_golden(gpu, golden, orc):
    names = {c["name"]: c for c in golden["full"]["cases"]}
    for b in golden["full"]["blocks"]:
        c = names[b["name"]]
        got = gpu.full_build_block([keys_of(c)], 10)[0]
        assert got.hex() == c["filter"] + b["trailer"], b["name"]


def test_filter_block_batch_vs_oracle(gpu, golden, orc):
    import torch

    import dlsm_amd

    specs = [(s, 16, 153_846) for s in range(16)] + [(0, 1, 1_600_000), (3, 7, 1), (5, 3, 0)]
    tables, outs, want = [], [], []
    for first, step, n in specs:
        k = orc.dbbench_keys(first, step, n) if n else np.zeros(16, np.uint8)
        want.append(orc.filter_block(orc.full_build(k, n)))
        tables.append(dlsm_amd.Keys(torch.from_numpy(k).cuda(), n, 20))
        outs.append(torch.full((dlsm_amd.full_size(n)[0] + 5,), 0xEE, dtype=torch.uint8, device="cuda"))
    lens = torch.zeros(len(specs), dtype=torch.uint64, device="cuda")
    gpu.full_build_block_dev(tables, outs, lens, 10)
    gpu.sync()
    L = lens.cpu().numpy()
    for j, w in enumerate(want):
        assert int(L[j]) == len(w)
        assert outs[j][: int(L[j])].cpu().numpy().tobytes() == w, specs[j]
    d = [x for x in golden["full"]["digests"] if x["name"] == "dbbench_seq_1600000"][0]
    assert want[16][-5:].hex() == d["block_trailer"]


def test_filter_block_capacity(gpu, orc):
    import dlsm_amd

    k = orc.dbbench_keys(0, 1, 1000)
    need = dlsm_amd.full_size(1000)[0] + 5
    with pytest.raises(dlsm_amd.DlsmError) as e:
        gpu.full_build_block([dlsm_amd.Keys(k, 1000, 20)], 10, caps=[need - 1])
    assert e.value.status == -2


def test_crc32c_dev_vs_oracle(gpu, golden, orc):
    import torch

    rng = np.random.default_rng(42)
    bufs, want = [], []
    for c in golden["full"]["crc32c"]:
        b = bytes.fromhex(c["data"])
        bufs.append(torch.tensor(list(b), dtype=torch.uint8, device="cuda"))
        want.append(c["crc"])
    for n in [1, 15, 16, 17, 1023, 1024, 16384, 65535, 65536, 65537, 2_000_069, 3_000_001]:
        b = rng.integers(0, 256, n, dtype=np.uint8)
        t = torch.from_numpy(b).cuda()
        bufs.append(t[1:] if n > 100 else t)  # also an unaligned start
        want.append(orc.crc32c((b[1:] if n > 100 else b).tobytes()))
    assert gpu.crc32c_dev(bufs) == want


@pytest.mark.parametrize("seed", range(6))
def test_full_probe_random_sets(gpu, orc, seed):
    """Random filter sets: 1-24 filters of 0-400 K keys each at bits_per_key
    2-20 (some sets of equal line counts, some mixed: stacked, packed and
    grouped images, direct groups), lookups of a random count and key length
    (16 / 20 / 28 / 33 bytes), half of them keys of the filters.  Every path
    (auto, direct, sliced where the set allows it) equals the oracle."""
    import dlsm_amd

    rng = np.random.default_rng(500 + seed)
    F = int(rng.integers(1, 25))
    key_len = [20, 28, 16, 33, 20, 28][seed]
    equal = seed % 2 == 0
    n_eq = int(rng.integers(1, 400_000))
    tabs, ns = [], []
    for f in range(F):
        n = n_eq if equal else int(rng.integers(0, 400_000))
        vals = rng.integers(0, 1 << 40, n).astype(np.uint64)
        tabs.append(vals)
        ns.append(n)
    bpk = int(rng.integers(2, 21)) if equal else None
    filters = [orc.full_build(orc.keys_from_values(t, key_len), n, stride=key_len,
                              bpk=bpk or int(rng.integers(2, 21))) for t, n in zip(tabs, ns)]
    nq = int(rng.integers(1, 700_000))
    pool = np.concatenate([t for t in tabs if t.size] + [np.zeros(1, np.uint64)])
    vals = np.where(rng.random(nq) < 0.5, pool[rng.integers(0, pool.size, nq)],
                    rng.integers(0, 1 << 40, nq).astype(np.uint64)).astype(np.uint64)
    q = orc.keys_from_values(vals, key_len)
    want = orc.full_probe(filters, q, nq, stride=key_len, nthreads=8)
    fs = gpu.filterset(filters)
    for path in PATHS:
        gpu.set_path(path)
        try:
            got = gpu.full_probe(fs, dlsm_amd.Keys(q, nq, key_len))
        except dlsm_amd.DlsmError:
            assert path == 2  # a set with an unsliceable group refuses the forced sliced path
            continue
        finally:
            gpu.set_path(0)
        assert np.array_equal(got, want), (path, F, key_len, equal)
    fs.close()
