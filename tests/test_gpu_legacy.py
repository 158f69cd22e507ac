"""GPU parity of the legacy FilterPolicy format (util/bloom.cc:25-81) at the
sizes BASELINE config 2 names, on both kernel families: the direct path
(global atomics, path 1) and the LDS-tiled path (tile-bucketed positions,
path 2 / auto).  Every filter byte is compared with the oracle (and the
survey-time digests of the compiled reference)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SURVEY_LEGACY = {1_600_000: (2_000_001, 0x5175E13CB3B564AB), 153_846: (192_309, 0xA95FEDF1B0F1CB89)}


@pytest.mark.parametrize("path", [1, 2])
def test_legacy_digests(gpu, golden, orc, path):
    """The reference's CreateFilter digests at 1.6 M and 153,846 keys."""
    import dlsm_amd

    gpu.set_path(path)
    try:
        for d in golden["full"]["digests"]:
            if d.get("format") != "legacy":
                continue
            keys = orc.dbbench_keys(d["first"], d["step"], d["n"])
            f = gpu.legacy_build([dlsm_amd.Keys(keys, d["n"], 20)], d["bpk"])[0]
            assert len(f) == d["len"] and orc.fnv1a64(f) == d["fnv1a64"], (d["name"], path)
            if d["n"] in SURVEY_LEGACY:
                assert (len(f), orc.fnv1a64(f)) == SURVEY_LEGACY[d["n"]]
    finally:
        gpu.set_path(0)


def _dev_batch(orc, n, tables=16):
    import torch

    import dlsm_amd

    keys, want, outs = [], [], []
    for s in range(tables):
        k = orc.dbbench_keys(s, tables, n)
        want.append(orc.legacy_build(k, n))
        keys.append(dlsm_amd.Keys(torch.from_numpy(k).cuda(), n, 20))
        outs.append(torch.full((dlsm_amd.legacy_size(n) + 64,), 0xEE, dtype=torch.uint8, device="cuda"))
    return keys, want, outs


@pytest.mark.parametrize("n", [1_600_000, 153_846])
def test_legacy_config4_batch_dev(gpu, orc, n):
    """16 SSTables (config 4's shape: table s <- v = 16 i + s) in one
    device-resident legacy call, every byte vs the oracle, both paths; nothing
    past a filter is written."""
    import torch

    keys, want, outs = _dev_batch(orc, n)
    lens = torch.zeros(16, dtype=torch.uint64, device="cuda")
    for path in (2, 1, 0):
        for o in outs:
            o.fill_(0xEE)
        lens.zero_()
        gpu.set_path(path)
        try:
            gpu.legacy_build_dev(keys, outs, lens, 10)
            gpu.sync()
        finally:
            gpu.set_path(0)
        L = lens.cpu().numpy()
        for s in range(16):
            assert int(L[s]) == len(want[s]), (s, path)
            got = outs[s][: int(L[s])].cpu().numpy().tobytes()
            assert got == want[s], (s, path, n)
            assert (outs[s][int(L[s]):].cpu().numpy() == 0xEE).all(), (s, path)


def test_legacy_shapes_vs_oracle(gpu, orc):
    """Sizes around the chunk / tile boundaries, bits-per-key 1..14 (k 1..9:
    k > 8 falls back to the direct path), one batch per bpk."""
    import dlsm_amd

    rng = np.random.default_rng(23)
    sizes = [0, 1, 5, 6, 7, 64, 1000, 4095, 4096, 4097, 6553, 6554, 33333, 200_000]
    for bpk in (1, 2, 3, 5, 8, 10, 12, 13, 14):
        tables, want = [], []
        for n in sizes:
            k = orc.dbbench_keys(int(rng.integers(0, 1 << 40)), int(rng.integers(1, 9)), n)
            want.append(orc.legacy_build(k, n, bpk=bpk))
            tables.append(dlsm_amd.Keys(k if n else np.zeros(20, np.uint8), n, 20))
        got = gpu.legacy_build(tables, bpk)
        for n, g, w in zip(sizes, got, want):
            assert g == w, (bpk, n)


def test_legacy_forced_sliced_path_falls_back_to_direct(gpu, orc):
    """Path 2 (sliced forced) with a batch the tiled kernels cannot take --
    bits_per_key 14 (k = 9 > 8) -- builds on the direct kernel with the same
    bytes instead of failing: a context set to path 2 for its full
    filters keeps building legacy ones."""
    import dlsm_amd

    sizes = [1, 7, 4097, 200_000]
    tabs = [orc.dbbench_keys(3 + s, 8, n) for s, n in enumerate(sizes)]
    gpu.set_path(2)
    try:
        for bpk in (10, 14, 20):
            got = gpu.legacy_build([dlsm_amd.Keys(t, n, 20) for t, n in zip(tabs, sizes)], bpk)
            assert got == [orc.legacy_build(t, n, bpk=bpk) for t, n in zip(tabs, sizes)], bpk
    finally:
        gpu.set_path(0)


def test_legacy_varlen_and_internal_keys(gpu, orc):
    """Variable-length keys (offsets, generic loader) and 28-byte internal
    keys (suffix 8: ExtractUserKey, K28 loader) on the tiled path."""
    import dlsm_amd

    rng = np.random.default_rng(5)
    tables, want = [], []
    for n in (1, 100, 4097, 50_000):
        keys = [bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8)) for _ in range(n)]
        data, offs = orc.pack_var(keys)
        want.append(orc.legacy_build(data, n, stride=0, offsets=offs))
        tables.append(dlsm_amd.Keys(np.concatenate([data, np.zeros(16, np.uint8)]), n, 0, offs))
    gpu.set_path(2)
    try:
        assert gpu.legacy_build(tables, 10) == want
    finally:
        gpu.set_path(0)
    # internal keys: user key (20 B) || Fixed64(seq << 8 | type); hashed as the user key
    n = 70_000
    uk = orc.dbbench_keys(7, 3, n).reshape(n, 20)
    trailer = rng.integers(0, 256, (n, 8), dtype=np.uint8)
    ik = np.ascontiguousarray(np.concatenate([uk, trailer], axis=1)).reshape(-1)
    w = orc.legacy_build(uk.reshape(-1), n)
    gpu.set_path(2)
    try:
        g = gpu.legacy_build([dlsm_amd.Keys(ik, n, 28, None, 8)], 10)[0]
    finally:
        gpu.set_path(0)
    assert g == w


@pytest.mark.parametrize("tps", ["0", "1", "2", "3", "4"])
def test_legacy_tiles_per_slice(gpu, orc, tps):
    """Every slice width (2^tps tiles of 8 KiB per workgroup) gives the same bytes."""
    import dlsm_amd

    n = 1_000_003
    k = orc.dbbench_keys(11, 5, n)
    want = orc.legacy_build(k, n)
    os.environ["DLSM_LEGACY_TPS_LG"] = tps
    try:
        got = gpu.legacy_build([dlsm_amd.Keys(k, n, 20), dlsm_amd.Keys(k[:20 * 9000], 9000, 20)], 10)
    finally:
        del os.environ["DLSM_LEGACY_TPS_LG"]
    assert got[0] == want
    assert got[1] == orc.legacy_build(k[:20 * 9000], 9000)


def test_legacy_large_filters(gpu, orc):
    """A filter past variant A's staging (partition variant B: 3 M keys) and
    one past every tiled variant (20 M keys: the direct path), in one batch
    each, bit-exact."""
    import torch

    import dlsm_amd

    for n in (3_000_000, 20_000_000):
        k = orc.dbbench_keys(3, 7, n)
        want = orc.legacy_build(k, n)
        out = torch.full((len(want) + 32,), 0xEE, dtype=torch.uint8, device="cuda")
        lens = torch.zeros(1, dtype=torch.uint64, device="cuda")
        gpu.legacy_build_dev([dlsm_amd.Keys(torch.from_numpy(k).cuda(), n, 20)], [out], lens, 10)
        gpu.sync()
        assert int(lens.cpu()[0]) == len(want)
        assert out[: len(want)].cpu().numpy().tobytes() == want, n
        assert (out[len(want):].cpu().numpy() == 0xEE).all()


def test_legacy_unaligned_slots(gpu, orc):
    """Output slots at odd offsets (the tiled path's byte-store epilogue)."""
    import torch

    import dlsm_amd

    n = 70_001
    k = orc.dbbench_keys(1, 2, n)
    want = orc.legacy_build(k, n)
    buf = torch.full((len(want) + 64,), 0xEE, dtype=torch.uint8, device="cuda")
    lens = torch.zeros(2, dtype=torch.uint64, device="cuda")
    kd = dlsm_amd.Keys(torch.from_numpy(k).cuda(), n, 20)
    for off in (1, 4):
        buf.fill_(0xEE)
        gpu.legacy_build_dev([kd], [buf[off: off + len(want)]], lens, 10)
        gpu.sync()
        assert buf[off: off + len(want)].cpu().numpy().tobytes() == want, off
        assert (buf[:off].cpu().numpy() == 0xEE).all() and (buf[off + len(want):].cpu().numpy() == 0xEE).all()


def test_back_to_back_batches_without_sync(gpu, orc):
    """Two different batched builds (full and legacy) queued back to back on
    one stream, no synchronisation in between: each call's job table comes
    from the context's page-locked upload slots, so the second call's tables
    cannot overwrite the first's before its kernels read them."""
    import torch

    import dlsm_amd

    calls, want_f, want_l = [], [], []
    for rep, n in enumerate((40_000, 90_001)):
        tabs = [orc.dbbench_keys(100 * rep + s, 5, n + s) for s in range(3)]
        keys = [dlsm_amd.Keys(torch.from_numpy(t).cuda(), n + s, 20) for s, t in enumerate(tabs)]
        of = [torch.zeros(dlsm_amd.full_size(n + s)[0] + 16, dtype=torch.uint8, device="cuda") for s in range(3)]
        ol = [torch.zeros(dlsm_amd.legacy_size(n + s) + 16, dtype=torch.uint8, device="cuda") for s in range(3)]
        lf = torch.zeros(3, dtype=torch.uint64, device="cuda")
        ll = torch.zeros(3, dtype=torch.uint64, device="cuda")
        calls.append((keys, of, ol, lf, ll))
        want_f.append([orc.full_build(t, n + s) for s, t in enumerate(tabs)])
        want_l.append([orc.legacy_build(t, n + s) for s, t in enumerate(tabs)])
    # the fixture runs torch and the context on one stream: the inputs above
    # are ordered before the builds, and nothing below waits between them
    for keys, of, ol, lf, ll in calls:
        gpu.full_build_dev(keys, of, lf, 10)
        gpu.legacy_build_dev(keys, ol, ll, 10)
    gpu.sync()
    for r, (keys, of, ol, lf, ll) in enumerate(calls):
        for s in range(3):
            nf, nl = int(lf.cpu()[s]), int(ll.cpu()[s])
            assert of[s][:nf].cpu().numpy().tobytes() == want_f[r][s], (r, s)
            assert ol[s][:nl].cpu().numpy().tobytes() == want_l[r][s], (r, s)


def test_legacy_probe_at_config2_size(gpu, orc):
    """util/bloom.cc KeyMayMatch (util/bloom.cc:57-81) against a 1.6 M-key
    legacy filter built on the GPU: 4 M lookups (the table's 1.6 M keys, then
    2.4 M random db_bench keys) through the device probe, every answer vs the
    oracle; members always match, the others at ~1 % (10 bits/key)."""
    import torch

    import dlsm_amd

    n, q = 1_600_000, 4_000_000
    t = orc.dbbench_keys(3, 16, n)
    keys = [dlsm_amd.Keys(torch.from_numpy(t).cuda(), n, 20)]
    out = torch.zeros(dlsm_amd.legacy_size(n) + 16, dtype=torch.uint8, device="cuda")
    lens = torch.zeros(1, dtype=torch.uint64, device="cuda")
    gpu.legacy_build_dev(keys, [out], lens, 10)
    gpu.sync()
    L = int(lens.cpu()[0])
    filt = out[:L].cpu().numpy().tobytes()
    assert filt == orc.legacy_build(t, n)
    look = np.concatenate([t.reshape(-1), orc.keys_from_values(orc.mt_values(77, 1 << 40, q - n)).reshape(-1)])
    assert look.size == 20 * q
    ans = torch.zeros(q, dtype=torch.uint8, device="cuda")
    gpu.legacy_probe_dev(out, L, dlsm_amd.Keys(torch.from_numpy(look).cuda(), q, 20), ans)
    gpu.sync()
    got = ans.cpu().numpy()
    want = orc.legacy_probe(filt, look, q)
    assert np.array_equal(got, want)
    assert got[:n].all()
    assert 0.005 < got[n:].mean() < 0.02
