"""BASELINE configs at their stated sizes, compared with the oracle in full:

* config 3: 100 M random lookups (v = mt19937_64(1000) mod 25.6 M) against the
  8 stacked 1.6 M-key filters -- every one of the 100 M mask bytes;
* configs 2 / 4: the 16 x 1.6 M-key SSTable batch -- every filter byte.

Sizes are the bench's; the oracle runs multi-threaded (at most 16 threads: a
GPU box's host share)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 1_600_000
F = 8
Q = 100_000_000
THREADS = max(1, min(16, os.cpu_count() or 1))


def test_config3_full_100m_lookups(gpu, orc):
    import torch

    import dlsm_amd
    from dlsm_amd import workload as W

    filters = []
    tabs, outs = [], []
    for f in range(F):
        v = torch.arange(N, device="cuda", dtype=torch.int64) * F + f
        tabs.append(dlsm_amd.Keys(W.dbbench_keys_torch(v), N, 20))
        outs.append(torch.zeros(dlsm_amd.full_size(N)[0], dtype=torch.uint8, device="cuda"))
    lens = torch.zeros(F, dtype=torch.uint64, device="cuda")
    torch.cuda.synchronize()  # inputs were made on torch's stream; the context has its own
    gpu.full_build_dev(tabs, outs, lens, 10)
    gpu.sync()
    del tabs
    filters = [o[: int(n)] for o, n in zip(outs, lens.cpu().numpy())]
    host_filters = [f.cpu().numpy().tobytes() for f in filters]
    for f in range(F):  # the filter set itself, byte for byte
        assert host_filters[f] == orc.full_build(orc.dbbench_keys(f, F, N), N), f
    qv = orc.mt_values(1000, 2 * F * N, Q)
    qk = orc.keys_from_values(qv)
    del qv
    fs = gpu.filterset(filters, on_device=True)
    qd = torch.from_numpy(qk).cuda()
    mask = torch.empty(Q, dtype=torch.uint8, device="cuda")
    for path in (0, 2):  # auto (the bench's sliced path) and sliced forced
        mask.fill_(0xEE)
        torch.cuda.synchronize()
        gpu.set_path(path)
        try:
            gpu.full_probe_dev(fs, dlsm_amd.Keys(qd, Q, 20), mask)
            gpu.sync()
        finally:
            gpu.set_path(0)
        got = mask.cpu().numpy()
        if path == 0:
            want = orc.full_probe(host_filters, qk, Q, nthreads=THREADS)
            # the present keys (v < 12.8 M: exactly one filter) all match
            assert want.mean() > 0  # sanity
        assert np.array_equal(got, want), path
    # about half the lookups are present, each in exactly one filter; FP ~1 %
    fs.close()


def test_config4_full_16x1p6m_batch(gpu, orc):
    import torch

    import dlsm_amd
    from dlsm_amd import workload as W

    T = 16
    tabs, outs, hk = [], [], []
    for s in range(T):
        v = torch.arange(N, device="cuda", dtype=torch.int64) * T + s
        k = W.dbbench_keys_torch(v)
        tabs.append(dlsm_amd.Keys(k, N, 20))
        hk.append(k.cpu().numpy())
        outs.append(torch.full((dlsm_amd.full_size(N)[0] + 64,), 0xEE, dtype=torch.uint8, device="cuda"))
    lens = torch.zeros(T, dtype=torch.uint64, device="cuda")
    torch.cuda.synchronize()
    gpu.full_build_dev(tabs, outs, lens, 10)
    gpu.sync()
    want = orc.full_build_many(hk, [N] * T, 20, 10, THREADS)
    L = lens.cpu().numpy()
    for s in range(T):
        got = outs[s].cpu().numpy()
        assert int(L[s]) == len(want[s]) == 2_000_069
        assert got[: int(L[s])].tobytes() == want[s], s
        assert (got[int(L[s]):] == 0xEE).all()


@pytest.mark.parametrize("shape", ["mixed_set", "dedup_shifted"])
def test_realistic_filter_sets_full_100m_lookups(gpu, orc, shape):
    """The bench's realistic probe legs (bench.py SHAPE_LEGS): the config-3
    lookups against 8 filters of different line counts -- the one-pass
    multi-group probe (round 6) -- every one of the 100 M mask bytes against
    the oracle, and against the per-group passes (DLSM_OPT_PROBE_MULTI = 0)."""
    import torch

    import bench
    import dlsm_amd
    from dlsm_amd import workload as W

    sizes = bench.SHAPE_LEGS[shape]
    Fs = len(sizes)
    tabs, outs = [], []
    for f, n in enumerate(sizes):
        v = torch.arange(n, device="cuda", dtype=torch.int64) * Fs + f
        tabs.append(dlsm_amd.Keys(W.dbbench_keys_torch(v), n, 20))
        outs.append(torch.zeros(dlsm_amd.full_size(n)[0], dtype=torch.uint8, device="cuda"))
    lens = torch.zeros(Fs, dtype=torch.uint64, device="cuda")
    torch.cuda.synchronize()
    gpu.full_build_dev(tabs, outs, lens, 10)
    gpu.sync()
    del tabs
    filters = [o[: int(n)] for o, n in zip(outs, lens.cpu().numpy())]
    host_filters = [f.cpu().numpy().tobytes() for f in filters]
    for f, n in enumerate(sizes):
        assert host_filters[f] == orc.full_build(orc.dbbench_keys(f, Fs, n), n), f
    qk = orc.keys_from_values(orc.mt_values(1000, 2 * F * N, Q))
    fs = gpu.filterset(filters, on_device=True)
    qd = torch.from_numpy(qk).cuda()
    mask = torch.empty(Q, dtype=torch.uint8, device="cuda")
    want = orc.full_probe(host_filters, qk, Q, nthreads=THREADS)
    assert want.any()
    for multi in (1, 0):
        mask.fill_(0xEE)
        torch.cuda.synchronize()
        gpu.set_option(dlsm_amd.OPT_PROBE_MULTI, multi)
        try:
            gpu.full_probe_dev(fs, dlsm_amd.Keys(qd, Q, 20), mask)
            gpu.sync()
        finally:
            gpu.set_option(dlsm_amd.OPT_PROBE_MULTI, 1)
        assert np.array_equal(mask.cpu().numpy(), want), multi
    fs.close()
