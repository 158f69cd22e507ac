"""The three ways a host-API call waits for its stream (DLSM_HOST_SYNC, read
when a context is created: 0 hipStreamSynchronize, 1 event poll + yield --
the default, 2 blocking-sync event) give the same bytes: host-key builds
(dlsm_bloom_full_build: keys H2D, kernels, the wait, the copy-out), a legacy
host build and a host probe, each vs the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["0", "1", "2"])
def test_host_calls_under_each_wait_mode(orc, mode, monkeypatch):
    import dlsm_amd

    if not dlsm_amd.device_available():
        pytest.fail("GPU test requested but no HIP device is visible")
    monkeypatch.setenv("DLSM_HOST_SYNC", mode)
    ctx = dlsm_amd.Context(0)
    try:
        sizes = [153_846, 20_001, 1]
        tabs = [orc.dbbench_keys(s + 7, 3, n) for s, n in enumerate(sizes)]
        keys = [dlsm_amd.Keys(t, n, 20) for t, n in zip(tabs, sizes)]
        for _ in range(3):  # repeated calls on the same context
            got = ctx.full_build(keys)
            assert got == [orc.full_build(t, n) for t, n in zip(tabs, sizes)], mode
        assert ctx.legacy_build(keys) == [orc.legacy_build(t, n) for t, n in zip(tabs, sizes)], mode
        q = orc.keys_from_values(orc.mt_values(11, 600_000, 100_003))
        fs = ctx.filterset(got)
        mask = ctx.full_probe(fs, dlsm_amd.Keys(q, 100_003, 20))
        fs.close()
        want = orc.full_probe(got, q, 100_003)
        assert np.array_equal(np.asarray(mask), np.asarray(want)), mode
    finally:
        ctx.close()
