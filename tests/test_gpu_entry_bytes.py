"""3-byte probe entries (DLSM_OPT_PROBE_ENTRY_BYTES, default 3): the sliced
probe's buckets ordered by quarter slice, entries packed 4 to a 12-byte unit,
the slice pass deriving each entry's sub-slice from its bucket's sub-bucket
starts.  Masks are compared byte for byte with the oracle and with 4-byte
entries, over image sizes (S = 16 .. 128 slices, the last slice short), chunk
shapes (4,096 / 8,192 keys: E3; 16,384: falls back to 4-byte entries), and
lookup counts that leave ragged last chunks.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import dlsm_amd

    if not dlsm_amd.device_available():
        pytest.skip("no HIP device")
    c = dlsm_amd.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("n_per,q,lgc", [(200_000, 1_000_003, 13), (1_600_000, 2_000_001, 13),
                                         (500_000, 777_777, 12), (500_000, 300_001, 14), (37_000, 8_191, 13)])
def test_entry_bytes_3_vs_4_vs_oracle(ctx, orc, n_per, q, lgc):
    import dlsm_amd

    F = 8
    tabs = [orc.dbbench_keys(f, F, n_per) for f in range(F)]
    filters = ctx.full_build([dlsm_amd.Keys(t, n_per, 20) for t in tabs], 10)
    fs = ctx.filterset(filters)
    qk = orc.keys_from_values(orc.mt_values(1000, 2 * F * n_per, q))
    keys = dlsm_amd.Keys(qk, q, 20)
    try:
        ctx.set_option(dlsm_amd.OPT_PROBE_CHUNK_LG, lgc)
        ctx.set_option(dlsm_amd.OPT_PATH, 2)  # sliced
        got = {}
        for eb in (3, 4):
            ctx.set_probe_entry_bytes(eb)
            got[eb] = ctx.full_probe(fs, keys)
        want = orc.full_probe(filters, qk, q, nthreads=8)
        assert np.array_equal(got[3], want)
        assert np.array_equal(got[4], want)
    finally:
        ctx.set_probe_entry_bytes(3)
        ctx.set_option(dlsm_amd.OPT_PROBE_CHUNK_LG, 13)
        ctx.set_option(dlsm_amd.OPT_PATH, 0)
        fs.close()


def test_entry_bytes_option_rules(ctx):
    import dlsm_amd

    assert ctx.get_option(dlsm_amd.OPT_PROBE_ENTRY_BYTES) == 3
    with pytest.raises(dlsm_amd.DlsmError):
        ctx.set_probe_entry_bytes(5)
    ctx.set_probe_entry_bytes(4)
    assert ctx.get_option(dlsm_amd.OPT_PROBE_ENTRY_BYTES) == 4
    ctx.set_probe_entry_bytes(3)
