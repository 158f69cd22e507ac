"""Packed filter images (bloom_capi.hip ProbeGroup::lgw, pack_filters_kernel,
probe_slice_kernel<LGR, LGW < 3>): a group of 1, 2 or 3-4 filters of one line
count is probed from an image of W = 1, 2 or 4 bits per bit position (2,048 /
1,024 / 512 lines per 128 KiB slice) instead of the byte-wide stacked image.

* equal-size sets of 1..5 filters (the single-group path: W = 1, 2, 4, 4, 8);
* a set whose largest filter (6.15 M keys, 120 K lines) is too large for the
  byte-wide image (470 slices of 256 lines) but fits packed (59 slices of
  2,048), forced onto the sliced path;
* a grouped set mixing W = 1, 2 and 4 groups in one mask byte and members in
  non-contiguous slots;
every answer against the oracle, and against the byte-wide images
(DLSM_PROBE_PACKED=0) where those exist."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _probe(gpu, filters, q, nq, path, packed=True):
    import torch

    import dlsm_amd

    old = os.environ.get("DLSM_PROBE_PACKED")
    os.environ["DLSM_PROBE_PACKED"] = "1" if packed else "0"
    try:
        fs = gpu.filterset(filters)
    finally:
        if old is None:
            del os.environ["DLSM_PROBE_PACKED"]
        else:
            os.environ["DLSM_PROBE_PACKED"] = old
    mb = (len(filters) + 7) // 8
    qd = torch.from_numpy(q).cuda()
    mask = torch.full((mb * nq,), 0xEE, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    gpu.set_path(path)
    try:
        gpu.full_probe_dev(fs, dlsm_amd.Keys(qd, nq, 20), mask)
        gpu.sync()
    finally:
        gpu.set_path(0)
        fs.close()
    return mask.cpu().numpy()


@pytest.mark.parametrize("F", [1, 2, 3, 4, 5])
def test_equal_sets_one_to_five_filters(gpu, orc, F):
    n = 1_600_000
    filters = [orc.full_build(orc.dbbench_keys(f, F, n), n) for f in range(F)]
    nq = 1_000_003
    q = orc.keys_from_values(orc.mt_values(99 + F, 2 * F * n, nq))
    want = orc.full_probe(filters, q, nq, nthreads=8)
    assert np.array_equal(_probe(gpu, filters, q, nq, 2), want)
    assert np.array_equal(_probe(gpu, filters, q, nq, 2, packed=False), want)


def test_big_single_filter_sliced_packed(gpu, orc):
    sizes = [6_153_840, 153_846, 153_846]
    F = len(sizes)
    filters = [orc.full_build(orc.dbbench_keys(f, F, n), n) for f, n in enumerate(sizes)]
    nq = 1_500_001
    q = orc.keys_from_values(orc.mt_values(5, 2 * F * max(sizes), nq))
    want = orc.full_probe(filters, q, nq, nthreads=8)
    for path in (2, 0):  # forced sliced: every group (W = 1 and W = 2) is sliceable now
        assert np.array_equal(_probe(gpu, filters, q, nq, path), want), path


def test_grouped_mixed_widths_scattered_slots(gpu, orc):
    # slots 0..7 of one mask byte: sizes chosen so the (L, k) groups are
    # {0, 5} (W 2), {1, 3, 6} (W 4), {2} (W 1), {4, 7} (W 2)
    a, b, c, d = 300_000, 500_000, 900_000, 130_000
    sizes = [a, b, c, b, d, a, b, d]
    F = len(sizes)
    filters = [orc.full_build(orc.dbbench_keys(f, F, n), n) for f, n in enumerate(sizes)]
    nq = 1_200_007
    q = orc.keys_from_values(orc.mt_values(77, 2 * F * max(sizes), nq))
    want = orc.full_probe(filters, q, nq, nthreads=8)
    for path in (2, 0):
        assert np.array_equal(_probe(gpu, filters, q, nq, path), want), path
    assert np.array_equal(_probe(gpu, filters, q, nq, 2, packed=False), want)
