"""Regression for the sliced-probe corruption fixed in commit 1c7c4c6
(DESIGN.md section 6): 1,024-thread probe slice workgroups in which waves
4..15 each walk 64-chunk groups of more than 2^16 entries.

The root cause is pinned by tests/diag/run_old_slice.py (the pre-fix kernel
run in isolation): wrong answers appeared only when a one-VGPR scratch spill
(__launch_bounds__(1024, 8)) and two 1,024-thread workgroups per CU came
together; either alone was clean.  The current kernels take no such bound and
spill nothing (the resource usage is checked on the CPU in
tests/test_host_abi.py); this test runs the shape on the GPU."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 1_600_000  # the bench filters: L = 31,251 lines
F = 8
NQ = 17_000_003  # > 2 parts x 16 waves x 64 chunks of 8,192 keys, ragged tail


def test_slice_waves_4_to_15_large_groups(gpu, orc):
    import torch

    import dlsm_amd

    # the launch shape this exercises (bloom_capi.hip group_slices / slice_parts)
    C, R = 8192, 256
    L = 31_251
    S = -(-L // R)
    nC = -(-NQ // C)
    parts = min(max(1, (256 + S // 2) // S), max(1, nC // 16))
    per_part = nC // parts
    groups = -(-per_part // 64)
    assert S == 123 and parts == 2 and groups >= 16  # every one of the 16 waves walks a group
    assert 64 * (C + 4 * 256) > (1 << 16)  # in-group entry offsets past 16 bits

    filters = [orc.full_build(orc.dbbench_keys(f, F, N), N) for f in range(F)]
    q = orc.keys_from_values(orc.mt_values(4242, 2 * F * N, NQ))
    want = orc.full_probe(filters, q, NQ, nthreads=16)
    fs = gpu.filterset(filters, on_device=False)
    qd = torch.from_numpy(q).cuda()
    mask = torch.full((NQ,), 0xEE, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    gpu.set_path(2)  # sliced, forced
    try:
        gpu.full_probe_dev(fs, dlsm_amd.Keys(qd, NQ, 20), mask)
        gpu.sync()
    finally:
        gpu.set_path(0)
    got = mask.cpu().numpy()
    bad = np.nonzero(got != want)[0]
    if bad.size:
        c = bad // C
        wave = ((c - (c * parts // nC) * nC // parts) // 64) % 16
        pytest.fail(f"{bad.size} wrong answers; per wave {np.bincount(wave, minlength=16).tolist()}")
    fs.close()
