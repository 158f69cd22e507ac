"""GPU parity of the co-scheduled step (dlsm_ctx_set_partition_stream over
CU-masked streams, bench.py --cosched): a build context whose slice pass runs
on a few CUs of every XCD and whose partition runs on the others, beside a
probe context whose partition shares that partition stream.  The filters and
masks of several back-to-back steps must equal the oracle byte for byte (the
events between the streams are the only thing ordering the workspace reuse)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("per_xcd", [1, 4])
def test_cosched_steps_match_oracle(orc, per_xcd):
    import torch

    import dlsm_amd

    dev = torch.device("cuda", 0)
    n, T, F, nq = 200_000, 16, 8, 3_000_000
    tabs, want = [], []
    for s in range(T):
        k = orc.dbbench_keys(s, T, n)
        want.append(orc.full_build(k, n))
        tabs.append(dlsm_amd.Keys(torch.from_numpy(k).to(dev), n, 20))
    rng = np.random.default_rng(7)
    q = orc.keys_from_values(rng.integers(0, T * n * 2, nq, dtype=np.uint64))
    fwant = want[:F]
    mwant = orc.full_probe(fwant, q, nq, nthreads=8)

    n_cus = torch.cuda.get_device_properties(dev).multi_processor_count
    small = dlsm_amd.cu_subset(per_xcd, n_cus)
    big = sorted(set(range(n_cus)) - set(small))
    s_small = dlsm_amd.cu_mask_stream(0, small, n_cus)
    s_big = dlsm_amd.cu_mask_stream(0, big, n_cus)
    s_all = torch.cuda.Stream(device=dev)
    cb, cp = dlsm_amd.Context(0), dlsm_amd.Context(0)
    cb.set_stream(s_small)
    cp.set_stream(s_all)
    for c in (cb, cp):
        c.set_partition_stream(s_big, len(big))
    torch.cuda.synchronize()
    fs = cp.filterset(fwant, on_device=False)
    qd = torch.from_numpy(q).to(dev)
    outs = [torch.zeros(dlsm_amd.full_size(n)[0] + 16, dtype=torch.uint8, device=dev) for _ in range(T)]
    lens = torch.zeros(T, dtype=torch.uint64, device=dev)
    mask = torch.zeros(nq, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    for step in range(4):
        with torch.cuda.stream(s_small):
            for o in outs:
                o.fill_(0xAB)
        with torch.cuda.stream(s_all):
            mask.fill_(0xAB)
        cb.full_build_dev(tabs, outs, lens, 10)
        cp.full_probe_dev(fs, dlsm_amd.Keys(qd, nq, 20), mask)
        s_small.synchronize()
        s_all.synchronize()
        s_big.synchronize()
        L = lens.cpu().numpy()
        for s in range(T):
            assert outs[s][: int(L[s])].cpu().numpy().tobytes() == want[s], (step, s)
        assert np.array_equal(mask.cpu().numpy(), mwant), step
    # back to one stream: the same answers
    cp.set_partition_stream(None)
    mask.zero_()
    torch.cuda.synchronize()
    cp.full_probe_dev(fs, dlsm_amd.Keys(qd, nq, 20), mask)
    cp.sync()
    assert np.array_equal(mask.cpu().numpy(), mwant)
