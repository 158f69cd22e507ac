"""Device-resident probe of 100 M lookups against the bench's 8 stacked
filters from host-computed BloomHash values (dlsm_bloom_full_probe_hashed_dev,
4 B/key) next to the probe from the 20-byte keys: one JSON line each."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dlsm_amd  # noqa: E402
from dlsm_amd import workload as W  # noqa: E402


def main(T=8, N=1_600_000, Q=100_000_000, reps=5):
    dev = torch.device("cuda", 0)
    ctx = dlsm_amd.Context(0)
    tabs = [dlsm_amd.Keys(W.dbbench_keys_torch(torch.arange(N, device=dev) * T + s).reshape(-1), N, 20)
            for s in range(T)]
    outs = [torch.zeros(dlsm_amd.full_size(N)[0], dtype=torch.uint8, device=dev) for _ in range(T)]
    lens = torch.zeros(T, dtype=torch.uint64, device=dev)
    torch.cuda.synchronize()
    ctx.full_build_dev(tabs, outs, lens, 10)
    ctx.sync()
    fl = lens.cpu().numpy()
    fs = ctx.filterset([outs[f][: int(fl[f])] for f in range(T)], on_device=True)
    qk = W.dbbench_keys_torch(torch.randint(0, 2 * T * N, (Q,), device=dev)).reshape(-1)
    hashes = torch.from_numpy(dlsm_amd.hash_batch(dlsm_amd.Keys(qk.cpu().numpy(), Q, 20)).view("int32")).to(dev)
    mask = torch.empty(Q, dtype=torch.uint8, device=dev)
    mask2 = torch.empty(Q, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(device=dev)
    ctx.set_stream(s)
    torch.cuda.synchronize()
    for name, call in (("keys", lambda: ctx.full_probe_dev(fs, dlsm_amd.Keys(qk, Q, 20), mask)),
                       ("hashes", lambda: ctx.full_probe_hashed_dev(fs, hashes, mask2, Q))):
        call()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record(s)
        for _ in range(reps):
            call()
        e[1].record(s)
        s.synchronize()
        ms = e[0].elapsed_time(e[1]) / reps
        print(json.dumps({"probe_from": name, "grid_env": os.environ.get("DLSM_PART_GRID_PER_CU", "default"),
                          "ms": round(ms, 4), "mkeys_s": round(Q / ms / 1e3, 1)}), flush=True)
    print(json.dumps({"masks_equal": bool(torch.equal(mask, mask2))}), flush=True)


if __name__ == "__main__":
    main()
