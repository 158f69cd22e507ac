"""Device-resident build + probe rates for internal keys (20-B user key + 8-B
trailer, dlsm_keyset.suffix_len = 8) next to plain 20-B user keys: what the
key loader costs when callers hand over iterator keys unchanged."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dlsm_amd  # noqa: E402
from dlsm_amd import workload as W  # noqa: E402


def keys(v, internal):
    k = W.dbbench_keys_torch(v).reshape(-1, 20)
    if internal:
        tr = torch.zeros((k.shape[0], 8), dtype=torch.uint8, device=k.device)
        tr[:, 0] = 1  # kTypeValue, sequence 0
        k = torch.cat([k, tr], dim=1)
    return k.reshape(-1).contiguous()


def run(internal, T=16, N=1_600_000, Q=100_000_000, reps=5, exact=0):
    dev = torch.device("cuda", 0)
    ctx = dlsm_amd.Context(0)
    ctx.set_build_exact(exact)  # 0 auto (internal keys count first), 2 never
    kl, sl = (28, 8) if internal else (20, 0)
    tabs = [dlsm_amd.Keys(keys(torch.arange(N, device=dev) * T + s, internal), N, kl, suffix_len=sl)
            for s in range(T)]
    outs = [torch.zeros(dlsm_amd.full_size(N)[0], dtype=torch.uint8, device=dev) for _ in range(T)]
    lens = torch.zeros(T, dtype=torch.uint64, device=dev)
    torch.cuda.synchronize()  # inputs were made on torch's stream; ctx runs on its own
    ctx.full_build_dev(tabs, outs, lens, 10)
    ctx.sync()
    fl = lens.cpu().numpy()
    fs = ctx.filterset([outs[f][: int(fl[f])] for f in range(8)], on_device=True)
    q = dlsm_amd.Keys(keys(torch.randint(0, 2 * T * N, (Q,), device=dev), internal), Q, kl, suffix_len=sl)
    mask = torch.empty(Q, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    ctx.full_probe_dev(fs, q, mask)
    ctx.sync()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    s = torch.cuda.Stream(device=dev)  # a real stream: handle 0 would mean "ctx's own"
    ctx.set_stream(s)
    e[0].record(s)
    for _ in range(reps):
        ctx.full_build_dev(tabs, outs, lens, 10)
    e[1].record(s)
    for _ in range(reps):
        ctx.full_probe_dev(fs, q, mask)
    e[2].record(s)
    s.synchronize()
    b = e[0].elapsed_time(e[1]) / reps
    p = e[1].elapsed_time(e[2]) / reps
    return {"internal_keys": internal, "key_bytes": kl, "build_exact": {0: "auto", 1: "always", 2: "never"}[exact],
            "build_ms": round(b, 4),
            "build_mkeys_s": round(T * N / b / 1e3, 1), "probe_ms": round(p, 4),
            "probe_mkeys_s": round(Q / p / 1e3, 1)}


if __name__ == "__main__":
    for internal in (False, True):
        print(json.dumps(run(internal)), flush=True)
    # the internal-key build without its count pass (speculative line count:
    # right for these unique user keys, slow fallback when versions repeat)
    print(json.dumps(run(True, exact=2)), flush=True)
