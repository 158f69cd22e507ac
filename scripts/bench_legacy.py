"""Time the legacy-format batch build (util/bloom.cc CreateFilter for 16 x
1.6 M db_bench keys, device-resident) alone: one JSON line with the tiled
path's ms per call (HIP events over --reps calls) and whether table 0 equals
the oracle.  For A/B of library variants (DLSM_LIB_VARIANT) in one session.

    python scripts/bench_legacy.py [--tables 16] [--keys 1600000] [--reps 30]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tables", type=int, default=16)
    ap.add_argument("--keys", type=int, default=1_600_000)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--bpk", type=int, default=10)
    ap.add_argument("--path", type=int, default=0)
    a = ap.parse_args()
    import torch

    import dlsm_amd
    import oracle  # checker only

    T, N = a.tables, a.keys
    ctx = dlsm_amd.Context(0)
    st = torch.cuda.Stream()
    ctx.set_stream(st)
    ctx.set_path(a.path)
    keys = [dlsm_amd.Keys(torch.from_numpy(oracle.dbbench_keys(s, T, N)).cuda(), N, 20) for s in range(T)]
    outs = [torch.zeros(dlsm_amd.legacy_size(N, a.bpk) + 16, dtype=torch.uint8, device="cuda") for _ in range(T)]
    lens = torch.zeros(T, dtype=torch.uint64, device="cuda")
    torch.cuda.synchronize()
    for _ in range(3):
        ctx.legacy_build_dev(keys, outs, lens, a.bpk)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(a.reps):
        ctx.legacy_build_dev(keys, outs, lens, a.bpk)
    e1.record(st)
    st.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    L = lens.cpu().numpy()
    want = oracle.legacy_build(keys[0].data.cpu().numpy(), N, bpk=a.bpk)
    ok = outs[0][: int(L[0])].cpu().numpy().tobytes() == want
    alg = T * N * 20 + int(L.sum())
    print(json.dumps({"variant": os.environ.get("DLSM_LIB_VARIANT", "base"),
                      "env": {k: v for k, v in os.environ.items() if k.startswith("DLSM_LEGACY")}, "tables": T, "keys": N,
                      "ms": round(ms, 4), "mkeys_s": round(T * N / ms / 1e3, 1),
                      "alg_GBs": round(alg / ms / 1e6, 1), "frac": round(alg / ms / 1e6 / 8000, 4),
                      "table0_matches_oracle": ok}))


if __name__ == "__main__":
    main()
