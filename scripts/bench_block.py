"""The sealed filter-block build against the plain batch build (bench.py
block_leg's shape: 16 x 1.6 M db_bench keys, 10 bits/key), device-resident,
HIP events over --reps calls each; run under rocprofv3 --stats for the
per-kernel split.  Prints one JSON line.  --only-block runs the sealed
builds alone, for the rocprofv3 --pmc passes behind the block leg's traffic.

    python scripts/bench_block.py [--reps 20] [--only-block]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tables", type=int, default=16)
    ap.add_argument("--keys", type=int, default=1_600_000)
    ap.add_argument("--only-block", action="store_true",
                    help="run only the sealed builds (one warm + --reps calls): the PMC passes' shape")
    args = ap.parse_args()
    import torch

    import bench
    import dlsm_amd
    from dlsm_amd import workload as W

    dev = torch.device("cuda", 0)
    ctx = dlsm_amd.Context(0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream)
    T, N = args.tables, args.keys
    tables = []
    for s in range(T):
        v = torch.arange(N, device=dev, dtype=torch.int64) * T + s
        tables.append(dlsm_amd.Keys(W.dbbench_keys_torch(v), N, 20))
    torch.cuda.synchronize()
    if args.only_block:
        outs = [torch.zeros(dlsm_amd.full_size(N)[0] + 64, dtype=torch.uint8, device=dev) for _ in tables]
        lens = torch.zeros(T, dtype=torch.uint64, device=dev)
        for _ in range(args.reps + 1):
            ctx.full_build_block_dev(tables, outs, lens, 10)
        stream.synchronize()
        print(json.dumps({"block_calls": args.reps + 1, "block_bytes": int(lens.cpu().sum())}), flush=True)
        return
    print(json.dumps(bench.block_leg(ctx, stream, tables, 10, reps=args.reps)), flush=True)


if __name__ == "__main__":
    main()
