"""Probe time by filter-set shape (device-resident, 20-byte keys, 10 bits/key):
the bench's 8 equal 1.6 M-key filters against the filter sets Version::Get
really walks (db/version_set.cc:273-321): filters of different sizes (memtable
flushes of 153,846 keys, compaction outputs of other sizes, dedup-shifted line
counts) and more than 8 of them.  Prints one JSON line per shape.

    python scripts/bench_probe_shapes.py [--lookups 20000000] [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {
    # name: keys per filter
    "equal_8x1.6M": [1_600_000] * 8,
    "mixed_8": [153_846, 153_846, 600_000, 600_000, 1_600_000, 1_600_000, 3_000_000, 3_000_000],
    "equal_8x153846": [153_846] * 8,
    "l0_plus_levels_16": [153_846] * 10 + [600_000, 1_600_000, 3_000_000, 153_846 * 4, 153_846 * 40, 2_000_000],
    "dedup_shifted_8": [1_600_000 - 97 * f for f in range(8)],
}
SHAPES["mixed_set"] = SHAPES["mixed_8"]  # bench.py SHAPE_LEGS names
SHAPES["dedup_shifted"] = SHAPES["dedup_shifted_8"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lookups", type=int, default=20_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--shapes", default="equal_8x1.6M,mixed_8,equal_8x153846,l0_plus_levels_16,dedup_shifted_8")
    ap.add_argument("--check", type=int, default=1_000_000, help="lookups checked against the oracle")
    ap.add_argument("--paths", default="auto,per_group,direct",
                    help="auto (one-pass multi-group), per_group (a pass per group), direct")
    args = ap.parse_args()

    import numpy as np
    import torch

    import dlsm_amd
    from dlsm_amd import workload as W

    dev = torch.device("cuda", 0)
    ctx = dlsm_amd.Context(0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)  # torch's input making and the library share one stream
    ctx.set_stream(stream)
    Q = args.lookups
    for name in args.shapes.split(","):
        sizes = SHAPES[name]
        F = len(sizes)
        # filter f <- v = F*i + f, i < sizes[f]
        tabs, outs = [], []
        with torch.cuda.stream(stream):
            for f, n in enumerate(sizes):
                v = torch.arange(n, device=dev, dtype=torch.int64) * F + f
                tabs.append(dlsm_amd.Keys(W.dbbench_keys_torch(v), n, 20))
                outs.append(torch.zeros(dlsm_amd.full_size(n)[0], dtype=torch.uint8, device=dev))
            lens = torch.zeros(F, dtype=torch.uint64, device=dev)
        ctx.full_build_dev(tabs, outs, lens, 10)
        ctx.sync()
        filters = [outs[f][: int(lens[f])] for f in range(F)]
        fs = ctx.filterset(filters, on_device=True)
        span = 2 * F * max(sizes)
        qv = W.mt19937_64(1000, Q) % np.uint64(span)
        q = dlsm_amd.Keys(W.dbbench_keys_torch(torch.from_numpy(qv.astype(np.int64)).to(dev)), Q, 20)
        mask = torch.empty(Q * fs.mask_bytes, dtype=torch.uint8, device=dev)
        rec = {"shape": name, "filters": F, "keys_per_filter": sizes, "lookups": Q}
        ref_mask = None
        for path, label, multi in ((0, "auto", 1), (0, "per_group", 0), (1, "direct", 1)):
            if label not in args.paths.split(",") or (label == "per_group" and len(set(sizes)) == 1):
                continue
            ctx.set_path(path)
            ctx.set_option(dlsm_amd.OPT_PROBE_MULTI, multi)
            ctx.full_probe_dev(fs, q, mask)  # warm
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.reps):
                ctx.full_probe_dev(fs, q, mask)
            e1.record(stream)
            stream.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            rec[label] = {"ms": round(ms, 4), "mkeys_s": round(Q / ms / 1e3, 1)}
            m = mask.cpu().numpy()
            if ref_mask is None:
                ref_mask = m
            rec["paths_agree"] = bool(np.array_equal(ref_mask, m))
        ctx.set_path(0)
        ctx.set_option(dlsm_amd.OPT_PROBE_MULTI, 1)
        if args.check:
            import oracle  # checker only

            nc = min(args.check, Q)
            hf = [f.cpu().numpy().tobytes() for f in filters]
            want = oracle.full_probe(hf, q.data[: nc * 20].cpu().numpy(), nc, nthreads=16)
            rec["matches_oracle_first"] = nc
            rec["oracle_ok"] = bool(np.array_equal(ref_mask[: nc * fs.mask_bytes], want))
        print(json.dumps(rec), flush=True)
        fs.close()
        del tabs, outs, filters, q, mask


if __name__ == "__main__":
    main()
