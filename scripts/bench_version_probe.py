"""Batched Get over a version, device-resident: the
files Version::Get visits for each lookup (db/version_set.cc:273-321) and
their full-filter answers (table/table.cc:350-358), one
dlsm_version_probe_dev call per batch.

The version has the shape of db_bench's final state at config 5 (the replay
of DESIGN.md §7: 5 + 40 + 377 files on levels 1-3 for 100 M keys) plus 4
level-0 flush files: level files partition the key space [0, V), each file's
filter holds every key of its range on that level (the key space is spread
over the levels as 1 : 10 : 100), level-0 files hold 153,846 keys of random
ranges.  Lookups are uniform over [0, 2V): half of them miss every file.
Prints one JSON line.

    python scripts/bench_version_probe.py [--lookups 100000000] [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lookups", type=int, default=100_000_000)
    ap.add_argument("--space", type=int, default=100_000_000, help="key space V")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--check", type=int, default=200_000, help="lookups checked against the oracle")
    ap.add_argument("--paths", default="both", choices=["both", "sliced", "direct"])
    ap.add_argument("--pass-slices", type=int, default=0, help="DLSM_OPT_VERSION_PASS_SLICES (0: default)")
    ap.add_argument("--slice-bytes", type=int, default=64 << 20,
                    help="DLSM_OPT_VERSION_SLICE_BYTES for the version (levels whose filters exceed it are "
                         "sliced; the library's default slices none): path 0 probes them sliced, path 1 direct")
    ap.add_argument("--no-filters", action="store_true", help="diagnostic: the same version without filters")
    args = ap.parse_args()

    import numpy as np
    import torch

    import dlsm_amd
    from dlsm_amd import VersionFile
    from dlsm_amd import workload as W

    dev = torch.device("cuda", 0)
    ctx = dlsm_amd.Context(0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream)
    if args.pass_slices:
        ctx.set_option(dlsm_amd.OPT_VERSION_PASS_SLICES, args.pass_slices)
    if args.slice_bytes and args.paths != "direct":
        ctx.set_option(dlsm_amd.OPT_VERSION_SLICE_BYTES, args.slice_bytes)
    res_slice = args.slice_bytes if args.paths != "direct" else None
    V = args.space
    files = W.dbbench_version(ctx, dev, V)
    rng = np.random.default_rng(11)
    for _ in range(4):  # the generator state the lookups were drawn from before the shared builder
        rng.integers(0, V - 153_846 * 600)
        rng.integers(50, 600)
    if args.no_filters:
        files = [VersionFile(f.level, f.number, f.smallest, f.largest, f.largest_trailer, None) for f in files]
    ver = ctx.version(files, on_device=True)
    filt_bytes = sum(int(f.filter.numel()) for f in files if f.filter is not None)

    Q = args.lookups
    qv = torch.from_numpy(rng.integers(0, 2 * V, Q, dtype=np.int64)).to(dev)
    qk = dlsm_amd.Keys(W.dbbench_keys_torch(qv), Q, 20)
    mask = torch.zeros(Q, dtype=torch.int64, device=dev)
    snap = (1 << 56) - 1
    res = {"what": "version probe (batched Get over a version), device-resident",
           "files_per_level": [4, 5, 40, 377, 0, 0], "filter_bytes": filt_bytes, "lookups": Q,
           "slice_bytes": res_slice}
    want = None
    if args.check:
        import oracle

        oracle.lib()
        n = min(args.check, Q)
        hf = [VersionFile(f.level, f.number, f.smallest, f.largest, f.largest_trailer,
                          f.filter.cpu().numpy().tobytes()) for f in files]
        hq = qk.data[: n * 20].cpu().numpy()
        want, _ = oracle.version_probe(hf, hq, n, snapshot=snap)
        res["oracle_checked"] = n
    # path 0: levels past --slice-bytes take the sliced probe (route /
    # partition / LDS slice / unpermute); path 1: every level direct.  With
    # both, the two alternate twice (the first timed run of a process can
    # run slow) and each keeps its faster run.
    order = [(0, "sliced"), (1, "direct")] * (2 if args.paths == "both" else 1)
    for path, label in order:
        if args.paths != "both" and args.paths != label:
            continue
        ctx.set_path(path)
        ctx.version_probe_dev(ver, qk, snap, mask)
        ctx.sync()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.reps):
            ctx.version_probe_dev(ver, qk, snap, mask)
        e1.record(stream)
        stream.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        rec = {"ms": round(ms, 3), "mgets_s": round(Q / ms / 1e3, 1)}
        if want is not None:
            got = mask[: res["oracle_checked"]].cpu().numpy().astype(np.uint64)
            rec["matches_oracle"] = bool(np.array_equal(got, np.asarray(want, dtype=np.uint64)))
        if label not in res or rec["ms"] < res[label]["ms"]:
            if label in res and "matches_oracle" in res[label]:
                rec["matches_oracle"] = rec.get("matches_oracle", True) and res[label]["matches_oracle"]
            res[label] = rec
    ctx.set_path(0)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
