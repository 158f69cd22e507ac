"""Headline benchmark: Bloom build+probe Mkeys/s (device-resident), 20 B keys,
10 bits/key -- BASELINE.json's metric.

One step (per GPU, weak scaling: SSTables shard one-per-GPU with no
collective):
  * build: 16 SSTable full filters (12 subcompaction + 4 flush outputs) of
    1.6M db_bench keys each, in one device-resident batch call
    (dlsm_bloom_full_build_dev) -- BASELINE configs[1]/[3] shape;
  * probe: 100M 20-byte lookups (v = mt19937_64(1000+rank) mod 25.6M) against
    8 stacked per-level full filters (dlsm_bloom_full_probe_dev) --
    BASELINE configs[2].
value = (build keys + probe keys) over all ranks / max-over-ranks wall time.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--keys-per-table", type=int, default=1_600_000)
    ap.add_argument("--tables", type=int, default=16)
    ap.add_argument("--lookups", type=int, default=100_000_000)
    ap.add_argument("--filters", type=int, default=8)
    ap.add_argument("--bits-per-key", type=int, default=10)
    ap.add_argument("--path", type=int, default=0, help="0 auto, 1 direct, 2 sliced")
    ap.add_argument("--probe-round", type=int, default=None,
                    help="keys per pipelined probe round (0 = one round, the default)")
    ap.add_argument("--build-groups", type=int, default=0, help="pipelined build job groups (0/1 = one group)")
    ap.add_argument("--probe-chunk-lg", type=int, default=13,
                    help="log2 keys per probe partition chunk (12..14; library default 13)")
    ap.add_argument("--probe-slice-lg", type=int, default=8,
                    help="log2 stacked lines per probe LDS slice (7, 8; library default 8)")
    ap.add_argument("--traffic", default=os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                      "profiles", "traffic.json"),
                    help="PMC traffic summary (scripts/pmc_traffic.py) reported as roofline.traffic "
                         "when its config matches this run")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-probe-sample", type=int, default=10_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    args = ap.parse_args()

    import numpy as np
    import torch

    import dlsm_amd
    from dlsm_amd import sharding as SH
    from dlsm_amd import workload as W

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one process per GPU; DLSM_BENCH_BACKEND=gloo (with ranks sharing GPUs,
    # LOCAL_RANK mod device count) rehearses the N>1 path on a 1-GPU box
    backend = os.environ.get("DLSM_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist

        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    N, T, Q, F, bpk = args.keys_per_table, args.tables, args.lookups, args.filters, args.bits_per_key
    ctx = dlsm_amd.Context(local)
    ctx.set_path(args.path)
    if args.probe_round is not None:
        ctx.set_probe_round(args.probe_round)
    ctx.set_build_groups(args.build_groups)
    ctx.set_probe_shape(args.probe_chunk_lg, args.probe_slice_lg)
    stream = torch.cuda.Stream(device=dev)
    ctx.set_stream(stream)

    # ---- inputs, resident in HBM before timing ---------------------------
    t_in = time.time()
    with torch.cuda.stream(stream):
        tables, outs = [], []
        for s in range(T):
            first, step = SH.table_values(rank, s, T, N)
            v = torch.arange(N, device=dev, dtype=torch.int64) * step + first
            tables.append(dlsm_amd.Keys(W.dbbench_keys_torch(v), N, 20))
            outs.append(torch.zeros(dlsm_amd.full_size(N, bpk)[0], dtype=torch.uint8, device=dev))
        lens = torch.zeros(T, dtype=torch.uint64, device=dev)
        # the F stacked per-level filters probed by the lookups: filter f <- v = F*i + f
        ftabs, fouts = [], []
        for f in range(F):
            v = torch.arange(N, device=dev, dtype=torch.int64) * F + f
            ftabs.append(dlsm_amd.Keys(W.dbbench_keys_torch(v), N, 20))
            fouts.append(torch.zeros(dlsm_amd.full_size(N, bpk)[0], dtype=torch.uint8, device=dev))
        flens = torch.zeros(F, dtype=torch.uint64, device=dev)
    ctx.full_build_dev(ftabs, fouts, flens, bpk)
    ctx.sync()
    fl = flens.cpu().numpy()
    filters = [fouts[f][: int(fl[f])] for f in range(F)]
    fs = ctx.filterset(filters, on_device=True)
    qv = W.mt19937_64(SH.lookup_seed(rank), Q) % np.uint64(2 * F * N)
    qkeys = W.dbbench_keys_torch(torch.from_numpy(qv.astype(np.int64)).to(dev))
    qk = dlsm_amd.Keys(qkeys, Q, 20)
    mask = torch.empty(Q * fs.mask_bytes, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    log(f"[rank {rank}] inputs ready in {time.time() - t_in:.1f}s")

    def step():
        ctx.full_build_dev(tables, outs, lens, bpk)
        ctx.full_probe_dev(fs, qk, mask)

    for _ in range(args.warmup):
        step()
    ctx.sync()

    # ---- timed region ----------------------------------------------------
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
            torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        ctx.full_build_dev(tables, outs, lens, bpk)
        evs[i][1].record(stream)
        ctx.full_probe_dev(fs, qk, mask)
        evs[i][2].record(stream)
    stream.synchronize()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = SH.max_over_ranks(elapsed, dist, dev)
    build_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in evs]))
    probe_ms = float(np.mean([b.elapsed_time(c) for _, b, c in evs]))

    keys_per_step = T * N + Q
    value = keys_per_step * world * args.steps / elapsed / 1e6
    filt_bytes = int(fl.sum())
    probe_bytes = Q * (20 + fs.mask_bytes) + filt_bytes           # 21.16 B/key
    build_bytes = T * N * 20 + int(lens.cpu().numpy().sum())       # 21.25 B/key
    probe_gbs = probe_bytes / (probe_ms * 1e-3) / 1e9
    build_gbs = build_bytes / (build_ms * 1e-3) / 1e9
    dominant = "probe" if probe_ms >= build_ms else "build"
    ach = probe_gbs if dominant == "probe" else build_gbs

    result = {
        "metric": "Bloom build+probe Mkeys/s (device-resident), 20B keys, 10 bits/key",
        "value": round(value, 2),
        "unit": "Mkeys/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic db_bench keys (GenerateKeyFromInt), mt19937_64 lookups",
        "config": {
            "workload": (f"per GPU: build {T} SSTable full filters x {N} keys (one batch) + probe "
                         f"{Q} lookups vs {F} stacked filters"),
            "key_bytes": 20, "bits_per_key": bpk, "tables": T, "keys_per_table": N,
            "lookups": Q, "filters": F, "parallelism": f"sstable-sharded x{world}, no collective",
            "path": {0: "auto", 1: "direct", 2: "sliced"}[args.path],
            "probe_round_keys": args.probe_round, "build_groups": args.build_groups,
            "probe_chunk_lg": args.probe_chunk_lg, "probe_slice_lg": args.probe_slice_lg,
        },
        "roofline": {
            "bound": "hbm", "kernel": f"{dominant} pass", "achieved": round(ach, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": None,
        },
        "build": {"ms": round(build_ms, 4), "mkeys_s": round(T * N / build_ms / 1e3, 1),
                  "alg_GBs": round(build_gbs, 1), "alg_bytes_per_key": round(build_bytes / (T * N), 3)},
        "probe": {"ms": round(probe_ms, 4), "mkeys_s": round(Q / probe_ms / 1e3, 1),
                  "alg_GBs": round(probe_gbs, 1), "alg_bytes_per_key": round(probe_bytes / Q, 3)},
    }

    traffic = load_traffic(args.traffic, result["config"], dominant)
    if traffic:
        result["roofline"]["traffic"] = traffic["traffic_bytes"]
        result["roofline"]["traffic_source"] = traffic["source"]
        result["roofline"]["traffic_alg_ratio"] = round(
            traffic["traffic_bytes"] / (probe_bytes if dominant == "probe" else build_bytes), 3)
    result["roofline"]["hbm_copy_GBs_measured"] = round(copy_bandwidth(dev, stream), 1)

    # ---- host-inclusive (PCIe) rate, N=1 only: recorded, never `value` ----
    if world == 1 and not args.no_e2e:
        result["e2e"] = e2e_rate(ctx, stream, tables, outs, lens, fs, qk, mask, bpk, dev)

    # ---- CPU baseline (oracle restatement, host cores), rank 0 at N=1 ----
    if world == 1 and rank == 0 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(args, tables, outs, lens, qk, mask, filters, N, T, bpk)

    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def load_traffic(path, config, dominant):
    """Per-launch fabric bytes of the dominant pass from a committed PMC
    summary (scripts/pmc_traffic.py), only if it was collected on this config."""
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return None
    if any(t["config"].get(k) != config.get(k) for k in t["config"]):
        return None
    d = t.get(dominant)
    return {"traffic_bytes": d["traffic_bytes"], "source": t["source"]} if d else None


def copy_bandwidth(dev, stream, nbytes=1 << 30, reps=10):
    """Measured device-to-device streaming rate (read + write bytes / s, GB/s)
    on this box: the achievable HBM ceiling beside the 8 TB/s spec peak."""
    import torch

    with torch.cuda.stream(stream):
        a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        b = torch.empty_like(a)
        b.copy_(a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            b.copy_(a)
        e1.record(stream)
    stream.synchronize()
    ms = e0.elapsed_time(e1) / reps
    del a, b
    return 2 * nbytes / (ms * 1e-3) / 1e9


def e2e_rate(ctx, stream, tables, outs, lens, fs, qk, mask, bpk, dev):
    """Keys start in pinned host memory, filters and masks end in pinned host
    memory (the RDMA slot / Get() caller), copies on the same stream."""
    import torch

    import dlsm_amd

    h_tabs = [t.data.cpu().pin_memory() for t in tables]
    h_q = qk.data.cpu().pin_memory()
    h_outs = [torch.empty_like(o, device="cpu").pin_memory() for o in outs]
    h_mask = torch.empty_like(mask, device="cpu").pin_memory()
    d_tabs = [torch.empty_like(t.data) for t in tables]
    d_q = torch.empty_like(qk.data)
    reps = 3
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        with torch.cuda.stream(stream):
            for d, h in zip(d_tabs, h_tabs):
                d.copy_(h, non_blocking=True)
            d_q.copy_(h_q, non_blocking=True)
        ctx.full_build_dev([dlsm_amd.Keys(d, t.n, 20) for d, t in zip(d_tabs, tables)], outs, lens, bpk)
        ctx.full_probe_dev(fs, dlsm_amd.Keys(d_q, qk.n, 20), mask)
        with torch.cuda.stream(stream):
            for h, o in zip(h_outs, outs):
                h.copy_(o, non_blocking=True)
            h_mask.copy_(mask, non_blocking=True)
        stream.synchronize()
    dt = (time.perf_counter() - t0) / reps
    nk = sum(t.n for t in tables) + qk.n
    return {"mkeys_s": round(nk / dt / 1e6, 1), "ms_per_step": round(dt * 1e3, 3),
            "note": "H2D keys + build + probe + D2H filters/masks, pinned host buffers"}


def cpu_baseline(args, tables, outs, lens, qk, mask, filters, N, T, bpk):
    """The oracle (clean-room C restatement with the reference's cost structure)
    on the host cores, on a bounded sample; also cross-checks the GPU output."""
    import numpy as np

    import oracle

    oracle.lib()
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    h_tabs = [t.data.cpu().numpy() for t in tables]
    h_filters = [f.cpu().numpy().tobytes() for f in filters]
    nq = min(args.cpu_probe_sample, qk.n)
    h_q = qk.data[: nq * 20].cpu().numpy()
    t0 = time.perf_counter()
    built = oracle.full_build_many(h_tabs, [N] * T, 20, bpk, threads)
    t1 = time.perf_counter()
    cmask = oracle.full_probe(h_filters, h_q, nq, nthreads=threads)
    t2 = time.perf_counter()
    # single-thread reference point on one table + 1M lookups
    s0 = time.perf_counter()
    oracle.full_build(h_tabs[0], N, bpk=bpk)
    s1 = time.perf_counter()
    n1 = min(1_000_000, nq)
    oracle.full_probe(h_filters, h_q[: n1 * 20], n1, nthreads=1)
    s2 = time.perf_counter()
    L = lens.cpu().numpy()
    gpu_filters = [outs[s][: int(L[s])].cpu().numpy().tobytes() for s in range(T)]
    gpu_mask = mask[:nq].cpu().numpy()
    parity = all(gpu_filters[s] == built[s] for s in range(T))
    parity = parity and bool(np.array_equal(gpu_mask, cmask))
    sample_keys = T * N + nq
    port = {
        "value": round(sample_keys / (t2 - t0) / 1e6, 2), "unit": "Mkeys/s", "cores": threads,
        "kind": "port",
        "sample": f"build {T}x{N} keys ({threads} threads, one table per thread) + probe {nq} "
                  f"lookups x {len(filters)} filters (re-hash per filter)",
        "build_mkeys_s": round(T * N / (t1 - t0) / 1e6, 2),
        "probe_mkeys_s": round(nq / (t2 - t1) / 1e6, 2),
        "single_thread": {"build_mkeys_s": round(N / (s1 - s0) / 1e6, 2),
                          "probe_mkeys_s": round(n1 / (s2 - s1) / 1e6, 2)},
        "host_cpu": cpu_model(),
        "gpu_output_matches_oracle": bool(parity),
    }
    # the reference's own bloom code (oracle/_ref/libref.so, built in place from
    # /root/reference by build()) on the same sample, when it travelled with the tree
    ref = oracle.ref_timed_baseline(h_tabs, N, h_filters, h_q, nq, bpk, threads)
    if ref is None:
        return port
    rb, rp, rbuilt, rmask = ref
    return {
        "value": round(sample_keys / (rb + rp) / 1e6, 2), "unit": "Mkeys/s", "cores": threads,
        "kind": "reference",
        "sample": port["sample"] + "; util/bloom_impl.h AddHash / HashMayMatch + util/hash.cc "
                  "compiled from the reference (full_filter_block.cc's bookkeeping restated)",
        "build_mkeys_s": round(T * N / rb / 1e6, 2),
        "probe_mkeys_s": round(nq / rp / 1e6, 2),
        "host_cpu": cpu_model(),
        "gpu_output_matches_reference": bool(all(gpu_filters[s] == rbuilt[s] for s in range(T))
                                             and np.array_equal(gpu_mask, rmask)),
        "port": port,
    }


if __name__ == "__main__":
    main()
