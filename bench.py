"""Headline benchmark: Bloom build+probe Mkeys/s (device-resident), 20 B keys,
10 bits/key -- BASELINE.json's metric.

One step = one pass of the path over one batch:
  * build: the 16 SSTable full filters of one flush/compaction round (12
    subcompaction + 4 flush outputs, 1.6 M db_bench keys each) in one
    device-resident batch call (dlsm_bloom_full_build_dev) -- configs[1]/[3];
  * probe: 100 M 20-byte lookups (v = mt19937_64(1000) mod 25.6 M) against 8
    stacked per-level full filters (dlsm_bloom_full_probe_dev) -- configs[2].

--gpus N > 1 is STRONG scaling, the north star's config 4: the SAME 16
SSTables split s mod N, the filter set replicated on every GPU, the ONE 100
M-key lookup stream split into N contiguous shards (dlsm_amd/sharding.py).
Two launch shapes, same work:
  * `python bench.py --gpus N`: ONE process, one host thread + dlsm_ctx +
    stream per GPU (dLSM's builders are threads of one
    process, db/db_impl.cc:3373-3386), dlsm_amd/multigpu.py.  Refuses to run
    when fewer than N GPUs are visible; --rehearse maps the N logical devices
    onto GPU 0 (a 1-GPU box runs the N-device code).
  * `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`:
    one process per GPU (RCCL only for the barrier, the max-over-ranks time and
    the one-time filter broadcast); --gpus must equal WORLD_SIZE.
--scaling weak (process mode) gives every rank its own 16 tables and 100 M
lookups instead.  value = (build keys + probe keys) of the whole job / wall
time of the slowest GPU.  A GPU whose build batch is under 16 M keys (strong
scaling at N >= 2) runs its build and probe on two streams (--overlap).

    python bench.py [--gpus N --steps K --warmup W] [--rehearse]
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
IC_RANDOM_ROW_GBS = 7900.0  # Infinity-Cache random-row gather, 151 MB table (MI355X_MICROARCH.md "Indexed rows")
# A rank's build batch below this many keys leaves the GPU partly idle (its
# kernels are latency-bound), so the step runs build and probe on two streams:
# +4 / +9 / +18 % per step at 12.8 / 6.4 / 3.2 M build keys, within +-1 % at
# the full 25.6 M (profiles/r02_overlap_shares.txt).


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
    ap.add_argument("--probe-serial", action="store_true",
                    help="probe rounds one after another on one stream (with --probe-round)")
    ap.add_argument("--build-groups", type=int, default=0, help="pipelined build job groups (0/1 = one group)")
    ap.add_argument("--probe-chunk-lg", type=int, default=13,
                    help="log2 keys per probe partition chunk (12..14; library default 13)")
    ap.add_argument("--probe-slice-lg", type=int, default=8,
                    help="log2 stacked lines per probe LDS slice (7, 8; library default 8)")
    ap.add_argument("--traffic", default=os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                      "profiles", "traffic.json"),
                    help="PMC traffic summary (scripts/pmc_traffic.py) reported as roofline.traffic "
                         "when its config matches this run")
    ap.add_argument("--scaling", choices=["auto", "strong", "weak"], default="auto",
                    help="strong (default: one fixed job split over the ranks) or weak (a job per rank)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the all-cores CPU baseline (0 = every host core)")
    ap.add_argument("--cpu-probe-sample", type=int, default=10_000_000)
    ap.add_argument("--overlap", choices=["auto", "on", "off"], default="auto",
                    help="run the step's build and probe on two streams (auto = on whenever the rank has "
                         "both; off = one stream, one pass after the other)")
    ap.add_argument("--cosched", type=int, default=0,
                    help="co-schedule build and probe on CU-masked streams: the build's slice pass on this "
                         "many CUs per XCD (1..4), every partition pass on the other CUs (0 = off)")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: capture one step (build + probe launches) in a HIP graph and replay it")
    ap.add_argument("--rehearse", action="store_true",
                    help="--gpus N in one process on a box with fewer GPUs: N logical devices on GPU 0")
    ap.add_argument("--python-loop", action="store_true",
                    help="issue the timed steps from a Python loop instead of the native runner")
    ap.add_argument("--native", action="store_true",
                    help="one process with a host thread per GPU, timed by the native runner "
                         "(dlsm_multi_device_run), even at N = 1 (the default shape for --gpus N > 1; at N = 1 "
                         "the default is this process's own native-runner loop, or the Python loop when an "
                         "A/B knob or --python-loop needs it)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-version", action="store_true",
                    help="skip the MultiGet-style version probe leg (SURVEY §8f row 3)")
    ap.add_argument("--no-mixed", action="store_true",
                    help="skip the realistic filter-set probe legs (mixed_set, dedup_shifted)")
    ap.add_argument("--no-block", action="store_true",
                    help="skip the sealed filter-block leg (full_build_block_dev: build + crc32c trailer)")
    ap.add_argument("--no-legacy", action="store_true",
                    help="skip the legacy-format leg (util/bloom.cc CreateFilter over the same tables)")
    args = ap.parse_args()

    # launch shape: torchrun (WORLD_SIZE set) = one process per GPU, and its
    # rank count must be the --gpus asked for; otherwise --gpus N > 1 = one
    # process with a host thread per GPU
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None and int(env_world) != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}: launch one rank per GPU "
            f"(--nproc-per-node {args.gpus}) or drop the launcher")
        sys.exit(2)
    if env_world is None and (args.gpus > 1 or args.native):
        sys.exit(run_threads(args))
    if args.rehearse and args.gpus == 1 and env_world is None:
        log("bench.py: --rehearse only applies to --gpus N > 1")

    import numpy as np
    import torch

    import dlsm_amd
    from dlsm_amd import sharding as SH
    from dlsm_amd.multigpu import event_stride

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
    # strong by default at every N (at N = 1 the two shapes are the same job)
    scaling = args.scaling if args.scaling != "auto" else "strong"

    N, T, Q, F, bpk = args.keys_per_table, args.tables, args.lookups, args.filters, args.bits_per_key

    def make_ctx():
        c = dlsm_amd.Context(local)
        c.set_path(args.path)
        if args.probe_round is not None:
            c.set_probe_round(args.probe_round)
        if args.probe_serial:
            c.set_probe_serial(True)
        c.set_build_groups(args.build_groups)
        c.set_probe_shape(args.probe_chunk_lg, args.probe_slice_lg)
        st = torch.cuda.Stream(device=dev)
        c.set_stream(st)
        return c, st

    ctx, stream = make_ctx()

    # ---- inputs, resident in HBM before timing ---------------------------
    t_in = time.time()
    work = SH.plan(rank, world, T, N, Q, scaling)
    inp = SH.make_inputs(ctx, work, N, F, bpk, dev, stream=stream, dist=dist)
    torch.cuda.synchronize()
    log(f"[rank {rank}] {scaling}: tables {work.tables}, lookups [{work.lookup_lo}, {work.lookup_hi}) "
        f"ready in {time.time() - t_in:.1f}s")
    tables, outs, lens, fs, qk, mask = inp.tables, inp.outs, inp.lens, inp.fs, inp.lookups, inp.mask

    # the build's context and stream: a second pair when the step overlaps
    # the build with the probe (their buffers are disjoint: the probe reads
    # the stacked filter set, the build writes the SSTable slots)
    overlap = bool(tables) and qk.n > 0 and args.overlap != "off"
    cosched = args.cosched if (tables and qk.n > 0) else 0
    part_stream = None
    if cosched:
        # the build's LDS-bound slice pass on a few CUs of every XCD (its own
        # context and stream), every HBM-bound partition pass -- build and
        # probe -- on the other CUs, the probe's slice / unpermute on all
        overlap = True
        n_cus = torch.cuda.get_device_properties(dev).multi_processor_count
        small = dlsm_amd.cu_subset(cosched, n_cus)
        big = sorted(set(range(n_cus)) - set(small))
        ctx_b = dlsm_amd.Context(local)
        ctx_b.set_path(args.path)
        stream_b = dlsm_amd.cu_mask_stream(local, small, n_cus)
        part_stream = dlsm_amd.cu_mask_stream(local, big, n_cus)
        ctx_b.set_stream(stream_b)
        for c in (ctx, ctx_b):
            c.set_partition_stream(part_stream, len(big))
    else:
        ctx_b, stream_b = make_ctx() if overlap else (ctx, stream)

    def step():
        if tables:
            ctx_b.full_build_dev(tables, outs, lens, bpk)
        if qk.n:
            ctx.full_probe_dev(fs, qk, mask)

    # The timed steps run from the library's native runner (a C++ loop issuing
    # the same calls, dlsm_multi_device_run) unless an A/B knob needs the
    # Python loop (HIP graph, co-scheduling, probe rounds, build groups) or
    # --python-loop asks for it; the Python loop costs 3 % of the step on
    # these boxes (profiles/r03_d_native_shares.txt vs r03_a_bench.json).
    # Under a launcher (one process per GPU) each rank times its own GPU's
    # steps with the same runner, between a barrier and the max over ranks.
    use_native = (not args.python_loop and not args.graph and not cosched
                  and args.probe_round is None and not args.probe_serial and not args.build_groups)
    if use_native:
        from dlsm_amd import multigpu as MG

        dwork, _keep = MG.device_work(ctx, ctx_b, inp)
        if dist:
            # warm-up first, then a barrier right before the timed steps
            if args.warmup:
                MG.native_run([dwork], args.warmup, 0, bpk, event_every=args.warmup)
            dist.barrier()
            elapsed, passes = MG.native_run([dwork], args.steps, 0, bpk)
        else:
            elapsed, passes = MG.native_run([dwork], args.steps, args.warmup, bpk)
        own_elapsed = elapsed
        elapsed = SH.max_over_ranks(elapsed, dist, dev)
        build_ms = float(np.mean([b for b, _ in passes]))
        probe_ms = float(np.mean([p for _, p in passes]))
        enqueue_s = float("nan")
    for _ in range(0 if use_native else args.warmup):
        step()
    ctx.sync()
    ctx_b.sync()
    graph = None
    if args.graph and not overlap:
        # the step's launches captured once (the warm-up sized every
        # workspace, so the capture allocates nothing and uploads nothing)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream, capture_error_mode="relaxed"):
            step()
        graph.replay()
        stream.synchronize()

    # ---- timed region (Python loop) ---------------------------------------
    def ev():
        return torch.cuda.Event(enable_timing=True)

    # the passes of every `every`-th timed step are bracketed with events (an
    # event pair at a call boundary idles the GPU for several microseconds:
    # timing every step would lengthen the steps being timed,
    # profiles/r03_o_pass_events_ab.txt)
    every = event_stride(args.steps)
    evs = [(ev(), ev(), ev(), ev()) for _ in range(0 if use_native else args.steps)]
    sampled = [i % every == every - 1 for i in range(args.steps)]
    gate = torch.cuda.Event()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pass_events = graph is None
    for i in range(0 if use_native else args.steps):
        if graph is not None:
            graph.replay()
            continue
        tev = pass_events and sampled[i]
        if tev:
            if overlap:  # a sampled step runs its passes alone (as dlsm_multi_device_run_sampled)
                gate.record(stream)
                stream_b.wait_event(gate)
            evs[i][0].record(stream_b)
        if tables:
            ctx_b.full_build_dev(tables, outs, lens, bpk)
        if tev:
            evs[i][1].record(stream_b)
            if overlap:
                stream.wait_event(evs[i][1])
            evs[i][2].record(stream)
        if qk.n:
            ctx.full_probe_dev(fs, qk, mask)
        if tev or cosched:
            evs[i][3].record(stream)
        if tev and overlap:
            stream_b.wait_event(evs[i][3])
        if cosched:
            # the next build partition starts behind this probe's slice /
            # unpermute passes (co-running with them slows both)
            w = torch.cuda.Event()
            w.record(stream)
            stream_b.wait_event(w)
    if not use_native:
        enqueue_s = time.perf_counter() - t0  # host time to submit the K steps
        stream.synchronize()
        stream_b.synchronize()
        if part_stream is not None:
            part_stream.synchronize()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        own_elapsed = elapsed
        elapsed = SH.max_over_ranks(elapsed, dist, dev)
    if not use_native and (cosched or not pass_events):
        # co-scheduled passes overlap, so the per-pass times (roofline) come
        # from the same K steps run one pass after another on one stream
        ctx.set_partition_stream(None)
        for i in range(args.steps):
            evs[i][0].record(stream)
            ctx.full_build_dev(tables, outs, lens, bpk)
            evs[i][1].record(stream)
            evs[i][2].record(stream)
            ctx.full_probe_dev(fs, qk, mask)
            evs[i][3].record(stream)
        stream.synchronize()
    if not use_native:
        if not pass_events or cosched:
            sampled = [True] * args.steps  # the instrumented re-run above timed every step
        build_ms = float(np.mean([e[0].elapsed_time(e[1]) for e, t in zip(evs, sampled) if t]))
        probe_ms = float(np.mean([e[2].elapsed_time(e[3]) for e, t in zip(evs, sampled) if t]))

    # keys of the whole job per step (every rank's share)
    rank_keys = len(tables) * N + qk.n
    job_keys = (T * N + Q) if scaling == "strong" else (T * N + Q) * world
    value = job_keys * args.steps / elapsed / 1e6
    filt_bytes = sum(int(f.numel()) for f in inp.filters)
    nb = max(1, len(tables) * N)
    probe_bytes = qk.n * (20 + fs.mask_bytes) + filt_bytes           # 21.16 B/key
    build_bytes = len(tables) * N * 20 + int(lens.cpu().numpy()[: len(tables)].sum())  # 21.25 B/key
    probe_gbs = probe_bytes / (probe_ms * 1e-3) / 1e9
    build_gbs = build_bytes / (build_ms * 1e-3) / 1e9
    dominant = "probe" if probe_ms >= build_ms else "build"
    ach = probe_gbs if dominant == "probe" else build_gbs
    if scaling == "strong":
        par = f"strong: {T} SSTables split s mod {world}, filters replicated, {Q} lookups sharded x{world}"
        wl = (f"build {T} SSTable full filters x {N} keys (one batch) + probe {Q} lookups vs {F} "
              f"stacked filters, split over {world} GPU(s)")
    else:
        par = f"weak: sstable-sharded x{world}, no collective"
        wl = (f"per GPU: build {T} SSTable full filters x {N} keys (one batch) + probe "
              f"{Q} lookups vs {F} stacked filters")

    result = {
        "metric": "Bloom build+probe Mkeys/s (device-resident), 20B keys, 10 bits/key",
        "value": round(value, 2),
        "unit": "Mkeys/s",
        "n_gpus": world,
        # ranks sharing a GPU (DLSM_BENCH_BACKEND=gloo on a smaller box) rehearse
        # the N-GPU path: such a line is not an N-GPU measurement
        "rehearsed": world > torch.cuda.device_count(),
        "physical_devices": min(world, torch.cuda.device_count()),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic db_bench keys (GenerateKeyFromInt), mt19937_64 lookups",
        "config": {
            "workload": wl,
            "key_bytes": 20, "bits_per_key": bpk, "tables": T, "keys_per_table": N,
            "lookups": Q, "filters": F, "parallelism": par,
            "rank0_tables": work.tables, "rank0_lookups": qk.n,
            "path": {0: "auto", 1: "direct", 2: "sliced"}[args.path],
            "probe_round_keys": args.probe_round, "probe_serial": args.probe_serial,
            "build_groups": args.build_groups,
            "overlap": overlap,
            "hip_graph": graph is not None,
            "timed_by": "dlsm_multi_device_run (C++ loop)" if use_native else "Python loop",
            "pass_events_every": event_stride(args.steps),
            "cosched_build_slice_cus_per_xcd": cosched,
            "probe_chunk_lg": args.probe_chunk_lg, "probe_slice_lg": args.probe_slice_lg,
        },
        "roofline": {
            "bound": "hbm", "kernel": f"{dominant} pass (rank 0's share)", "achieved": round(ach, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": None,
            **pass_timing_note(overlap, every),
            **step_roofline(probe_bytes + build_bytes, elapsed / args.steps),
        },
        "host_enqueue_ms_per_step": None if use_native else round(enqueue_s / args.steps * 1e3, 4),
        "build": {"ms": round(build_ms, 4), "mkeys_s": round(nb / build_ms / 1e3, 1),
                  "alg_GBs": round(build_gbs, 1), "alg_bytes_per_key": round(build_bytes / nb, 3)},
        "probe": {"ms": round(probe_ms, 4), "mkeys_s": round(max(1, qk.n) / probe_ms / 1e3, 1),
                  "alg_GBs": round(probe_gbs, 1), "alg_bytes_per_key": round(probe_bytes / max(1, qk.n), 3)},
    }
    del rank_keys

    # the committed PMC traffic is for the whole job on one GPU: a rank's
    # share at N > 1 is not what was counted, so it is reported only at N = 1
    traffic = load_traffic(args.traffic, result["config"], dominant) if world == 1 else None
    if traffic:
        result["roofline"]["traffic"] = traffic["traffic_bytes"]
        result["roofline"]["traffic_source"] = traffic["source"]
        result["roofline"]["traffic_alg_ratio"] = round(
            traffic["traffic_bytes"] / (probe_bytes if dominant == "probe" else build_bytes), 3)
    ceil, shapes = stream_ceilings(dev, stream)
    result["roofline"]["hbm_read_GBs_measured"] = ceil["read"]
    result["roofline"]["hbm_copy_GBs_measured"] = ceil["copy"]
    result["roofline"]["frac_of_measured_read"] = round(ach / ceil["read"], 4)
    result["roofline"]["frac_of_measured_copy"] = round(ach / ceil["copy"], 4)
    result["roofline"]["ceiling_kernels"] = ("dlsm_stream_kernel, best of plain/nt x grid-stride/chunked x "
                                             f"1-4K workgroups of 512: {shapes}")

    # ---- host-inclusive (PCIe) rate, N=1 only: recorded, never `value` ----
    if world == 1 and not args.no_e2e:
        result["e2e"] = e2e_rate(ctx, stream, tables, outs, lens, fs, qk, mask, bpk, dev)
        L = lens.cpu().numpy()
        ref = ([outs[s][: int(L[s])].cpu().numpy().tobytes() for s in range(len(tables))], mask.cpu().numpy())
        result["e2e_hashed"] = e2e_hashed_rate(ctx, stream, tables, fs, qk, bpk, dev, ref)
        # the same build with the job table changing every call (a flush
        # stream hands over new tables each time: the upload is paid)
        result["build"]["rotating_batches_ms"] = round(rotating_build_ms(ctx, stream, tables, outs, lens, bpk), 4)
        # the other step shape (two streams if the timed step was sequential):
        # recorded beside `value`
        result["other_step_shape"] = other_shape_rate(args, ctx, stream, tables, outs, lens, fs, qk, mask, bpk,
                                                      local, elapsed / args.steps, overlap)

    # ---- legacy FilterPolicy format over the same tables (config 2's
    # "bit-exact vs util/bloom.cc"), N=1: recorded beside `value` ----
    legacy_out = None
    if world == 1 and tables and not args.no_legacy:
        result["legacy"], legacy_out = legacy_leg(ctx, stream, tables, bpk)
        lt = load_traffic(args.traffic, result["config"], "legacy") if world == 1 else None
        if lt:  # PMC fabric bytes of one legacy batch build (partition + slice)
            result["legacy"]["traffic"] = lt["traffic_bytes"]
            result["legacy"]["traffic_alg_ratio"] = round(
                lt["traffic_bytes"] / (result["legacy"]["alg_bytes_per_key"] * len(tables) * tables[0].n), 3)

    # ---- the sealed filter block, N=1: recorded ----
    if world == 1 and tables and not args.no_block:
        result["block"] = block_leg(ctx, stream, tables, bpk)
        bt = load_traffic(args.traffic, result["config"], "block")
        if bt:  # PMC fabric bytes of one sealed batch build (partition + slice + seal)
            result["block"]["traffic"] = bt["traffic_bytes"]
            result["block"]["traffic_alg_ratio"] = round(
                bt["traffic_bytes"] / (result["block"]["alg_bytes_per_key"] * len(tables) * tables[0].n), 3)

    # ---- the read shapes a Version presents, N=1:
    # recorded beside `value` ----
    if world == 1 and not args.no_version:
        result["version_probe"] = version_leg(ctx, stream, dev)
        vt = load_traffic(args.traffic, result["config"], "version")
        if vt:  # fabric bytes (L2 misses, Infinity-Cache hits included) per call
            vp = result["version_probe"]
            vp["traffic"] = vt["traffic_bytes"]
            vp["traffic_alg_ratio"] = round(vt["traffic_bytes"] / (vp["alg_bytes_per_get"] * vp["lookups"]), 3)
            # the bytes the kernel does move (filter lines past L2 dominate) per
            # second, against the same 8 TB/s: what bounds it, unlike `frac`
            vp["traffic_GBs"] = round(vt["traffic_bytes"] / (vp["ms"] * 1e-3) / 1e9, 1)
            vp["traffic_frac"] = round(vp["traffic_GBs"] / HBM_PEAK_GBS, 4)
            # Floor: the filter lines fetched past L2 (the call's PMC fetch
            # bytes less its streamed key reads) at the guide's Infinity-Cache
            # random-row rate, or the pass without filters, whichever is longer
            # (MI355X_MICROARCH.md "Indexed rows": 7.4-7.9 TB/s from a 151 MB
            # table of uniformly random rows; 1,152-B rows there, 128-B lines
            # here, so it is a lower bound)
            line_bytes = max(0, vt["fetch_bytes"] - vp["lookups"] * 20)
            lines_ms = line_bytes / IC_RANDOM_ROW_GBS / 1e9 * 1e3
            vp["lines_past_l2_per_get"] = round(line_bytes / 128 / vp["lookups"], 3)
            vp["floor_ms"] = round(max(lines_ms, vp["nofilter_ms"]), 4)
            vp["floor_parts_ms"] = {"lines_past_l2_at_ic_rate": round(lines_ms, 4), "nofilter": vp["nofilter_ms"]}
            vp["ms_over_floor"] = round(vp["ms"] / vp["floor_ms"], 3)
    if world == 1 and not args.no_mixed:
        for name, sizes in SHAPE_LEGS.items():
            rec = shape_leg(ctx, stream, dev, qk, bpk, sizes)
            st = load_traffic(args.traffic, result["config"], name)
            if st:  # PMC fabric bytes of one call (partition + slice + unpermute)
                rec["traffic"] = st["traffic_bytes"]
                rec["traffic_alg_ratio"] = round(st["traffic_bytes"] / (rec["alg_bytes_per_key"] * rec["lookups"]), 3)
            result[name] = rec

    # ---- CPU baseline (host cores), rank 0 at N=1 ----
    if dist:  # every rank's share, so the N-GPU line shows each GPU's passes
        mine = gpu_share_record(rank, local, len(tables) * N, qk.n, build_bytes, probe_bytes,
                                [(build_ms, probe_ms)], own_elapsed, args.steps)
        recs = [None] * world
        dist.all_gather_object(recs, mine)
        result["per_gpu"] = recs
        result["imbalance"] = imbalance(recs)
    if world == 1 and rank == 0 and not args.no_cpu:
        filters = [f for f in inp.filters]
        L = lens.cpu().numpy()
        gpu_filters = [outs[s][: int(L[s])].cpu().numpy().tobytes() for s in range(T)]
        result["cpu_baseline"] = cpu_baseline(args, tables, gpu_filters, qk, mask, filters, N, T, bpk,
                                              legacy_out=legacy_out)

    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def run_threads(args) -> int:
    """--gpus N in one process: a host thread + dlsm_ctx + stream per GPU
    (dlsm_amd/multigpu.py) timed by the native runner, strong scaling of
    config 4 (N = 1 with --native).  Returns the exit code."""
    import numpy as np
    import torch

    from dlsm_amd import multigpu as MG

    N_GPU = args.gpus
    available = torch.cuda.device_count()  # counting does not initialise the GPU
    try:
        devices = MG.device_map(N_GPU, args.rehearse, available)
    except MG.DeviceCountError as e:
        log(f"bench.py: {e}")
        return 2
    if args.scaling == "weak":
        log("bench.py: --scaling weak needs the process launcher (torchrun); one process runs strong scaling")
        return 2
    if args.cosched or args.graph or args.probe_round is not None or args.build_groups:
        log("bench.py: --cosched / --graph / --probe-round / --build-groups are single-GPU A/B knobs")
        return 2
    N, T, Q, F, bpk = args.keys_per_table, args.tables, args.lookups, args.filters, args.bits_per_key
    from dlsm_amd import workload as W

    t_in = time.time()
    stream_vals = W.mt19937_64(1000, Q) % np.uint64(2 * F * N)  # the ONE lookup stream, generated once
    opts = MG.WorkerOptions(path=args.path, probe_chunk_lg=args.probe_chunk_lg, probe_slice_lg=args.probe_slice_lg,
                            overlap=args.overlap, pass_events=True)
    workers = MG.build_workers(N_GPU, devices, T, N, Q, F, bpk, opts, lookup_stream=stream_vals)
    digests = {w.filter_digest() for w in workers}
    if len(digests) != 1:
        log("bench.py: the devices' filter sets differ")
        return 3
    for w in workers:
        log(f"[gpu {w.rank} -> device {w.device}] tables {w.work.tables}, lookups "
            f"[{w.work.lookup_lo}, {w.work.lookup_hi}), overlap {w.overlap}")
    log(f"inputs ready in {time.time() - t_in:.1f}s")
    # the timed steps run from the library's native runner: a std::thread per
    # device, host barriers around the timed region, every device's passes
    # timed on the sampled steps (dlsm_multi_device_run_timed)
    elapsed, passes, dev_s = MG.native_timed_run(workers, args.steps, args.warmup, bpk)
    per_gpu = []
    for w, ps, ds in zip(workers, passes, dev_s):
        inp = w.inp
        per_gpu.append(gpu_share_record(w.rank, w.device, len(inp.tables) * N, inp.lookups.n,
                                        len(inp.tables) * N * 20 + int(inp.lens.cpu().numpy()[: len(inp.tables)].sum()),
                                        inp.lookups.n * (20 + inp.fs.mask_bytes) + sum(int(f.numel()) for f in inp.filters),
                                        ps, ds, args.steps))
    result = threads_line(args, N_GPU, devices, workers, per_gpu, elapsed, T, N, Q, F, bpk)
    if not args.no_cpu:
        # the CPU baseline once, from this process, on the job's first tables
        # and GPU 0's lookup shard (bounded sample, as at N = 1)
        order = sorted((s, w, j) for w in workers for j, s in enumerate(w.work.tables))
        tabs = [w.inp.tables[j] for _, w, j in order]
        gpu_filters = [w.inp.outs[j][: int(w.inp.lens.cpu().numpy()[j])].cpu().numpy().tobytes() for _, w, j in order]
        w0 = workers[0]
        result["cpu_baseline"] = cpu_baseline(args, tabs, gpu_filters, w0.inp.lookups, w0.inp.mask,
                                              list(w0.inp.filters), N, len(tabs), bpk)
    print(json.dumps(result), flush=True)
    for w in workers:
        w.close()
    return 0


def gpu_share_record(rank, device, build_keys, probe_keys, build_bytes, probe_bytes, passes, device_s, steps):
    """One GPU's share of the N-GPU job: its sampled pass times (HIP events on
    its own streams), algorithmic bytes and rates, and its own time over the
    timed steps."""
    import numpy as np

    b = float(np.mean([x for x, _ in passes])) if passes else float("nan")
    p = float(np.mean([y for _, y in passes])) if passes else float("nan")
    rec = {"gpu": rank, "device": device, "build_keys": build_keys, "probe_keys": probe_keys,
           "build_ms": round(b, 4), "probe_ms": round(p, 4),
           "build_alg_GBs": round(build_bytes / (b * 1e-3) / 1e9, 1) if build_keys and b > 0 else None,
           "probe_alg_GBs": round(probe_bytes / (p * 1e-3) / 1e9, 1) if probe_keys and p > 0 else None,
           "ms_per_step": round(device_s / steps * 1e3, 4), "sampled_steps": len(passes)}
    for k in ("build", "probe"):
        g = rec[k + "_alg_GBs"]
        rec[k + "_frac"] = round(g / HBM_PEAK_GBS, 4) if g else None
    return rec


def threads_line(args, n_gpu, devices, workers, per_gpu, elapsed, T, N, Q, F, bpk):
    """The bench line of `--gpus N` (one process, a host thread per GPU): the
    whole job's rate, every GPU's share (pass times, rates, own step time) and
    the imbalance between them; the roofline is the dominant pass of the
    slowest GPU's share."""
    value = (T * N + Q) * args.steps / elapsed / 1e6
    slow = max(per_gpu, key=lambda r: r["ms_per_step"])
    dominant = "probe" if (slow["probe_ms"] or 0) >= (slow["build_ms"] or 0) else "build"
    ach = slow[dominant + "_alg_GBs"] or 0.0
    step_bytes = sum(r["build_keys"] * 21.25 + r["probe_keys"] * 21.16 for r in per_gpu)
    return {
        "metric": "Bloom build+probe Mkeys/s (device-resident), 20B keys, 10 bits/key",
        "value": round(value, 2),
        "unit": "Mkeys/s",
        "n_gpus": n_gpu,
        # --rehearse maps the N logical devices onto fewer physical ones: such a
        # line is not an N-GPU measurement
        "rehearsed": bool(args.rehearse),
        "physical_devices": len(set(devices)),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic db_bench keys (GenerateKeyFromInt), mt19937_64 lookups",
        "config": {
            "workload": (f"build {T} SSTable full filters x {N} keys + probe {Q} lookups vs {F} stacked "
                         f"filters, split over {n_gpu} GPUs"),
            "key_bytes": 20, "bits_per_key": bpk, "tables": T, "keys_per_table": N,
            "lookups": Q, "filters": F,
            "parallelism": (f"strong: {T} SSTables split s mod {n_gpu}, filters replicated, {Q} lookups "
                            f"sharded x{n_gpu}; one process, one host thread + context + stream per GPU"),
            "launch": "threads (dlsm_multi_device_run_timed)",
            "pass_events_every": event_stride_of(args.steps),
            "devices": devices,
            "rehearsal": bool(args.rehearse),
            "gpu_tables": [w.work.tables for w in workers],
            "gpu_lookups": [[w.work.lookup_lo, w.work.lookup_hi] for w in workers],
            "overlap": [w.overlap for w in workers],
            "path": {0: "auto", 1: "direct", 2: "sliced"}[args.path],
            "probe_chunk_lg": args.probe_chunk_lg, "probe_slice_lg": args.probe_slice_lg,
        },
        "roofline": {
            "bound": "hbm", "kernel": f"{dominant} pass of the slowest GPU's share (gpu {slow['gpu']})",
            "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": None,
            "traffic_note": "PMC traffic is committed for the one-GPU job only (profiles/traffic.json)",
            **pass_timing_note(any(w.overlap for w in workers), event_stride_of(args.steps)),
            **step_roofline(step_bytes, elapsed / args.steps),
        },
        "per_gpu": per_gpu,
        "imbalance": imbalance(per_gpu),
        "build": {"ms": slow["build_ms"], "note": "slowest GPU's share; per_gpu has every GPU"},
        "probe": {"ms": slow["probe_ms"], "note": "slowest GPU's share; per_gpu has every GPU"},
    }


def imbalance(per_gpu):
    """Slowest vs fastest GPU of an N-GPU line (by each GPU's own step time)."""
    slow = max(per_gpu, key=lambda r: r["ms_per_step"])
    fast = min(per_gpu, key=lambda r: r["ms_per_step"])
    return {"slowest_gpu": slow["gpu"], "fastest_gpu": fast["gpu"],
            "max_over_min_ms_per_step": round(slow["ms_per_step"] / fast["ms_per_step"], 4)
            if fast["ms_per_step"] > 0 else None,
            "max_minus_min_ms_per_step": round(slow["ms_per_step"] - fast["ms_per_step"], 4)}


def event_stride_of(steps):
    from dlsm_amd.multigpu import event_stride

    return event_stride(steps)


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
    return ({"traffic_bytes": d["traffic_bytes"], "fetch_bytes": d.get("fetch_bytes", 0),
             "write_bytes": d.get("write_bytes", 0), "source": t["source"]} if d else None)


def stream_ceilings(dev, stream, nbytes=1 << 31, reps=5):
    """The box's own HBM streaming ceilings, measured in this run with the
    library's 16-byte-per-lane kernels (dlsm_stream_kernel): the best of the
    read-only and of the copy shapes (plain / non-temporal, grid-stride /
    one range per workgroup, 1-4 K workgroups).  GB/s of bytes moved (copy:
    read + write)."""
    import ctypes

    import torch

    import dlsm_amd

    fn = dlsm_amd.lib().dlsm_stream_kernel
    src = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    raw = ctypes.c_void_p(stream.cuda_stream)
    best = {}
    for kind, name in ((0, "read"), (1, "copy")):
        for variant in range(4):
            for blocks in (1024, 2048, 4096):
                args = (raw, kind, variant, ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                        ctypes.c_uint64(nbytes), ctypes.c_uint32(blocks))
                if fn(*args) != 0:
                    raise RuntimeError("dlsm_stream_kernel failed")
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(reps):
                    fn(*args)
                e1.record(stream)
                stream.synchronize()
                ms = e0.elapsed_time(e1) / reps
                gbs = nbytes * (1 + kind) / (ms * 1e-3) / 1e9
                if gbs > best.get(name, (0,))[0]:
                    best[name] = (gbs, {"variant": variant, "blocks": blocks, "ms": round(ms, 4)})
    del src, dst
    return {k: round(v[0], 1) for k, v in best.items()}, {k: v[1] for k, v in best.items()}


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


def e2e_hashed_rate(ctx, stream, tables, fs, qk, bpk, dev, ref, chunk_keys=12_500_000, reps=3, table_group=4):
    """Host-inclusive rate with part of the hashing on the host, as the
    reference does it (BloomHash in AddKey and in KeyMayMatch,
    full_filter_block.cc:45,271).  Keys start in pinned host memory; filters
    and masks end in pinned host memory.  Two feeds run at once:
      - host-hashed keys: the host's cores hash them (dlsm_bloom_hash_batch,
        inside the timed region) -- the build's tables first (one hashed
        batch build, dlsm_bloom_full_build_hashed_dev), then lookups in
        chunks (hashed probe, dlsm_bloom_full_probe_hashed_dev), each chunk's
        4 B/key copy and kernels running while the host hashes the next (a
        pinned hash slot per key: no staging to wait for);
      - raw keys: the remaining tables and lookups go H2D as 20-byte keys on
        a second context and stream, hashed on the GPU (the DMA engines read
        them, not the host's cores).
    Every key is read from host DRAM once either way (20 B); the split puts
    as many keys on the host's cores as their hash rate allows while the PCIe
    link carries the rest: it is set from the hash rate and the H2D rate
    measured in the warm-up (time on the cores = time on the link).  D2H
    copies run on a third stream (PCIe is full duplex).  `ref` = (filters,
    mask) of the device-resident run: the outputs are checked against them."""
    import numpy as np
    import torch

    import dlsm_amd

    T, N, Q = len(tables), tables[0].n, qk.n
    mb = fs.mask_bytes
    h_tabs = [t.data.cpu().pin_memory() for t in tables]
    tab_np = [h.numpy() for h in h_tabs]
    h_q = qk.data.cpu().pin_memory()
    q_np = h_q.numpy()
    hb = torch.empty(Q, dtype=torch.int32).pin_memory()     # lookups' hashes
    hb_np = hb.numpy()
    hbt = torch.empty(T * N, dtype=torch.int32).pin_memory()  # tables' hashes
    hbt_np = hbt.numpy()
    db = torch.empty(Q, dtype=torch.int32, device=dev)
    dbt = torch.empty(T * N, dtype=torch.int32, device=dev)
    d_tabs = [torch.empty_like(t.data) for t in tables]
    d_q = torch.empty_like(qk.data)
    outs = [torch.zeros(dlsm_amd.full_size(t.n, bpk)[0] + 16, dtype=torch.uint8, device=dev) for t in tables]
    lens = torch.zeros(T, dtype=torch.uint64, device=dev)
    h_outs = [torch.empty_like(o, device="cpu").pin_memory() for o in outs]
    h_lens = torch.empty(T, dtype=torch.uint64).pin_memory()
    mask = torch.empty(Q * mb, dtype=torch.uint8, device=dev)
    h_mask = torch.empty(Q * mb, dtype=torch.uint8).pin_memory()
    s_raw = torch.cuda.Stream(device=dev)
    s_out = torch.cuda.Stream(device=dev)
    ctx_raw = dlsm_amd.Context(dev.index or 0)
    ctx_raw.set_stream(s_raw)

    def to_host(lo_t, hi_t, lo_q, hi_q, st):
        """D2H of tables [lo_t, hi_t) and lookups [lo_q, hi_q), behind st's work."""
        done = torch.cuda.Event()
        done.record(st)
        s_out.wait_event(done)
        with torch.cuda.stream(s_out):
            for s_ in range(lo_t, hi_t):
                h_outs[s_].copy_(outs[s_], non_blocking=True)
            if hi_t > lo_t:
                h_lens[lo_t:hi_t].copy_(lens[lo_t:hi_t], non_blocking=True)
            if hi_q > lo_q:
                h_mask[lo_q * mb:hi_q * mb].copy_(mask[lo_q * mb:hi_q * mb], non_blocking=True)

    def one_step(raw_t, raw_q):
        """Tables [0, raw_t) and lookups [0, raw_q) go as keys; tables
        [raw_t, T) and lookups [raw_q, Q) are hashed on the host."""
        hash_s = 0.0
        with torch.cuda.stream(s_raw):  # the raw feed, queued up front
            for s_ in range(raw_t):
                d_tabs[s_].copy_(h_tabs[s_], non_blocking=True)
            if raw_q:
                d_q[: raw_q * 20].copy_(h_q[: raw_q * 20], non_blocking=True)
        if raw_t:
            ctx_raw.full_build_dev([dlsm_amd.Keys(d_tabs[s_], N, 20) for s_ in range(raw_t)], outs[:raw_t],
                                   lens[:raw_t], bpk)
        if raw_q:
            ctx_raw.full_probe_dev(fs, dlsm_amd.Keys(d_q[: raw_q * 20], raw_q, 20), mask[: raw_q * mb])
        to_host(0, raw_t, 0, raw_q, s_raw)
        # the hashed tables in groups of `table_group`: each group's 4 B/key
        # copy and batched build run while the host hashes the next group
        for g0 in range(raw_t, T, table_group):
            g1 = min(T, g0 + table_group)
            t0 = time.perf_counter()
            for s_ in range(g0, g1):
                dlsm_amd.hash_batch(dlsm_amd.Keys(tab_np[s_], N, 20), out=hbt_np[s_ * N:(s_ + 1) * N])
            hash_s += time.perf_counter() - t0
            with torch.cuda.stream(stream):
                dbt[g0 * N:g1 * N].copy_(hbt[g0 * N:g1 * N], non_blocking=True)
            ctx.full_build_hashed_dev([dbt[s_ * N:(s_ + 1) * N] for s_ in range(g0, g1)], outs[g0:g1],
                                      lens[g0:g1], bpk)
            to_host(g0, g1, 0, 0, stream)
        for lo in range(raw_q, Q, chunk_keys):
            hi = min(Q, lo + chunk_keys)
            n = hi - lo
            t0 = time.perf_counter()
            dlsm_amd.hash_batch(dlsm_amd.Keys(q_np[lo * 20:hi * 20], n, 20), out=hb_np[lo:hi])
            hash_s += time.perf_counter() - t0
            with torch.cuda.stream(stream):
                db[lo:hi].copy_(hb[lo:hi], non_blocking=True)
            ctx.full_probe_hashed_dev(fs, db[lo:hi], mask[lo * mb:hi * mb], n)
            to_host(0, 0, lo, hi, stream)
        stream.synchronize()
        s_raw.synchronize()
        s_out.synchronize()
        return hash_s

    # warm-up: workspaces, pool threads, and the two rates the split is set
    # by (half the lookups and every table hashed on the host)
    hs = one_step(0, Q // 2)
    hash_rate = (T * N + Q - Q // 2) / max(hs, 1e-9)  # keys/s on the host's cores
    one_step(T, Q)  # the raw feed's workspaces
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s_raw):
        d_q.copy_(h_q, non_blocking=True)
    s_raw.synchronize()
    h2d_Bps = h_q.numel() / (time.perf_counter() - t0)
    raw_t, raw_q = e2e_split(T, N, Q, hash_rate, h2d_Bps)
    K = T * N + Q
    one_step(raw_t, raw_q)
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        one_step(raw_t, raw_q)
        times.append(time.perf_counter() - t0)
    dt = float(np.median(times))
    L = h_lens.numpy()
    ref_filters, ref_mask = ref
    ok = (all(h_outs[s_][: int(L[s_])].numpy().tobytes() == ref_filters[s_] for s_ in range(T))
          and bool(np.array_equal(h_mask.numpy(), ref_mask)))
    ctx_raw.close()
    hashed = (T - raw_t) * N + (Q - raw_q)
    # the host's own bound: every key's 20 bytes come out of host DRAM once
    # (the cores read the hashed ones, the DMA engines the raw ones) and each
    # hashed key's 4 B hash is written and read back by the DMA; against the
    # host's streaming read rate measured now, on the same cores
    host_bytes = 20 * K + 8 * hashed
    # the cores' own share of those bytes: each hashed key's 20 B read and its
    # 4 B hash written (the DMA engines read the rest); this is what the cores'
    # read ceiling bounds
    core_bytes = 24 * hashed
    host_read = host_read_rate(h_q)
    return {"mkeys_s": round(K / dt / 1e6, 1), "ms_per_step": round(dt * 1e3, 3),
            "host_bytes_per_step": host_bytes, "host_GBs": round(host_bytes / dt / 1e9, 2),
            "host_read_GBs_measured": host_read["GBs"], "host_read_method": host_read["method"],
            "frac_of_host_read": round(host_bytes / dt / 1e9 / host_read["GBs"], 4) if host_read["GBs"] else None,
            "host_core_bytes_per_step": core_bytes, "host_core_GBs": round(core_bytes / dt / 1e9, 2),
            "frac_of_host_read_cores": (round(core_bytes / dt / 1e9 / host_read["GBs"], 4)
                                        if host_read["GBs"] else None),
            "ms_per_step_reps": [round(x * 1e3, 3) for x in times],
            "host_hashed_keys": hashed, "raw_keys": K - hashed,
            "host_hashed_tables": T - raw_t, "host_hashed_lookups": Q - raw_q,
            "host_hash_gkeys_s": round(hash_rate / 1e9, 3), "h2d_GBs": round(h2d_Bps / 1e9, 1),
            "host_hash_threads": "all usable cores (dlsm_bloom_hash_batch pool)",
            "chunk_keys": chunk_keys, "h2d_bytes_per_key": {"host_hashed": 4, "raw": 20},
            "matches_device_resident": ok,
            "note": ("host BloomHash (timed) of as many keys as the host's cores keep up with -- the tables "
                     "first (hashed batch build), then lookups (hashed probe) -- 4 B/key H2D; the other keys "
                     "H2D as 20-byte keys on a second context and stream, hashed on the GPU; D2H filters/masks "
                     "on a third stream; pinned host buffers")}


def host_read_rate(buf, reps=5):
    """The host's read ceiling for the memory the host hashing reads: the
    pinned lookup-key buffer streamed by the same pool of threads, NUMA-placed
    the same way (dlsm_host_read_bytes: a 64-bit XOR fold, no hashing), best
    of `reps` after one warm pass.  GB/s."""
    import dlsm_amd

    n = (buf.numel() * buf.element_size()) // 8 * 8
    view = buf.view(-1)[: n // buf.element_size()] if buf.element_size() == 1 else buf
    best = 0.0
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        dlsm_amd.host_read_bytes(view)
        best = max(best, n / (time.perf_counter() - t0) / 1e9)
    return {"GBs": round(best, 1),
            "method": (f"dlsm_host_read_bytes over the {n >> 20} MiB pinned lookup-key buffer on the host-hash "
                       f"pool ({host_cores()} threads, NUMA-placed like the hashing), best of {reps}")}


def e2e_split(T, N, Q, hash_rate, h2d_Bps):
    """How many of a step's keys e2e_hashed sends raw: (raw tables, raw
    lookups).  H host-hashed keys of K = T N + Q balance the host's cores
    against the link: H / hash_rate = (20 (K - H) + 4 H) / h2d_Bps.  The
    tables are hashed first (their build is one call), then lookups; raw
    lookups are rounded to 4,096 keys."""
    K = T * N + Q
    H = (20 * K / h2d_Bps) / (1 / hash_rate + 16 / h2d_Bps)
    H = min(K, max(0.0, H))
    if H >= T * N:
        return 0, int(min(Q, max(0, round((K - H) / 4096) * 4096)))
    return T - int(round(H / N)), Q


def host_cores() -> int:
    """Host cores this process may use: the CPU affinity set, capped by a
    cgroup CPU quota when one is set (a GPU box's share of its host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_baseline(args, tables, gpu_filters, qk, mask, filters, N, T, bpk, legacy_out=None):
    """The CPU path timed on this box's host cores on a bounded sample of the
    bench workload, at T = 1 and T = all cores: the reference's own code
    (oracle/_ref/libref.so, built in place from /root/reference, when it
    travelled with the tree) else the oracle's C restatement -- `kind` says
    which.  Also cross-checks the GPU output against it."""
    import numpy as np

    import oracle

    oracle.lib()
    cores = host_cores()
    threads = args.cpu_threads or cores
    h_tabs = [t.data.cpu().numpy() for t in tables]
    h_filters = [f.cpu().numpy().tobytes() for f in filters]
    nq = min(args.cpu_probe_sample, qk.n)
    n1 = min(1_000_000, nq)
    h_q = qk.data[: nq * 20].cpu().numpy()
    gpu_mask = mask[:nq].cpu().numpy()
    kind = "reference" if oracle.ref_lib() is not None else "port"
    one = oracle.timed_cpu_baseline(kind, h_tabs[:1], N, h_filters, h_q[: n1 * 20], n1, bpk, 1)
    allc = oracle.timed_cpu_baseline(kind, h_tabs, N, h_filters, h_q, nq, bpk, threads)
    parity = (all(gpu_filters[s] == allc["built"][s] for s in range(T))
              and bool(np.array_equal(gpu_mask, allc["mask"])) and one["built"][0] == gpu_filters[0])
    legacy_parity = None
    if legacy_out is not None:
        legacy_parity = all(legacy_out[s] == allc["legacy"][s] for s in range(len(allc["legacy"])))
    sample_keys = T * N + nq

    def rates(r, nt, nqq, nth):
        return {"build_mkeys_s": round(nt * N / r["build_s"] / 1e6, 2),
                "probe_mkeys_s": round(nqq / r["probe_s"] / 1e6, 2),
                "legacy_create_mkeys_s": round(r["legacy_tables"] * N / r["legacy_s"] / 1e6, 2),
                # one table per thread: a table's build time on one core
                "build_ms_per_table": round(r["build_s"] * min(nth, nt) / nt * 1e3, 3)}

    out = {
        "value": round(sample_keys / (allc["build_s"] + allc["probe_s"]) / 1e6, 2), "unit": "Mkeys/s",
        "cores": threads, "kind": kind,
        "sample": (f"build {T}x{N} keys (one SSTable per thread, FullFilterBlockBuilder) + probe {nq} "
                   f"lookups x {len(filters)} filters (lookups split over the threads, BloomHash per "
                   f"filter like KeyMayMatch), on all {threads} host cores; T=1: 1 table + {n1} lookups"),
        "all_cores": rates(allc, T, nq, threads),
        "single_thread": rates(one, 1, n1, 1),
        "legacy_note": "util/bloom.cc CreateFilter (legacy FilterPolicy format) over the same tables",
        "host_cpu": cpu_model(),
        "host_cores_available": cores,
        "gpu_output_matches_" + kind: bool(parity),
    }
    if legacy_parity is not None:
        out["gpu_legacy_output_matches_" + kind] = bool(legacy_parity)
    if kind == "reference":
        out["sample"] += ("; util/bloom_impl.h AddHash / HashMayMatch + util/hash.cc + util/bloom.cc "
                          "compiled from the reference (full_filter_block.cc's bookkeeping restated)")
    return out


def version_leg(ctx, stream, dev, lookups=100_000_000, reps=5, space=100_000_000):
    """MultiGet-style probe of a version (dlsm_version_probe_dev): db_bench's
    final version at config 5 (dlsm_amd.workload.dbbench_version: 4 level-0
    files + 5 / 40 / 377 files on levels 1-3, 139.5 MB of filters) and
    `lookups` Gets uniform over [0, 2 x space) -- half of them past every
    file's range, which FindFile still sends to each level's last file
    (db/version_set.cc:95-118).  Per lookup the files Version::Get visits
    whose filter passes it (a u64 slot mask).  Device-resident, HIP events
    over `reps` calls.  Algorithmic bytes: 20 B key read + 8 B mask written
    per lookup + every filter read once.  Parity: tests/test_version_probe.py
    (oracle) and scripts/bench_version_probe.py (first 2 M Gets)."""
    import torch

    import dlsm_amd
    from dlsm_amd import workload as W

    t0 = time.time()
    with torch.cuda.stream(stream):  # torch's input making and the library share one stream
        files = W.dbbench_version(ctx, dev, space)
        ver = ctx.version(files, on_device=True)
        filt = sum(int(f.filter.numel()) for f in files)
        g = torch.Generator(device=dev)
        g.manual_seed(11)
        qv = torch.randint(0, 2 * space, (lookups,), device=dev, dtype=torch.int64, generator=g)
        qk = dlsm_amd.Keys(W.dbbench_keys_torch(qv), lookups, 20)
        del qv
        mask = torch.zeros(lookups, dtype=torch.int64, device=dev)
    snap = (1 << 56) - 1
    ctx.version_probe_dev(ver, qk, snap, mask)  # warm
    ctx.sync()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        ctx.version_probe_dev(ver, qk, snap, mask)
    e1.record(stream)
    stream.synchronize()
    ms = e0.elapsed_time(e1) / reps
    visits = int((mask != 0).sum().item())
    # the same Gets against the same files without filters: the keys, interval
    # search, picks and stores alone -- the part of the pass no filter-line
    # read can hide behind (a floor for the probe, with the line reads below)
    import dataclasses

    bare = ctx.version([dataclasses.replace(f, filter=None) for f in files], on_device=True)
    ctx.version_probe_dev(bare, qk, snap, mask)  # warm
    e0.record(stream)
    for _ in range(reps):
        ctx.version_probe_dev(bare, qk, snap, mask)
    e1.record(stream)
    stream.synchronize()
    nofilter_ms = e0.elapsed_time(e1) / reps
    bare.close()
    alg = lookups * (20 + 8) + filt
    gbs = alg / (ms * 1e-3) / 1e9
    rec = {"ms": round(ms, 4), "mgets_s": round(lookups / ms / 1e3, 1), "lookups": lookups,
           "files_per_level": [4, 5, 40, 377, 0, 0], "filter_bytes": filt,
           "alg_bytes_per_get": round(alg / lookups, 3), "alg_GBs": round(gbs, 1),
           "frac": round(gbs / HBM_PEAK_GBS, 4),
           "gets_with_a_visit": visits, "nofilter_ms": round(nofilter_ms, 4),
           "note": ("roofline vs HBM streaming; the pass is bound by the random 64-byte filter-line "
                    "reads of ~4 probes per Get (Infinity Cache / L2), not by its streamed bytes"),
           "setup_s": round(time.time() - t0, 2)}
    ver.close()
    del qk, mask, files
    return rec


# The filter sets Version::Get really walks (db/version_set.cc:273-321), as
# probe legs beside the headline's 8 equal filters: filter f holds v = 8 i + f.
#   mixed_set      level-0 flushes and compaction outputs of 4 sizes (4 pairs)
#   dedup_shifted  8 flushes whose dedup left each its own line count
#                  (db/memtable_list.cc:855-886 -> full_filter_block.cc:95-96)
SHAPE_LEGS = {
    "mixed_set": [153_846, 153_846, 600_000, 600_000, 1_600_000, 1_600_000, 3_000_000, 3_000_000],
    "dedup_shifted": [1_600_000 - 97 * f for f in range(8)],
}


def shape_leg(ctx, stream, dev, qk, bpk, sizes, reps=5):
    """Batch probe of the bench's lookups against one of SHAPE_LEGS's filter
    sets (the one-pass multi-group probe, round 6), device-resident, HIP
    events; the per-group passes (DLSM_OPT_PROBE_MULTI = 0) timed beside it.
    Algorithmic bytes: 20 B key + 1 B mask per lookup + every filter read
    once.  Parity: tests/test_gpu_fullsize.py (all 100 M mask bytes against
    the oracle), tests/test_gpu_multi_group.py."""
    import torch

    import dlsm_amd
    from dlsm_amd import workload as W

    F = len(sizes)
    tabs, outs = [], []
    with torch.cuda.stream(stream):  # torch's input making and the library share one stream
        for f, n in enumerate(sizes):
            v = torch.arange(n, device=dev, dtype=torch.int64) * F + f
            tabs.append(dlsm_amd.Keys(W.dbbench_keys_torch(v), n, 20))
            outs.append(torch.zeros(dlsm_amd.full_size(n)[0], dtype=torch.uint8, device=dev))
        lens = torch.zeros(F, dtype=torch.uint64, device=dev)
        ctx.full_build_dev(tabs, outs, lens, bpk)
        ctx.sync()
        L = lens.cpu().numpy()
        filters = [outs[f][: int(L[f])] for f in range(F)]
        fs = ctx.filterset(filters, on_device=True)
        mask = torch.empty(qk.n * fs.mask_bytes, dtype=torch.uint8, device=dev)

    def timed(multi):
        ctx.set_option(dlsm_amd.OPT_PROBE_MULTI, multi)
        try:
            ctx.full_probe_dev(fs, qk, mask)  # warm
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                ctx.full_probe_dev(fs, qk, mask)
            e1.record(stream)
            stream.synchronize()
        finally:
            ctx.set_option(dlsm_amd.OPT_PROBE_MULTI, 1)
        return e0.elapsed_time(e1) / reps

    per_group_ms = timed(0)
    ms = timed(1)
    filt = sum(int(f.numel()) for f in filters)
    alg = qk.n * (20 + fs.mask_bytes) + filt
    gbs = alg / (ms * 1e-3) / 1e9
    rec = {"ms": round(ms, 4), "mkeys_s": round(qk.n / ms / 1e3, 1), "lookups": qk.n,
           "keys_per_filter": sizes, "filter_bytes": filt, "alg_bytes_per_key": round(alg / qk.n, 3),
           "alg_GBs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
           "per_group_passes_ms": round(per_group_ms, 4)}
    fs.close()
    del tabs, outs, filters, mask
    return rec


def block_leg(ctx, stream, tables, bpk, reps=20):
    """The sealed wire image: the same tables' full filters
    built as filter BLOCKS -- filter bytes + the 5-byte trailer (type byte +
    masked crc32c, table/table_builder_computeside.cc:418-428,
    util/crc32c.h:17-37) -- in one device-resident batch
    (dlsm_bloom_full_build_block_dev: the build's slice pass also computes
    the crc32c register of each slice's lines from LDS, and one small seal
    kernel folds a filter's slice registers and appends the trailer), against
    the plain batch build on the same stream, HIP events over `reps` calls
    each, interleaved in groups of 5 (the box's clock drifts over a run).
    Algorithmic bytes: 20 B key read + the block written once (the crc reads
    the filter bytes from LDS, not HBM).  Parity: tests/test_gpu_block_seal.py,
    tests/test_gpu_parity.py (trailers equal the reference crc32c.cc
    goldens)."""
    import torch

    import dlsm_amd

    dev = tables[0].data.device
    T = len(tables)
    with torch.cuda.stream(stream):
        outs = [torch.zeros(dlsm_amd.full_size(t.n)[0] + 64, dtype=torch.uint8, device=dev) for t in tables]
        lens = torch.zeros(T, dtype=torch.uint64, device=dev)

    def timed(fn, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(n):
            fn(tables, outs, lens, bpk)
        e1.record(stream)
        stream.synchronize()
        return e0.elapsed_time(e1)

    ctx.full_build_dev(tables, outs, lens, bpk)  # warm both
    ctx.full_build_block_dev(tables, outs, lens, bpk)
    # interleaved groups of 5 calls, so that clock drift over the run falls on
    # both forms alike
    plain = block = 0.0
    groups = max(1, reps // 5)
    for _ in range(groups):
        plain += timed(ctx.full_build_dev, 5)
        block += timed(ctx.full_build_block_dev, 5)
    plain /= groups * 5
    block /= groups * 5
    L = lens.cpu().numpy()
    nk = sum(t.n for t in tables)
    alg = nk * 20 + int(L.sum())
    gbs = alg / (block * 1e-3) / 1e9
    rec = {"ms": round(block, 4), "build_ms": round(plain, 4),
           "crc_seal_ms": round(block - plain, 4), "crc_overhead_frac": round((block - plain) / plain, 4),
           "tables": T, "block_bytes": int(L.sum()), "mkeys_s": round(nk / block / 1e3, 1),
           "alg_GBs": round(gbs, 1), "alg_bytes_per_key": round(alg / nk, 3), "frac": round(gbs / HBM_PEAK_GBS, 4)}
    del outs, lens
    return rec


def legacy_leg(ctx, stream, tables, bpk, reps=20, direct_reps=3):
    """util/bloom.cc CreateFilter (the legacy FilterPolicy format) for the same
    tables in one device-resident batch (dlsm_bloom_legacy_build_dev): the
    LDS-tiled path (auto) timed with HIP events over `reps` calls on the
    context's stream, the direct global-atomic path (path 1) beside it.
    Algorithmic bytes: 20 B key read + the filter written once (bits/8 + 1 B,
    1.25 B/key at 10 bits/key).  Returns (record, host filters of the tiled
    path)."""
    import torch

    import dlsm_amd

    dev = tables[0].data.device
    outs = [torch.zeros(dlsm_amd.legacy_size(t.n, bpk) + 16, dtype=torch.uint8, device=dev) for t in tables]
    lens = torch.zeros(len(tables), dtype=torch.uint64, device=dev)

    def timed(path, n):
        ctx.set_path(path)
        try:
            for _ in range(2):
                ctx.legacy_build_dev(tables, outs, lens, bpk)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(n):
                ctx.legacy_build_dev(tables, outs, lens, bpk)
            e1.record(stream)
            stream.synchronize()
        finally:
            ctx.set_path(0)
        return e0.elapsed_time(e1) / n

    direct_ms = timed(1, direct_reps)
    direct = [o[: int(n)].cpu().numpy().tobytes() for o, n in zip(outs, lens.cpu().numpy())]
    ms = timed(0, reps)
    L = lens.cpu().numpy()
    got = [o[: int(n)].cpu().numpy().tobytes() for o, n in zip(outs, L)]
    nk = sum(t.n for t in tables)
    alg = nk * 20 + int(L.sum())
    gbs = alg / (ms * 1e-3) / 1e9
    rec = {"ms": round(ms, 4), "mkeys_s": round(nk / ms / 1e3, 1), "alg_GBs": round(gbs, 1),
           "alg_bytes_per_key": round(alg / nk, 3), "frac": round(gbs / HBM_PEAK_GBS, 4),
           "kernels": "legacy_partition_kernel + legacy_slice_kernel (tile-bucketed u16 positions, LDS ds_or)",
           "direct_path_ms": round(direct_ms, 4), "direct_path_mkeys_s": round(nk / direct_ms / 1e3, 1),
           "tiled_equals_direct": got == direct,
           "note": "util/bloom.cc CreateFilter for the same tables (config 2's format), not `value`"}
    return rec, got


def pass_timing_note(overlapped: bool, every: int) -> dict:
    """How the pass times behind `achieved` were taken."""
    how = (f"HIP events around each pass of every {every}-th timed step; those steps run their two passes "
           "one after the other, alone on the GPU (the other steps overlap the build with the probe on two "
           "streams), so `achieved` is the pass's own rate" if overlapped else
           f"HIP events around each pass of every {every}-th timed step (one stream)")
    return {"pass_timing": how}


def step_roofline(step_alg_bytes: float, step_s: float) -> dict:
    """The whole step's algorithmic bytes (build 21.25 + probe 21.16 B/key,
    SURVEY.md §8d) over the step time: with the two passes co-running this is
    the rate the GPU sustains on the job, beside the dominant pass's own."""
    gbs = step_alg_bytes / step_s / 1e9
    return {"step_alg_GBs": round(gbs, 1), "step_frac": round(gbs / HBM_PEAK_GBS, 4)}


def other_shape_rate(args, ctx, stream, tables, outs, lens, fs, qk, mask, bpk, device, timed_step_s, overlapped,
                     reps=10):
    """The step in the shape the timed region did not use -- one pass after
    the other on one stream when the timed steps overlapped the build (second
    context and stream) with the probe, and the overlapped shape otherwise;
    recorded beside `value`, never `value`."""
    import torch

    import dlsm_amd

    if not tables or not qk.n:
        return None
    ctx2, s2 = ctx, stream
    if not overlapped:
        ctx2 = dlsm_amd.Context(device)
        ctx2.set_path(args.path)
        ctx2.set_build_groups(args.build_groups)
        ctx2.set_probe_shape(args.probe_chunk_lg, args.probe_slice_lg)
        s2 = torch.cuda.Stream(device=torch.device("cuda", device))
        ctx2.set_stream(s2)

    def one():
        ctx2.full_build_dev(tables, outs, lens, bpk)
        ctx.full_probe_dev(fs, qk, mask)

    for _ in range(3):
        one()
    stream.synchronize()
    s2.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        one()
    stream.synchronize()
    s2.synchronize()
    dt = (time.perf_counter() - t0) / reps
    if not overlapped:
        ctx2.sync()
        del ctx2
    nk = len(tables) * tables[0].n + qk.n
    shape = "build and probe one after the other on one stream" if overlapped else \
        "build on a second stream concurrent with the probe"
    return {"shape": shape, "mkeys_s": round(nk / dt / 1e6, 1), "ms_per_step": round(dt * 1e3, 4),
            "this_vs_timed_step": round(dt / timed_step_s, 3), "note": "not `value`"}


def rotating_build_ms(ctx, stream, tables, outs, lens, bpk, reps=10):
    """Build ms when consecutive calls alternate between two different job
    tables (output slots swapped): every call uploads its job table, as a
    flush stream that hands over new tables each time does."""
    import torch

    if len(tables) < 2:
        return float("nan")
    outs_b = outs[1:] + outs[:1]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for r in range(reps):
        ctx.full_build_dev(tables, outs if r % 2 == 0 else outs_b, lens, bpk)
    e1.record(stream)
    stream.synchronize()
    ctx.full_build_dev(tables, outs, lens, bpk)  # leave the slots as the timed loop wrote them
    ctx.sync()
    return e0.elapsed_time(e1) / reps


if __name__ == "__main__":
    main()
