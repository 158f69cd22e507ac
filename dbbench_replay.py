"""db_bench-shape replay with the GPU filter path plugged in (BASELINE config 5,
SURVEY.md §8d): `db_bench --benchmarks=fillrandom,readrandom --value_size=400
--bloom_bits=10 --threads=16`, host buffers in and out (H2D / D2H included).

Real db_bench cannot run here or on the GPU box: Env::Default() builds an
RDMA_Manager (util/env_posix.cc:36-42) that needs ibverbs, a memory node and
connection.conf.  This replays the part that reaches the filter path:

* fillrandom (benchmarks/db_bench.cc:1220-1245): thread t (ThreadState seed
  1000 + t + 1, :943-947) writes k = Random64.Next() % (num * threads)
  (Random64 = std::mt19937_64, util/random.h:140-165) as GenerateKeyFromInt(k)
  (:677-711).  The threads' writes enter one memtable round-robin (a
  deterministic stand-in for the reference's concurrent interleaving); every
  153,846 entries (db/memtable.h:7) the memtable flushes: its user keys sorted,
  one entry per user key (FlushJob::BuildTable, db/memtable_list.cc:855-886)
  -> one full filter per flushed SSTable, built on the GPU from HOST keys into
  HOST slots (dlsm_bloom_full_build: H2D keys + build + D2H filters).
* readrandom (:1379-1404): thread t reads k = Random64(1000 + threads + t + 1)
  .Next() % (num * threads); each Get visits the level-0 flush files newest
  first (Version::ForEachOverlapping) and checks their filters -> one batched
  dlsm_version_probe_dev per call from HOST keys (H2D keys + probe + D2H
  masks).  No compaction is modelled: every flush stays in level 0 (at most 59
  files -- pick --num accordingly).

Prints one JSON line.  Parity of these calls against the oracle is covered by
tests/ (test_dbbench_replay.py runs a small replay and checks it).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import dlsm_amd  # noqa: E402
from dlsm_amd import workload as W  # noqa: E402

MEMTABLE_ENTRIES = 153_846  # db/memtable.h:7


def fill_stream(num: int, threads: int) -> np.ndarray:
    """fillrandom key values in memtable arrival order (thread round-robin)."""
    cols = [W.mt19937_64(1000 + t + 1, num) % np.uint64(num * threads) for t in range(threads)]
    return np.stack(cols, axis=1).reshape(-1)


def read_stream(num: int, threads: int) -> np.ndarray:
    cols = [W.mt19937_64(1000 + threads + t + 1, num) % np.uint64(num * threads) for t in range(threads)]
    return np.stack(cols, axis=1).reshape(-1)


def flushes(stream: np.ndarray):
    """Per flushed memtable: its distinct user-key values, ascending (the
    flush keeps one entry per user key; big-endian keys sort like values)."""
    out = []
    for s in range(0, stream.size, MEMTABLE_ENTRIES):
        out.append(np.unique(stream[s:s + MEMTABLE_ENTRIES]))
    return out


def run(num: int, threads: int, bpk: int, device: int = 0, reps: int = 3):
    import torch

    ctx = dlsm_amd.Context(device)
    t0 = time.time()
    fill = fill_stream(num, threads)
    mem = flushes(fill)
    tables = [dlsm_amd.Keys(W.dbbench_keys_np(v), v.size, 20) for v in mem]
    gen_s = time.time() - t0
    n_fill_keys = int(sum(v.size for v in mem))

    # ---- fillrandom: every flush's filter, host keys -> host slots -------
    filters = ctx.full_build(tables, bpk)  # warm (allocations)
    t1 = time.perf_counter()
    for _ in range(reps):
        filters = ctx.full_build(tables, bpk)
    build_s = (time.perf_counter() - t1) / reps

    # ---- readrandom: Gets over the level-0 flush files ---------------------
    files = [dlsm_amd.VersionFile(0, j + 1, bytes(t.data[:20]), bytes(t.data[-20:]), (1 << 8) | 1, f)
             for j, (t, f) in enumerate(zip(tables, filters))]
    ver = ctx.version(files)
    reads = read_stream(num, threads)
    q = W.dbbench_keys_np(reads)
    nq = reads.size
    dev = torch.device(f"cuda:{device}")
    qh = torch.from_numpy(q).pin_memory()
    mh = torch.empty(nq, dtype=torch.int64).pin_memory()
    qd = torch.empty(q.size, dtype=torch.uint8, device=dev)
    md = torch.empty(nq, dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(device=dev)
    ctx.set_stream(stream)

    def get_batch():
        with torch.cuda.stream(stream):
            qd.copy_(qh, non_blocking=True)
            ctx.version_probe_dev(ver, dlsm_amd.Keys(qd, nq, 20), (1 << 56) - 1, md)
            mh.copy_(md, non_blocking=True)
        stream.synchronize()

    get_batch()
    t2 = time.perf_counter()
    for _ in range(reps):
        get_batch()
    read_s = (time.perf_counter() - t2) / reps
    # device-resident probe alone
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(reps):
        ctx.version_probe_dev(ver, dlsm_amd.Keys(qd, nq, 20), (1 << 56) - 1, md)
    ev1.record(stream)
    stream.synchronize()
    probe_dev_ms = ev0.elapsed_time(ev1) / reps
    masks = mh.numpy().view(np.uint64)
    hits = int(np.count_nonzero(masks))
    filter_checks = len(mem) * nq  # what per-key Gets would do: every L0 file whose range holds the key
    ctx.set_stream(None)
    ver.close()
    return {
        "workload": "db_bench fillrandom,readrandom replay (filter path), host buffers",
        "num": num, "threads": threads, "bloom_bits": bpk, "value_size": 400,
        "memtable_entries": MEMTABLE_ENTRIES, "flushes": len(mem),
        "fill": {"writes": int(fill.size), "distinct_keys_flushed": n_fill_keys,
                 "build_ms": round(build_s * 1e3, 3),
                 "mkeys_s_incl_h2d_d2h": round(n_fill_keys / build_s / 1e6, 1),
                 "filter_bytes": int(sum(len(f) for f in filters))},
        "read": {"gets": int(nq), "ms": round(read_s * 1e3, 3),
                 "mgets_s_incl_h2d_d2h": round(nq / read_s / 1e6, 1),
                 "probe_dev_ms": round(probe_dev_ms, 3),
                 "mgets_s_device": round(nq / probe_dev_ms / 1e3, 1),
                 "keys_with_a_candidate": hits, "l0_files_per_get": len(mem)},
        "host_keygen_s": round(gen_s, 1),
    }, (mem, filters, reads, masks)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num", type=int, default=500_000, help="db_bench --num (per thread)")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--bloom-bits", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    if not dlsm_amd.device_available():
        raise SystemExit("dbbench_replay: no HIP device")
    res, _ = run(args.num, args.threads, args.bloom_bits, reps=args.reps)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
