"""db_bench-shape replay with the GPU filter path plugged in (BASELINE config 5,
SURVEY.md §8d): `db_bench --benchmarks=fillrandom,readrandom --value_size=400
--bloom_bits=10 --threads=16 --num=N`, host buffers in and out (H2D / D2H
included in every timed call).

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
  -> a level-0 SSTable whose full filter is built on the GPU from HOST keys into
  HOST slots (dlsm_bloom_full_build: H2D keys + build + D2H filters).
* leveled compaction with dLSM's constants, a model of DBImpl::
  BackgroundCompaction / VersionSet::PickCompaction (db/version_set.cc:
  1340-1400, 1816-1870): level 0 compacts as soon as it holds
  kL0_CompactionTrigger = 1 file (db/dbformat.h:31); level L >= 1 when its bytes
  exceed max_mega_bytes_for_level_base = 256 MiB x 10^(L-1) (db/dbformat.h:52,
  version_set.cc:48-59), taking the next file after the level's compact
  pointer; the inputs merge with the overlapping files of level L+1 into
  outputs of at most max_file_size = 64 MiB (include/TimberSaw/options.h:157;
  64 MiB / 436 B per entry = 153,846 entries), a single input with no overlap
  moves down unchanged (Compaction::IsTrivialMove, version_set.cc:2112-2121).
  Every compaction's outputs are ONE batched GPU filter build from host keys
  (the outputs of one compaction round, built together).
* readrandom (:1379-1404): thread t reads k = Random64(1000 + threads + t + 1)
  .Next() % (num * threads); each Get visits the files Version::Get would
  (level-0 newest first, then one file per level: ForEachOverlapping,
  version_set.cc:273-321) and checks their filters -> one batched
  dlsm_version_probe_dev per batch of host keys (H2D keys + probe + D2H masks).

Prints one JSON line.  Parity against the oracle: tests/test_dbbench_replay.py
(every filter and Get of a small replay) and tests/replay_fullsize_check.py
(sampled, at --num 6,250,000 x 16 threads = 100 M writes).
"""
from __future__ import annotations

import argparse
import bisect
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import dlsm_amd  # noqa: E402
from dlsm_amd import workload as W  # noqa: E402

MEMTABLE_ENTRIES = 153_846         # db/memtable.h:7
ENTRY_BYTES = 436                  # 20 B key + 8 B seq/type + 400 B value + ~8 B framing
MAX_FILE_ENTRIES = 153_846         # max_file_size 64 MiB (options.h:157) / ENTRY_BYTES
L0_TRIGGER = 1                     # config::kL0_CompactionTrigger (db/dbformat.h:31)
LEVEL_BASE_BYTES = 256 * 1048576   # config::max_mega_bytes_for_level_base (db/dbformat.h:52)
NUM_LEVELS = 6                     # config::kNumLevels (db/dbformat.h:26)


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


def max_bytes_for_level(level: int) -> float:
    r = float(LEVEL_BASE_BYTES)
    while level > 1:
        r *= 10
        level -= 1
    return r


class SSTable:
    __slots__ = ("values", "number", "filter")

    def __init__(self, values, number, filt):
        self.values, self.number, self.filter = values, number, filt

    @property
    def smallest(self):
        return int(self.values[0])

    @property
    def largest(self):
        return int(self.values[-1])


class LSM:
    """Leveled LSM over key VALUES (the filter path needs only the user keys);
    every new SSTable's filter is built on the GPU from host keys."""

    def __init__(self, ctx, bpk: int, on_build=None):
        self.ctx, self.bpk = ctx, bpk
        self.levels = [[] for _ in range(NUM_LEVELS)]
        self.pointer = [None] * NUM_LEVELS  # compact_index_: largest value last compacted
        self.next_number = 1
        self.on_build = on_build  # test hook: (values list, filters list)
        self.stats = {"flush_builds": 0, "flush_keys": 0, "flush_s": 0.0,
                      "compactions": 0, "trivial_moves": 0, "compaction_builds": 0,
                      "compaction_keys": 0, "compaction_s": 0.0, "merge_s": 0.0}

    def _build(self, value_sets, kind):
        tables = [dlsm_amd.Keys(W.dbbench_keys_np(v), v.size, 20) for v in value_sets]
        t0 = time.perf_counter()
        filters = self.ctx.full_build(tables, self.bpk)  # host keys -> host slots
        dt = time.perf_counter() - t0
        self.stats[kind + "_builds"] += len(value_sets)
        self.stats[kind + "_keys"] += int(sum(v.size for v in value_sets))
        self.stats[kind + "_s"] += dt
        if self.on_build:
            self.on_build(value_sets, filters)
        out = []
        for v, f in zip(value_sets, filters):
            out.append(SSTable(v, self.next_number, f))
            self.next_number += 1
        return out

    def flush(self, values):
        self.levels[0].extend(self._build([values], "flush"))
        self.compact_while_needed()

    def _score(self, level):
        if level == 0:
            return len(self.levels[0]) / L0_TRIGGER
        return sum(f.values.size for f in self.levels[level]) * ENTRY_BYTES / max_bytes_for_level(level)

    def compact_while_needed(self):
        while True:
            scores = [(self._score(lv), -lv) for lv in range(NUM_LEVELS - 1)]
            best, neg = max(scores)
            if best < 1:
                return
            self.compact(-neg)

    def compact(self, level):
        files = self.levels[level]
        if level == 0:
            inputs = list(files)  # level-0 files overlap: all of them (trigger 1: usually one)
        else:
            p = self.pointer[level]
            cand = [f for f in files if p is None or f.largest > p]
            inputs = [cand[0] if cand else files[0]]
        lo = min(f.smallest for f in inputs)
        hi = max(f.largest for f in inputs)
        nxt = self.levels[level + 1]
        over = [f for f in nxt if not (f.largest < lo or f.smallest > hi)]
        self.pointer[level] = hi
        self.stats["compactions"] += 1
        if level > 0 and len(inputs) == 1 and not over:  # IsTrivialMove
            files.remove(inputs[0])
            self._insert(level + 1, [inputs[0]])
            self.stats["trivial_moves"] += 1
            return
        t0 = time.perf_counter()
        merged = np.concatenate([f.values for f in inputs + over])
        merged.sort(kind="stable")  # sorted runs: timsort merges them
        keep = np.empty(merged.size, dtype=bool)
        keep[0] = True
        np.not_equal(merged[1:], merged[:-1], out=keep[1:])
        merged = merged[keep]
        outs = [merged[s:s + MAX_FILE_ENTRIES] for s in range(0, merged.size, MAX_FILE_ENTRIES)]
        self.stats["merge_s"] += time.perf_counter() - t0
        new = self._build(outs, "compaction")
        for f in inputs:
            files.remove(f)
        for f in over:
            nxt.remove(f)
        self._insert(level + 1, new)

    def _insert(self, level, new):
        lst = self.levels[level]
        for f in new:  # levels >= 1 stay in key order (non-overlapping)
            bisect.insort(lst, f, key=lambda x: x.smallest)

    def version_files(self):
        files = []
        for lv, lst in enumerate(self.levels):
            for f in lst:
                files.append(dlsm_amd.VersionFile(lv, f.number, W.dbbench_keys_np(f.values[:1]).tobytes(),
                                                  W.dbbench_keys_np(f.values[-1:]).tobytes(),
                                                  (1 << 8) | 1, f.filter))
        return files


def run(num: int, threads: int, bpk: int, device: int = 0, reps: int = 1, read_batch: int = 25_000_000,
        on_build=None, on_read=None):
    import torch

    ctx = dlsm_amd.Context(device)
    t0 = time.time()
    fill = fill_stream(num, threads)
    mem = flushes(fill)
    gen_s = time.time() - t0

    # ---- fillrandom: flushes + leveled compactions, every filter on the GPU --
    lsm = LSM(ctx, bpk, on_build)
    ctx.full_build([dlsm_amd.Keys(W.dbbench_keys_np(mem[0]), mem[0].size, 20)], bpk)  # warm-up (allocations)
    t1 = time.perf_counter()
    for v in mem:
        lsm.flush(v)
    fill_wall_s = time.perf_counter() - t1
    st = lsm.stats

    # ---- readrandom: Gets over the final version -------------------------
    files = lsm.version_files()
    ver = ctx.version(files)
    reads = read_stream(num, threads)
    nq = reads.size
    dev = torch.device(f"cuda:{device}")
    B = min(read_batch, nq)
    qh = torch.empty(B * 20, dtype=torch.uint8).pin_memory()
    mh = torch.empty(B, dtype=torch.int64).pin_memory()
    qd = torch.empty(B * 20, dtype=torch.uint8, device=dev)
    md = torch.empty(B, dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(device=dev)
    ctx.set_stream(stream)
    read_s, probe_ms, hits = 0.0, 0.0, 0
    for b0 in range(0, nq, B):
        nb = min(B, nq - b0)
        qh[: nb * 20].numpy()[:] = W.dbbench_keys_np(reads[b0:b0 + nb])
        t2 = time.perf_counter()
        with torch.cuda.stream(stream):
            qd[: nb * 20].copy_(qh[: nb * 20], non_blocking=True)
            ctx.version_probe_dev(ver, dlsm_amd.Keys(qd, nb, 20), (1 << 56) - 1, md)
            mh[:nb].copy_(md[:nb], non_blocking=True)
        stream.synchronize()
        read_s += time.perf_counter() - t2
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        ctx.version_probe_dev(ver, dlsm_amd.Keys(qd, nb, 20), (1 << 56) - 1, md)  # device-resident alone
        ev1.record(stream)
        stream.synchronize()
        probe_ms += ev0.elapsed_time(ev1)
        m = mh[:nb].numpy().view(np.uint64)
        hits += int(np.count_nonzero(m))
        if on_read:
            on_read(b0, reads[b0:b0 + nb], m.copy(), files)
    ctx.set_stream(None)
    ver.close()
    built_keys = st["flush_keys"] + st["compaction_keys"]
    build_s = st["flush_s"] + st["compaction_s"]
    return {
        "workload": "db_bench fillrandom,readrandom replay (filter path, leveled compaction model), host buffers",
        "num": num, "threads": threads, "bloom_bits": bpk, "value_size": 400,
        "memtable_entries": MEMTABLE_ENTRIES, "flushes": len(mem),
        "fill": {"writes": int(fill.size), "wall_s": round(fill_wall_s, 2),
                 "flush_builds": st["flush_builds"], "flush_keys": st["flush_keys"],
                 "compactions": st["compactions"], "trivial_moves": st["trivial_moves"],
                 "compaction_builds": st["compaction_builds"], "compaction_keys": st["compaction_keys"],
                 "filter_build_s_incl_h2d_d2h": round(build_s, 3),
                 "filter_mkeys_s_incl_h2d_d2h": round(built_keys / build_s / 1e6, 1),
                 "flush_filter_mkeys_s": round(st["flush_keys"] / max(st["flush_s"], 1e-9) / 1e6, 1),
                 "compaction_filter_mkeys_s": round(st["compaction_keys"] / max(st["compaction_s"], 1e-9) / 1e6, 1),
                 "host_merge_s": round(st["merge_s"], 2)},
        "version": {"files_per_level": [len(l) for l in lsm.levels],
                    "keys_per_level": [int(sum(f.values.size for f in l)) for l in lsm.levels]},
        "read": {"gets": int(nq), "s_incl_h2d_d2h": round(read_s, 3),
                 "mgets_s_incl_h2d_d2h": round(nq / read_s / 1e6, 1),
                 "probe_dev_ms": round(probe_ms, 3),
                 "mgets_s_device": round(nq / probe_ms / 1e3, 1),
                 "gets_with_a_candidate": hits},
        "host_keygen_s": round(gen_s, 1),
    }, lsm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num", type=int, default=500_000, help="db_bench --num (per thread)")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--bloom-bits", type=int, default=10)
    args = ap.parse_args()
    if not dlsm_amd.device_available():
        raise SystemExit("dbbench_replay: no HIP device")
    res, _ = run(args.num, args.threads, args.bloom_bits)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
