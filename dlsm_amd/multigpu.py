"""One process, one host thread per GPU ("all GPUs
launched concurrently from one host thread per GPU").

dLSM runs its filter builders as threads of one process -- one std::thread
per subcompaction (db/db_impl.cc:3373-3386) beside 4 flush + 12 compaction
background threads (include/TimberSaw/options.h:73-78) -- so the multi-GPU
shape here is the same: a DeviceWorker per GPU, each owning a dlsm_ctx and a
HIP stream on its device, building the SSTables s mod G of the job and
probing its contiguous shard of the lookup stream against its own copy of the
stacked filter set.  Nothing crosses devices in the hot loop.

The ctypes calls release the GIL, and every per-step call is bound once
(Context.bind_*: the job tables and key descriptors are marshalled before
timing), so the workers' launches run in parallel on the host.

`rehearse=True` maps every logical device onto device 0 (a 1-GPU box runs the
same code with N contexts sharing one GPU).
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field

from . import sharding as SH

# timed steps whose passes are bracketed with HIP events (event_stride)
PASS_EVENT_SAMPLES = 4


class DeviceCountError(RuntimeError):
    """More GPUs requested than the node has (and no rehearsal)."""


def device_map(n_gpus: int, rehearse: bool, available: int) -> list:
    """Physical device of each logical rank: rank r -> device r, or device 0
    for every rank when rehearsing.  Refuses to run N ranks on fewer devices."""
    if n_gpus < 1:
        raise ValueError("n_gpus must be >= 1")
    if rehearse:
        if available < 1:
            raise DeviceCountError("rehearsal needs one visible GPU, found none")
        return [0] * n_gpus
    if available < n_gpus:
        raise DeviceCountError(
            f"--gpus {n_gpus} asks for {n_gpus} GPUs but only {available} are visible "
            f"(use --rehearse to map {n_gpus} logical devices onto GPU 0)")
    return list(range(n_gpus))


@dataclass
class WorkerOptions:
    path: int = 0
    probe_chunk_lg: int = 13
    probe_slice_lg: int = 8
    overlap: str = "auto"        # build on a second stream: auto (= on when both passes run) | on | off
    pass_events: bool = False    # record per-pass HIP events (device 0's worker)


@dataclass
class DeviceWorker:
    rank: int
    world: int
    device: int
    work: SH.RankWork
    N: int
    F: int
    bpk: int
    lookup_values: object        # numpy u64 values of this rank's lookup shard
    opts: WorkerOptions = field(default_factory=WorkerOptions)
    # filled by setup()
    inp: object = None
    overlap: bool = False
    build_ms: list = field(default_factory=list)
    probe_ms: list = field(default_factory=list)

    def setup(self):
        import torch

        import dlsm_amd

        torch.cuda.set_device(self.device)
        dev = torch.device("cuda", self.device)
        self.dev = dev

        def make_ctx():
            c = dlsm_amd.Context(self.device)
            c.set_path(self.opts.path)
            c.set_probe_shape(self.opts.probe_chunk_lg, self.opts.probe_slice_lg)
            st = torch.cuda.Stream(device=dev)
            c.set_stream(st)
            return c, st

        self.ctx, self.stream = make_ctx()
        # the filter set is built on this device from the same keys as every
        # other device's (deterministic: byte-identical copies, checked by
        # filter_digest) -- the one-time set-up exchange of SURVEY.md §8e
        self.inp = SH.make_inputs(self.ctx, self.work, self.N, self.F, self.bpk, dev, stream=self.stream,
                                  dist=None, lookup_shard=self.lookup_values)
        inp = self.inp
        self.overlap = bool(inp.tables) and inp.lookups.n > 0 and self.opts.overlap != "off"
        self.ctx_b, self.stream_b = make_ctx() if self.overlap else (self.ctx, self.stream)
        self._build = (self.ctx_b.bind_full_build_dev(inp.tables, inp.outs, inp.lens, self.bpk)
                       if inp.tables else None)
        self._probe = self.ctx.bind_full_probe_dev(inp.fs, inp.lookups, inp.mask) if inp.lookups.n else None

    def step(self):
        if self._build:
            self._build()
        if self._probe:
            self._probe()

    def sync(self):
        self.stream.synchronize()
        self.stream_b.synchronize()

    def timed_steps(self, k: int):
        """k steps; with pass_events, HIP events bracket each pass of every
        event_stride(k)-th step on its stream."""
        import torch

        if not self.opts.pass_events:
            for _ in range(k):
                self.step()
            return
        every = event_stride(k)
        evs = []
        for i in range(k):
            if i % every != every - 1:
                self.step()
                continue
            # a sampled step runs its passes alone: its build after the probes
            # before it, its probe after its build, the next build after its
            # probe (dlsm_multi_device_run_sampled does the same)
            e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            two = self.stream_b is not self.stream
            if two:
                gate = torch.cuda.Event()
                gate.record(self.stream)
                self.stream_b.wait_event(gate)
            e[0].record(self.stream_b)
            if self._build:
                self._build()
            e[1].record(self.stream_b)
            if two:
                self.stream.wait_event(e[1])
            e[2].record(self.stream)
            if self._probe:
                self._probe()
            e[3].record(self.stream)
            if two:
                self.stream_b.wait_event(e[3])
            evs.append(e)
        self._evs = evs

    def collect_pass_times(self):
        evs = getattr(self, "_evs", None)
        if evs:
            self.build_ms = [e[0].elapsed_time(e[1]) for e in evs]
            self.probe_ms = [e[2].elapsed_time(e[3]) for e in evs]

    def device_work(self):
        """This device's dlsm_device_work (the native runner's argument)."""
        w, keep = device_work(self.ctx, self.ctx_b, self.inp)
        self._work_keep = keep
        return w

    def filter_digest(self) -> int:
        """Checksum of this device's stacked-filter inputs (all devices must agree)."""
        import hashlib

        h = hashlib.sha256()
        for f in self.inp.filters:
            h.update(f.cpu().numpy().tobytes())
        return int.from_bytes(h.digest()[:8], "little")

    def close(self):
        if self.inp is not None:
            self.inp.fs.close()
        for c in {id(self.ctx): self.ctx, id(self.ctx_b): self.ctx_b}.values():
            c.close()


def _run_threads(workers, fn):
    """fn(worker) on one thread per worker; re-raises the first failure."""
    errs = [None] * len(workers)

    def body(i):
        try:
            fn(workers[i])
        except BaseException as e:  # noqa: BLE001 -- reported below
            errs[i] = e

    ts = [threading.Thread(target=body, args=(i,), name=f"dlsm-gpu{w.rank}") for i, w in enumerate(workers)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in errs:
        if e is not None:
            raise e


def timed_run(workers, steps: int, warmup: int):
    """Warm up every device, then time `steps` steps on all devices at once:
    a barrier + device synchronisation on both sides, the wall time covering
    the slowest device (the max over ranks).  Returns seconds."""
    n = len(workers)
    start, end = threading.Barrier(n + 1), threading.Barrier(n + 1)
    errs = [None] * n

    def body(i):
        w = workers[i]
        try:
            import torch

            torch.cuda.set_device(w.device)
            for _ in range(warmup):
                w.step()
            w.sync()
            torch.cuda.synchronize(w.device)
        except BaseException as e:  # noqa: BLE001
            errs[i] = e
            start.abort()
            end.abort()
            return
        try:
            start.wait()
            w.timed_steps(steps)
            w.sync()
            torch.cuda.synchronize(w.device)
            end.wait()
        except threading.BrokenBarrierError:
            return
        except BaseException as e:  # noqa: BLE001
            errs[i] = e
            end.abort()

    ts = [threading.Thread(target=body, args=(i,), name=f"dlsm-gpu{workers[i].rank}") for i in range(n)]
    for t in ts:
        t.start()
    t0 = t1 = None
    try:
        start.wait()
        t0 = time.perf_counter()
        end.wait()
        t1 = time.perf_counter()
    except threading.BrokenBarrierError:
        pass
    for t in ts:
        t.join()
    for e in errs:
        if e is not None:
            raise e
    if t0 is None or t1 is None:
        raise RuntimeError("a device worker failed before the timed region ended")
    return t1 - t0


def device_work(ctx, build_ctx, inp):
    """dlsm_device_work for one device's inputs (sharding.RankInputs): the
    build jobs on build_ctx, the probe on ctx.  Returns (struct, keep-alive)."""
    import ctypes as C

    from . import _lib as L
    from . import _ptr

    caps = [int(o.numel()) for o in inp.outs]
    jobs = build_ctx._jobs(inp.tables, inp.outs, caps)
    w = L.dlsm_device_work()
    w.probe_ctx, w.build_ctx = ctx.h.value, build_ctx.h.value
    w.jobs = C.cast(jobs, C.c_void_p).value
    w.n_jobs = len(inp.tables)
    w.out_len_dev = _ptr(inp.lens)
    w.fs = inp.fs.h.value if inp.lookups.n else None
    w.keys = inp.lookups.c()
    w.mask_dev = _ptr(inp.mask)
    return w, (jobs, w)


def event_stride(steps: int, samples: int = PASS_EVENT_SAMPLES) -> int:
    """Every how many timed steps the passes are bracketed with HIP events:
    `samples` steps spread over the timed region (each event pair at a call
    boundary idles the GPU for several microseconds, so timing every step
    lengthens the very steps being timed: profiles/r03_o_pass_events_ab.txt)."""
    return max(1, steps // max(1, samples))


def native_run(works, steps: int, warmup: int, bits_per_key: int, event_every: int | None = None,
               per_device: bool = False):
    """dlsm_multi_device_run_timed over dlsm_device_work structs: (seconds,
    [(build_ms, probe_ms) per sampled step] of the first device), or with
    per_device (seconds, [that list per device], [each device's own seconds])."""
    import ctypes as C

    from . import _lib as L
    from . import check, lib

    n = len(works)
    every = event_stride(steps) if event_every is None else event_every
    arr = (L.dlsm_device_work * n)(*works)
    wall = C.c_double(0.0)
    pm = (C.c_float * (2 * steps * n))()
    ds = (C.c_double * n)()
    check(lib().dlsm_multi_device_run_timed(arr, n, bits_per_key, steps, warmup, every, C.byref(wall), pm, ds),
          "multi_device_run")
    passes = [[(pm[2 * steps * d + 2 * i], pm[2 * steps * d + 2 * i + 1]) for i in range(steps)
               if pm[2 * steps * d + 2 * i + 1] >= 0] for d in range(n)]
    if per_device:
        return wall.value, passes, [ds[d] for d in range(n)]
    return wall.value, passes[0]


def native_timed_run(workers, steps: int, warmup: int, bits_per_key: int):
    """The timed region run by the library's native runner
    (dlsm_multi_device_run_timed: a std::thread per device, host barriers on
    both sides of the timed steps, every device's passes timed with HIP events
    on the sampled steps).  Returns (seconds, [(build_ms, probe_ms) per sampled
    step] per device, [each device's own seconds])."""
    return native_run([w.device_work() for w in workers], steps, warmup, bits_per_key, per_device=True)


def build_workers(n_gpus: int, devices: list, T: int, N: int, Q: int, F: int, bpk: int,
                  opts: WorkerOptions, lookup_stream=None):
    """One DeviceWorker per logical rank (strong scaling: tables s mod G,
    lookups split into contiguous shards of ONE stream), set up on its own
    thread.  `lookup_stream`: the full stream's u64 values (generated once)."""
    import numpy as np

    if lookup_stream is None:
        from . import workload as W

        lookup_stream = W.mt19937_64(1000, Q) % np.uint64(2 * F * N)
    workers = []
    for r in range(n_gpus):
        work = SH.plan(r, n_gpus, T, N, Q, "strong")
        o = WorkerOptions(**{**opts.__dict__, "pass_events": opts.pass_events and r == 0})
        workers.append(DeviceWorker(r, n_gpus, devices[r], work, N, F, bpk,
                                    lookup_stream[work.lookup_lo:work.lookup_hi], o))
    # set-up runs one device at a time: torch's tensor factories hold the GIL
    # anyway, and a serial set-up keeps the first-touch allocations ordered
    for w in workers:
        _run_threads([w], DeviceWorker.setup)
    return workers
