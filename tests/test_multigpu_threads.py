"""`bench.py --gpus N` in ONE process, a host thread + context + stream per GPU
(dlsm_amd/multigpu.py; SURVEY.md §8d config 4, "all GPUs launched
concurrently from one host thread per GPU").

* CPU: the launch-shape rules -- N > visible GPUs exits non-zero instead of
  silently running one GPU, --gpus must equal a launcher's WORLD_SIZE, the
  rehearsal map, the device map of a full node.
* GPU (-m gpu): two logical devices rehearsed on GPU 0 through the bench's own
  worker code (build_workers / timed_run): the union of the two devices'
  filters and the concatenation of their mask shards equal the oracle's
  single-device answer, and `bench.py --gpus 2 --rehearse` prints
  n_gpus 2 with tables [0,2,..]/[1,3,..] and lookups [0,Q/2)/[Q/2,Q).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env=None, timeout=300):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    if env:
        e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True,
                          text=True, timeout=timeout, env=e, cwd=ROOT)


def test_device_map_rules():
    from dlsm_amd import multigpu as MG

    assert MG.device_map(8, False, 8) == list(range(8))
    assert MG.device_map(4, False, 8) == [0, 1, 2, 3]
    assert MG.device_map(2, True, 1) == [0, 0]
    with pytest.raises(MG.DeviceCountError):
        MG.device_map(8, False, 1)
    with pytest.raises(MG.DeviceCountError):
        MG.device_map(2, True, 0)


def test_pass_events_are_sampled():
    """The timed steps carry per-pass HIP events on only PASS_EVENT_SAMPLES of
    them (an event pair at a call boundary idles the GPU for microseconds:
    profiles/r03_o_pass_events_ab.txt), spread over the timed region."""
    from dlsm_amd import multigpu as MG

    assert MG.PASS_EVENT_SAMPLES == 4
    for steps in (1, 3, 4, 20, 100, 101):
        every = MG.event_stride(steps)
        sampled = [i for i in range(steps) if i % every == every - 1]
        assert 1 <= len(sampled) <= max(4, steps // every)
        assert sampled[-1] >= steps - every  # the region's end is sampled too
    assert MG.event_stride(20) == 5 and MG.event_stride(3) == 1


def test_too_many_gpus_exits_nonzero():
    """No silent one-GPU run: --gpus 8 where fewer GPUs are visible fails."""
    import torch

    if torch.cuda.device_count() >= 8:
        pytest.skip("this node has 8 GPUs")
    r = _bench(["--gpus", "8", "--steps", "1", "--warmup", "0", "--no-cpu", "--no-e2e"])
    assert r.returncode != 0
    assert "GPUs but only" in r.stderr, r.stderr[-2000:]


def test_gpus_must_match_launcher_world_size():
    r = _bench(["--gpus", "1", "--steps", "1", "--warmup", "0"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr, r.stderr[-2000:]
    r = _bench(["--gpus", "4", "--steps", "1", "--warmup", "0"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2


# ---------------------------------------------------------------------------
# GPU: two logical devices on GPU 0
# ---------------------------------------------------------------------------
_T, _N, _Q, _F = 16, 20_000, 1_000_003, 8


@pytest.mark.gpu
def test_two_logical_devices_strong_scaling_parity(orc):
    from dlsm_amd import multigpu as MG

    opts = MG.WorkerOptions(overlap="auto", pass_events=True)
    workers = MG.build_workers(2, [0, 0], _T, _N, _Q, _F, 10, opts,
                               lookup_stream=orc.mt_values(1000, 2 * _F * _N, _Q))
    try:
        dt = MG.timed_run(workers, steps=3, warmup=1)  # Python threads
        assert dt > 0
        workers[0].collect_pass_times()
        assert len(workers[0].probe_ms) == 3 and len(workers[1].probe_ms) == 0
        for w in workers:  # the native runner (what bench.py times) over the same buffers
            w.inp.mask.zero_()
            for o in w.inp.outs:
                o.zero_()
        dt, passes, dev_s = MG.native_timed_run(workers, steps=2, warmup=1, bits_per_key=10)
        # every device's sampled passes are timed, and each device's own time is at most the wall time
        assert dt > 0 and len(passes) == 2 and all(len(p) == 2 for p in passes)
        assert all(b > 0 and p > 0 for d in passes for b, p in d)
        assert len(dev_s) == 2 and all(0 < x <= dt * 1.001 for x in dev_s)
        # the older entry points time device 0's passes only: the
        # other devices keep their overlapped steps; pass_ms holds device 0's
        import ctypes as C

        from dlsm_amd import _lib as L
        from dlsm_amd import check, lib

        arr = (L.dlsm_device_work * 2)(*[w.device_work() for w in workers])
        for fn, every in (("dlsm_multi_device_run", None), ("dlsm_multi_device_run_sampled", 1)):
            wall, pm = C.c_double(0.0), (C.c_float * 4)(-2, -2, -2, -2)
            args = (arr, 2, 10, 2, 1) + ((every,) if every else ()) + (C.byref(wall), pm)
            check(getattr(lib(), fn)(*args), fn)
            assert wall.value > 0 and all(x > 0 for x in pm), (fn, list(pm))
        assert [w.work.tables for w in workers] == [list(range(0, 16, 2)), list(range(1, 16, 2))]
        assert [(w.work.lookup_lo, w.work.lookup_hi) for w in workers] == [(0, _Q // 2), (_Q // 2, _Q)]
        union = {}
        for w in workers:
            L = w.inp.lens.cpu().numpy()
            for j, s in enumerate(w.work.tables):
                union[s] = w.inp.outs[j][: int(L[j])].cpu().numpy().tobytes()
        for s in range(_T):
            assert union[s] == orc.full_build(orc.dbbench_keys(s, _T, _N), _N), s
        filters = [orc.full_build(orc.dbbench_keys(f, _F, _N), _N) for f in range(_F)]
        for w in workers:
            assert [f.cpu().numpy().tobytes() for f in w.inp.filters] == filters
        qk = orc.keys_from_values(orc.mt_values(1000, 2 * _F * _N, _Q))
        want = orc.full_probe(filters, qk, _Q, nthreads=8)
        got = np.concatenate([w.inp.mask[: w.work.n_lookups].cpu().numpy() for w in workers])
        assert got.size == _Q and np.array_equal(got, want)
    finally:
        for w in workers:
            w.close()


@pytest.mark.gpu
def test_bench_two_gpus_rehearsed():
    r = _bench(["--gpus", "2", "--rehearse", "--steps", "3", "--warmup", "1", "--keys-per-table", "200000",
                "--lookups", "4000000"], timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["launch"].startswith("threads")
    assert line["config"]["devices"] == [0, 0] and line["config"]["rehearsal"]
    assert line["rehearsed"] is True and line["physical_devices"] == 1
    assert line["config"]["gpu_tables"] == [list(range(0, 16, 2)), list(range(1, 16, 2))]
    assert line["config"]["gpu_lookups"] == [[0, 2_000_000], [2_000_000, 4_000_000]]
    assert line["value"] > 0 and line["roofline"]["achieved"] > 0
    # self-describing: both GPUs' pass times, the imbalance, and the CPU baseline once
    assert [g["gpu"] for g in line["per_gpu"]] == [0, 1]
    assert all(g["build_ms"] > 0 and g["probe_ms"] > 0 and g["ms_per_step"] > 0 for g in line["per_gpu"])
    assert line["imbalance"]["max_over_min_ms_per_step"] >= 1.0
    cb = line["cpu_baseline"]
    assert cb["cores"] >= 1 and cb["value"] > 0 and cb["gpu_output_matches_" + cb["kind"]]


@pytest.mark.gpu
def test_bench_one_gpu_native_and_python_loop():
    """N = 1: the default times the steps with the native runner; --python-loop
    the same calls from Python.  Both print a complete bench line."""
    base = ["--steps", "3", "--warmup", "1", "--keys-per-table", "200000", "--lookups", "4000000",
            "--no-cpu", "--no-e2e"]
    for extra, timed_by in (([], "dlsm_multi_device_run"), (["--python-loop"], "Python loop")):
        r = _bench(base + extra, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        line = json.loads(r.stdout.strip().splitlines()[-1])
        assert line["n_gpus"] == 1 and line["config"]["timed_by"].startswith(timed_by)
        assert line["rehearsed"] is False and line["physical_devices"] == 1
        assert line["value"] > 0 and line["probe"]["ms"] > 0 and line["build"]["ms"] > 0
        assert line["roofline"]["hbm_read_GBs_measured"] > 1000


@pytest.mark.gpu
def test_bench_under_launcher_two_ranks_rehearsed():
    """The driver's N > 1 launch: torch.distributed.run, one process per GPU.
    Rehearsed as two gloo ranks sharing GPU 0 (LOCAL_RANK mod device count):
    each rank times its share with the native runner between a barrier and
    the max over ranks; rank 0 prints one line for both."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        e.pop(k, None)
    e["DLSM_BENCH_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "3", "--warmup", "1", "--keys-per-table", "200000",
                        "--lookups", "4000000", "--no-cpu", "--no-e2e"],
                       capture_output=True, text=True, timeout=600, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["rehearsed"] is True and line["physical_devices"] == 1  # two ranks on one GPU
    assert line["config"]["timed_by"].startswith("dlsm_multi_device_run")
    assert line["config"]["rank0_tables"] == list(range(0, 16, 2))
    assert line["config"]["rank0_lookups"] == 2_000_000
    assert line["value"] > 0 and line["probe"]["ms"] > 0 and line["build"]["ms"] > 0
    # every rank's share, gathered to rank 0
    assert [r["gpu"] for r in line["per_gpu"]] == [0, 1]
    assert all(r["build_ms"] > 0 and r["probe_ms"] > 0 and r["probe_keys"] == 2_000_000 for r in line["per_gpu"])
    assert line["imbalance"]["max_over_min_ms_per_step"] >= 1.0
