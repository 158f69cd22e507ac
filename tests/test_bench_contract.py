"""CPU checks of bench.py's reporting helpers: the committed PMC traffic
summary (profiles/traffic.json) is found for the default workload, so the
bench line's roofline.traffic is filled, and it is per launch of the dominant
pass in a plausible range of its algorithmic bytes."""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_traffic_summary_matches_default_config():
    b = _bench()
    cfg = {"tables": 16, "keys_per_table": 1_600_000, "lookups": 100_000_000, "filters": 8,
           "probe_chunk_lg": 13, "probe_slice_lg": 8}
    path = os.path.join(ROOT, "profiles", "traffic.json")
    t = b.load_traffic(path, cfg, "probe")
    assert t is not None, "profiles/traffic.json no longer matches the bench's default config"
    alg = 100_000_000 * 21 + 16_000_552  # 20 B key + 1 B mask per lookup + the filters
    assert 1.0 <= t["traffic_bytes"] / alg <= 2.5
    build = b.load_traffic(path, cfg, "build")
    assert build is not None and build["traffic_bytes"] >= 16 * 1_600_000 * 20
    # a different workload must not pick up the default's counters
    assert b.load_traffic(path, dict(cfg, lookups=12_500_000), "probe") is None
    src = json.load(open(path))["source"]
    assert src.startswith("profiles/")
    # every leg the bench line reports traffic for has its own PMC record
    for leg in ("legacy", "version", "mixed_set", "dedup_shifted", "block"):
        rec = b.load_traffic(path, cfg, leg)
        assert rec is not None and rec["traffic_bytes"] > 0, leg
    # the sealed block build moves the plain build's bytes (the crc reads LDS)
    blk = b.load_traffic(path, cfg, "block")
    assert 0.95 <= blk["traffic_bytes"] / build["traffic_bytes"] <= 1.1


def test_host_cores_positive():
    assert _bench().host_cores() >= 1


def test_step_roofline_and_pass_timing_note():
    """The whole step's algorithmic rate beside the dominant pass's own, and
    the note saying how the pass times were taken (sampled steps, run alone
    when the build overlaps the probe)."""
    b = _bench()
    step_bytes = 100_000_000 * 21 + 16_000_552 + 16 * 1_600_000 * 20 + 16 * 2_000_069
    r = b.step_roofline(step_bytes, 0.82e-3)
    assert abs(r["step_alg_GBs"] - step_bytes / 0.82e-3 / 1e9) < 0.1
    assert abs(r["step_frac"] - r["step_alg_GBs"] / b.HBM_PEAK_GBS) < 1e-4
    assert "alone" in b.pass_timing_note(True, 12)["pass_timing"]
    assert "every 12-th" in b.pass_timing_note(False, 12)["pass_timing"]


def test_threads_line_schema_per_gpu():
    """The `--gpus N` line (one process, a thread per GPU) is self-describing:
    every GPU's share with its own sampled pass times, rates and step time,
    the imbalance between the slowest and fastest GPU, and the roofline of the
    slowest GPU's dominant pass."""
    import argparse
    from types import SimpleNamespace

    b = _bench()
    n_gpu, T, N, Q, F, steps = 4, 16, 1_600_000, 100_000_000, 8, 20
    args = argparse.Namespace(steps=steps, warmup=5, rehearse=False, path=0, probe_chunk_lg=13, probe_slice_lg=8)
    workers, per_gpu = [], []
    for r in range(n_gpu):
        tables = list(range(r, T, n_gpu))
        lo, hi = Q * r // n_gpu, Q * (r + 1) // n_gpu
        workers.append(SimpleNamespace(work=SimpleNamespace(tables=tables, lookup_lo=lo, lookup_hi=hi), overlap=True))
        passes = [(0.04 + 0.001 * r, 0.17 + 0.002 * r)] * 4
        per_gpu.append(b.gpu_share_record(r, r, len(tables) * N, hi - lo, len(tables) * N * 21,
                                          (hi - lo) * 21 + 16_000_552, passes, (0.2 + 0.01 * r) * steps / 1e3,
                                          steps))
    line = b.threads_line(args, n_gpu, list(range(n_gpu)), workers, per_gpu, 0.23 * steps / 1e3, T, N, Q, F, 10)
    assert line["n_gpus"] == n_gpu and line["scaling"] == "strong"
    assert abs(line["value"] - (T * N + Q) / 0.23e-3 / 1e6) < 1
    assert [g["gpu"] for g in line["per_gpu"]] == list(range(n_gpu))
    for g in line["per_gpu"]:
        assert g["build_ms"] > 0 and g["probe_ms"] > 0 and g["ms_per_step"] > 0 and g["sampled_steps"] == 4
        assert 0 < g["probe_frac"] < 1 and 0 < g["build_frac"] < 1
    imb = line["imbalance"]
    assert imb["slowest_gpu"] == n_gpu - 1 and imb["fastest_gpu"] == 0
    assert abs(imb["max_over_min_ms_per_step"] - 0.23 / 0.2) < 1e-3
    assert line["roofline"]["kernel"].startswith("probe pass of the slowest GPU")
    assert line["roofline"]["frac"] == per_gpu[-1]["probe_frac"]
    assert line["config"]["gpu_tables"][1] == list(range(1, T, n_gpu))


def test_e2e_split_balances_cores_and_link():
    """e2e_hashed's split: the host-hashed keys take as long on the host's
    cores as the rest take on the link; tables are hashed before lookups."""
    b = _bench()
    T, N, Q, bw = 16, 1_600_000, 100_000_000, 57e9
    K = T * N + Q
    for rate in (2e9, 4e9, 8.3e9, 50e9):
        raw_t, raw_q = b.e2e_split(T, N, Q, rate, bw)
        assert 0 <= raw_t <= T and 0 <= raw_q <= Q
        hashed = (T - raw_t) * N + (Q - raw_q)
        if raw_t:  # lookups are hashed only once every table is
            assert raw_q == Q
        cores = hashed / rate
        link = (20 * (K - hashed) + 4 * hashed) / bw
        if hashed == K:  # the host outruns the link even at 4 B/key: hash everything
            assert cores <= link
        else:
            assert abs(cores - link) <= max(N, 4096) * (1 / rate + 16 / bw) + 1e-9, (rate, cores, link)
    assert b.e2e_split(T, N, Q, 1e15, bw) == (0, 0)  # a host that hashes everything
