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
