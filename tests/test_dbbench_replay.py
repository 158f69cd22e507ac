"""dbbench_replay.py (BASELINE config 5): every filter the replay builds --
memtable flushes and leveled-compaction outputs -- and every Get's filter
answers equal the oracle's on the same streams."""
import numpy as np
import pytest

import oracle


def test_streams_match_oracle_generators():
    """The replay's Random64 streams (numpy MT19937-64) equal the oracle's C
    mt19937_64 (util/random.h:140-165) -- CPU only."""
    import dbbench_replay as R

    num, threads = 3000, 16
    fill = R.fill_stream(num, threads).reshape(num, threads)
    for t in (0, 7, 15):
        assert np.array_equal(fill[:, t], oracle.mt_values(1000 + t + 1, num * threads, num))
    reads = R.read_stream(num, threads).reshape(num, threads)
    assert np.array_equal(reads[:, 3], oracle.mt_values(1000 + threads + 3 + 1, num * threads, num))


def test_level_limits_follow_reference_constants():
    import dbbench_replay as R

    assert R.max_bytes_for_level(1) == 256 * 1048576 and R.max_bytes_for_level(3) == 25600 * 1048576
    # a 64 MiB SSTable (options.h:157) holds one memtable's worth of entries (db/memtable.h:7)
    assert R.MAX_FILE_ENTRIES == R.MEMTABLE_ENTRIES
    assert abs(R.MAX_FILE_ENTRIES * R.ENTRY_BYTES - 64 * 1048576) < 0.001 * 64 * 1048576


def _files_for_oracle(files):
    return [type("F", (), dict(level=f.level, number=f.number, smallest=f.smallest, largest=f.largest,
                               largest_trailer=f.largest_trailer, filter=f.filter)) for f in files]


@pytest.mark.gpu
def test_replay_parity_with_compactions(gpu):
    """640 K writes: 5 flushes, their L0 -> L1 compactions and L1 -> L2 spills
    (level limits scaled down so every level is exercised)."""
    import dbbench_replay as R

    built = []

    def on_build(values, filters):
        built.extend(zip(values, filters))

    reads_seen = []

    def on_read(b0, vals, masks, files):
        reads_seen.append((vals, masks, files))

    saved = R.LEVEL_BASE_BYTES
    R.LEVEL_BASE_BYTES = 2 * R.MAX_FILE_ENTRIES * R.ENTRY_BYTES  # L1 spills after 2 files
    try:
        res, lsm = R.run(40_000, 16, 10, on_build=on_build, on_read=on_read, read_batch=200_000)
    finally:
        R.LEVEL_BASE_BYTES = saved
    assert res["flushes"] == 5 and res["fill"]["compactions"] >= 5
    assert res["fill"]["compaction_builds"] > 5 and sum(res["version"]["files_per_level"][2:]) > 0
    assert res["fill"]["flush_builds"] + res["fill"]["compaction_builds"] == len(built)
    for v, f in built:  # every filter the replay built
        assert f == oracle.full_build(oracle.keys_from_values(v), v.size)
    # the final version holds every written key (a key may sit in several
    # levels: an older version below a newer one), each level key-disjoint
    allv = np.concatenate([f.values for lv in lsm.levels for f in lv])
    assert np.array_equal(np.unique(allv), np.unique(R.fill_stream(40_000, 16)))
    for lv in lsm.levels[1:]:
        assert all(a.largest < b.smallest for a, b in zip(lv, lv[1:]))
    for vals, masks, files in reads_seen[:2]:
        want, _ = oracle.version_probe(_files_for_oracle(files), oracle.keys_from_values(vals), vals.size,
                                       (1 << 56) - 1)
        assert np.array_equal(masks, want)


@pytest.mark.gpu
@pytest.mark.timeout(600)  # ~150 s of work; outlasts a suite-wide --timeout 120
def test_replay_config5_full_size(gpu):
    """BASELINE config 5 at its stated size: db_bench --num=6250000 x 16
    threads = 100 M fillrandom writes (651 flushes + leveled compactions, every
    filter built on the GPU from host keys into host slots, H2D/D2H included)
    then 100 M readrandom Gets over the final version
    (benchmarks/db_bench.cc:943-947,1232,1379-1404).  Oracle-sampled: every
    97th filter byte for byte, and the first 2 M Gets' per-file answers.
    Progress goes to gpurun_out/ every ~20 s (pytest holds stdout/stderr)."""
    import json
    import os
    import time

    import replay_fullsize_check as RC

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    prog = os.path.join(root, "gpurun_out", "replay_fullsize.progress")

    def progress(msg):
        with open(prog, "a") as f:
            f.write(f"{time.time():.0f} {msg}\n")

    res = RC.run_check(6_250_000, 16, 97, 2_000_000, progress=progress)
    chk = res["oracle_check"]
    progress("done " + json.dumps(chk))
    assert res["fill"]["writes"] == 100_000_000
    assert chk["filters_checked"] > 1000 and chk["filters_bad"] == 0
    assert chk["gets_checked"] == 2_000_000 and chk["gets_bad"] == 0
