"""dbbench_replay.py (BASELINE config 5): the replayed flush filters and Get
probes equal the oracle's on the same streams."""
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


@pytest.mark.gpu
def test_replay_parity(gpu):
    import dbbench_replay as R

    res, (mem, filters, reads, masks) = R.run(20_000, 16, 10, reps=1)
    assert res["flushes"] == len(mem) == 3
    for v, f in zip(mem, filters):
        assert f == oracle.full_build(oracle.keys_from_values(v), v.size)
    files = [type("F", (), dict(level=0, number=j + 1, smallest=oracle.keys_from_values(v[:1]).tobytes(),
                                largest=oracle.keys_from_values(v[-1:]).tobytes(),
                                largest_trailer=(1 << 8) | 1, filter=f))
             for j, (v, f) in enumerate(zip(mem, filters))]
    sample = slice(0, 50_000)
    want, _ = oracle.version_probe(files, oracle.keys_from_values(reads[sample]), 50_000, (1 << 56) - 1)
    assert np.array_equal(masks[sample], want)
