"""dlsm_bloom_hash_batch -- the host side of the hashed build and probe:
BloomHash of every key (util/hash.cc:22-62 with the sign-extended tail;
ExtractUserKey for internal keys) on the host's cores, AVX-512 for 20-byte
keys.  Runs on the CPU (no device is touched); checked against the oracle and
the golden hashes of the compiled reference."""
import numpy as np
import pytest

import dlsm_amd


def test_hash_batch_fixed20_vs_oracle(orc):
    for n in (1, 15, 16, 17, 31, 32, 33, 63, 64, 65, 65_535, 65_536, 65_537, 300_001):
        k = orc.dbbench_keys(7, 13, n)
        got = dlsm_amd.hash_batch(dlsm_amd.Keys(k, n, 20))
        idx = np.unique(np.concatenate([np.arange(min(n, 64)), np.arange(0, n, 997), [n - 1]]))
        want = np.array([orc.bloom_hash(k[20 * i:20 * i + 20].tobytes()) for i in idx], dtype=np.uint32)
        assert np.array_equal(got[idx], want), n


def test_hash_batch_threads_agree(orc):
    n = 1_000_003
    k = orc.dbbench_keys(1, 1, n)
    a = dlsm_amd.hash_batch(dlsm_amd.Keys(k, n, 20), threads=1).copy()
    for t in (0, 2, 3):
        assert np.array_equal(dlsm_amd.hash_batch(dlsm_amd.Keys(k, n, 20), threads=t), a)


def test_hash_batch_varlen_internal_and_golden(orc, golden):
    rng = np.random.default_rng(3)
    keys = [bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8)) for _ in range(70_000)]
    data, offs = orc.pack_var(keys)
    got = dlsm_amd.hash_batch(dlsm_amd.Keys(data, len(keys), 0, offs))
    assert all(int(got[i]) == orc.bloom_hash(keys[i]) for i in range(0, len(keys), 7))
    # 28-byte internal keys hash as their 20-byte user key (ExtractUserKey)
    n = 10_000
    uk = orc.dbbench_keys(3, 5, n).reshape(n, 20)
    ik = np.ascontiguousarray(np.concatenate([uk, rng.integers(0, 256, (n, 8), dtype=np.uint8)], axis=1)).reshape(-1)
    a = dlsm_amd.hash_batch(dlsm_amd.Keys(ik, n, 28, None, 8))
    b = dlsm_amd.hash_batch(dlsm_amd.Keys(uk.reshape(-1).copy(), n, 20))
    assert np.array_equal(a, b)
    # the reference's golden hashes (sign-extended tails included)
    cases = [c for c in golden["hash"]["cases"] if c["seed"] == 0xBC9F1D34]
    assert len(cases) > 100
    ks = [bytes.fromhex(c["key"]) for c in cases]
    data, offs = orc.pack_var(ks)
    got = dlsm_amd.hash_batch(dlsm_amd.Keys(np.concatenate([data, np.zeros(16, np.uint8)]), len(ks), 0, offs))
    assert [int(x) for x in got] == [int(c["hash"]) for c in cases]


def test_hash_batch_rejects_a_short_or_wide_out(orc):
    import dlsm_amd

    k = orc.dbbench_keys(0, 1, 100)
    with pytest.raises(ValueError):
        dlsm_amd.hash_batch(dlsm_amd.Keys(k, 100, 20), out=np.empty(99, dtype=np.uint32))
    with pytest.raises(ValueError):
        dlsm_amd.hash_batch(dlsm_amd.Keys(k, 100, 20), out=np.empty(100, dtype=np.uint64))
