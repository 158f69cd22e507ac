"""Randomized soak of the version probe, the full probe and the full / legacy
builds against the oracle: the shapes of
tests/test_version_probe.py::test_gpu_version_probe_random_shapes and
tests/test_gpu_parity.py::test_full_probe_random_sets over many seeds, and
build batches of random table counts, sizes, duplicates, bits_per_key 1-24
and key lengths (checker only: the oracle is test infrastructure).
    python scripts/diag_random_soak.py [SEEDS]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import dlsm_amd  # noqa: E402
import oracle  # noqa: E402
from test_version_probe import random_version  # noqa: E402


def version_case(ctx, seed):
    rng = np.random.default_rng(10_000 + seed)
    span = int(rng.integers(1_000, 5_000_000))
    files = random_version(rng, int(rng.integers(0, 55)), span)
    n = int(rng.integers(1, 300_000))
    v_ = np.where(rng.random(n) < 0.5, rng.integers(0, span + 1, n),
                  rng.integers(0, span + span // 5 + 2, n)).astype(np.uint64)
    q = oracle.keys_from_values(v_)
    snap = int(rng.integers(1, 1 << 52))
    want, want_lf = oracle.version_probe(files, q, n, snapshot=snap)
    v = ctx.version(files)
    mask = torch.zeros(n, dtype=torch.uint64, device="cuda")
    lf = torch.zeros((n, 5), dtype=torch.int32, device="cuda")
    ctx.version_probe_dev(v, dlsm_amd.Keys(torch.from_numpy(q).cuda(), n, 20), snap, mask, lf)
    ctx.sync()
    ok = np.array_equal(mask.cpu().numpy().view(np.uint64), want) and \
        np.array_equal(lf.cpu().numpy().view(np.uint32), want_lf)
    v.close()
    return ok, len(files)


def probe_case(ctx, seed):
    rng = np.random.default_rng(20_000 + seed)
    F = int(rng.integers(1, 25))
    key_len = int(rng.choice([16, 20, 24, 28, 33]))
    equal = bool(rng.integers(0, 2))
    n_eq = int(rng.integers(1, 300_000))
    tabs = [rng.integers(0, 1 << 40, n_eq if equal else int(rng.integers(0, 300_000))).astype(np.uint64)
            for _ in range(F)]
    bpk = int(rng.integers(2, 21))
    filters = [oracle.full_build(oracle.keys_from_values(t, key_len), t.size, stride=key_len,
                                 bpk=bpk if equal else int(rng.integers(2, 21))) for t in tabs]
    nq = int(rng.integers(1, 500_000))
    pool = np.concatenate([t for t in tabs if t.size] + [np.zeros(1, np.uint64)])
    vals = np.where(rng.random(nq) < 0.5, pool[rng.integers(0, pool.size, nq)],
                    rng.integers(0, 1 << 40, nq).astype(np.uint64)).astype(np.uint64)
    q = oracle.keys_from_values(vals, key_len)
    want = oracle.full_probe(filters, q, nq, stride=key_len, nthreads=8)
    fs = ctx.filterset(filters)
    got = ctx.full_probe(fs, dlsm_amd.Keys(q, nq, key_len))
    fs.close()
    return np.array_equal(got, want), F


def build_case(ctx, seed):
    """A batch of 1-24 tables of 0-200 K keys (duplicates included), one
    bits_per_key, one key length: full and legacy filters and sealed filter
    blocks byte-equal."""
    rng = np.random.default_rng(30_000 + seed)
    T = int(rng.integers(1, 25))
    key_len = int(rng.choice([16, 20, 24, 28, 33]))
    bpk = int(rng.integers(1, 25))
    tabs = []
    for _ in range(T):
        n = int(rng.integers(0, 200_000))
        v = rng.integers(0, max(1, n // int(rng.integers(1, 4))) + 1, n).astype(np.uint64)  # some repeats
        if rng.random() < 0.5:
            v = np.sort(v)  # consecutive duplicates: AddKey's dedup
        tabs.append(oracle.keys_from_values(v, key_len))
    ns = [t.size // key_len for t in tabs]
    got = ctx.full_build([dlsm_amd.Keys(t, n, key_len) for t, n in zip(tabs, ns)], bpk)
    ok = all(g == oracle.full_build(t, n, stride=key_len, bpk=bpk) for g, t, n in zip(got, tabs, ns))
    lg = ctx.legacy_build([dlsm_amd.Keys(t, n, key_len) for t, n in zip(tabs, ns)], bpk)
    ok_l = all(g == oracle.legacy_build(t, n, stride=key_len, bpk=bpk) for g, t, n in zip(lg, tabs, ns))
    # the same batch as sealed filter blocks (crc32c fused into the slice pass)
    blk = ctx.full_build_block([dlsm_amd.Keys(t, n, key_len) for t, n in zip(tabs, ns)], bpk)
    ok_b = all(b == oracle.filter_block(g) for b, g in zip(blk, got))
    return ok and ok_l and ok_b, T


def varlen_keys(rng, vals):
    """Variable-length keys (0-40 bytes, a value's 8 bytes inside random
    padding): data (16 zero bytes past the end) and offsets[n + 1]."""
    n = vals.size
    lens = rng.integers(0, 41, n)
    parts = []
    for v, l in zip(vals.tolist(), lens.tolist()):
        b = int(v).to_bytes(8, "little") + bytes(rng.integers(0, 256, 32, dtype=np.uint8))
        parts.append(b[:l])
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(x) for x in parts])
    data = np.frombuffer(b"".join(parts) + b"\0" * 16, dtype=np.uint8).copy()
    return data, offs


def varlen_case(ctx, seed):
    """Variable-length keys: a build batch and a probe of its filters."""
    rng = np.random.default_rng(40_000 + seed)
    T = int(rng.integers(1, 10))
    bpk = int(rng.integers(2, 21))
    tabs = [varlen_keys(rng, rng.integers(0, 1 << 20, int(rng.integers(0, 60_000))).astype(np.uint64))
            for _ in range(T)]
    ns = [o.size - 1 for _, o in tabs]
    got = ctx.full_build([dlsm_amd.Keys(d, n, 0, o) for (d, o), n in zip(tabs, ns)], bpk)
    ok = all(g == oracle.full_build(d, n, offsets=o, bpk=bpk) for g, (d, o), n in zip(got, tabs, ns))
    nq = int(rng.integers(1, 200_000))
    qd, qo = varlen_keys(rng, rng.integers(0, 1 << 20, nq).astype(np.uint64))
    want = oracle.full_probe(got, qd, nq, offsets=qo)
    fs = ctx.filterset(got)
    mask = ctx.full_probe(fs, dlsm_amd.Keys(qd, nq, 0, qo))
    fs.close()
    return ok and np.array_equal(mask, want), T


def internal_case(ctx, seed):
    """Internal keys (user key + 8-byte trailer, suffix_len 8): filters and
    answers equal the user keys' (full_filter_block.cc hashes ExtractUserKey)."""
    rng = np.random.default_rng(50_000 + seed)
    T = int(rng.integers(1, 12))
    ulen = int(rng.choice([16, 20, 24]))
    bpk = int(rng.integers(2, 21))

    def internal(u, n):
        tr = rng.integers(0, 1 << 62, n).astype(np.uint64).view(np.uint8).reshape(n, 8)
        return np.ascontiguousarray(np.concatenate([u.reshape(n, ulen), tr], axis=1).reshape(-1))

    ns = [int(rng.integers(0, 150_000)) for _ in range(T)]
    users = [oracle.keys_from_values(rng.integers(0, 1 << 30, n).astype(np.uint64), ulen) for n in ns]
    got = ctx.full_build([dlsm_amd.Keys(internal(u, n), n, ulen + 8, suffix_len=8) for u, n in zip(users, ns)], bpk)
    ok = all(g == oracle.full_build(u, n, stride=ulen, bpk=bpk) for g, u, n in zip(got, users, ns))
    nq = int(rng.integers(1, 300_000))
    qu = oracle.keys_from_values(rng.integers(0, 1 << 30, nq).astype(np.uint64), ulen)
    want = oracle.full_probe(got, qu, nq, stride=ulen, nthreads=8)
    fs = ctx.filterset(got)
    mask = ctx.full_probe(fs, dlsm_amd.Keys(internal(qu, nq), nq, ulen + 8, suffix_len=8))
    fs.close()
    return ok and np.array_equal(mask, want), T


def main():
    seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    ctx = dlsm_amd.Context(0)
    bad = []
    t0 = time.time()
    for s in range(seeds):
        ok, nf = version_case(ctx, s)
        if not ok:
            bad.append(("version", s, nf))
        ok, F = probe_case(ctx, s)
        if not ok:
            bad.append(("probe", s, F))
        ok, T = build_case(ctx, s)
        if not ok:
            bad.append(("build", s, T))
        ok, T = varlen_case(ctx, s)
        if not ok:
            bad.append(("varlen", s, T))
        ok, T = internal_case(ctx, s)
        if not ok:
            bad.append(("internal", s, T))
        if s % 10 == 9:
            print(f"seed {s + 1}/{seeds}: {len(bad)} mismatches, {time.time() - t0:.0f} s", flush=True)
    ctx.close()
    print("soak:", seeds, "version cases,", seeds, "probe cases,", seeds, "build batches (full + legacy + sealed blocks),", seeds,
          "variable-length and", seeds, "internal-key build + probe cases, mismatches:",
          bad, flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
