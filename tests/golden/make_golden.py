"""Generate the committed golden fixtures from the dLSM reference itself.

Runs ONLY in the build container, where /root/reference is mounted: it calls
the reference sources compiled in place (oracle/_ref/libref.so, built by
oracle/build_ref.sh from util/hash.cc, util/bloom.cc, util/filter_policy.cc and
util/bloom_impl.h -- see oracle/ref_driver.cc).  The fixtures are pure data
(inputs and expected outputs); nothing here is reference source.

    python tests/golden/make_golden.py

Outputs tests/golden/{hash,full,legacy,probe}.json.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle  # noqa: E402

SEED = 0xbc9f1d34


def R():
    r = oracle.ref_lib()
    if r is None:
        oracle.build()
        r = oracle.ref_lib()
    if r is None:
        sys.exit("reference not available: run in the build container")
    return r


def dbkey(v: int, ks: int = 20) -> bytes:
    return oracle.dbbench_keys(v, 1, 1, ks).tobytes()


def pack(keys):
    offs = np.zeros(len(keys) + 1, dtype=np.uint64)
    if keys:
        offs[1:] = np.cumsum([len(k) for k in keys])
    return b"".join(keys) + b"\0", offs


def ref_full(keys, bpk=10) -> bytes:
    data, offs = pack(keys)
    cap = 64 * ((len(keys) * max(bpk, 1)) // 512 + 4) + 64
    out = C.create_string_buffer(cap)
    n = R().ref_full_build(data, offs.ctypes.data_as(oracle.u64p), len(keys), bpk, out, cap)
    assert n > 0
    return out.raw[:n]


def ref_legacy(keys, bpk=10) -> bytes:
    data, offs = pack(keys)
    cap = (len(keys) * bpk) // 8 + 64
    out = C.create_string_buffer(cap)
    n = R().ref_legacy_create(data, offs.ctypes.data_as(oracle.u64p), len(keys), bpk, out)
    return out.raw[:n]


def hx(b: bytes) -> str:
    return b.hex()


def main():
    rng = random.Random(20241015)
    # ---------------- hash ----------------
    kat_inputs = [
        (b"", SEED), (bytes([0x62]), SEED), (bytes([0xc3, 0x97]), SEED),
        (bytes([0xe2, 0x99, 0xa5]), SEED), (bytes([0xe1, 0x80, 0xb9, 0x32]), SEED),
        (bytes([0x01, 0xc0] + [0] * 14 + [0x14, 0, 0, 0, 0, 0, 4, 0, 0, 0, 0, 0x14, 0, 0, 0, 0x18,
                                         0x28] + [0] * 7 + [2] + [0] * 7), 0x12345678),
    ]
    hashes = []
    for k, s in kat_inputs:
        hashes.append({"key": hx(k), "seed": s, "hash": R().ref_hash(k, len(k), s), "src": "hash_test.cc"})
    for ln in range(0, 65):
        for _ in range(3):
            k = bytes(rng.randrange(256) for _ in range(ln))
            hashes.append({"key": hx(k), "seed": SEED, "hash": R().ref_hash(k, len(k), SEED)})
    for v in [0, 1, 2, 255, 256, 1 << 32, 25_599_999, (1 << 64) - 1]:
        k = dbkey(v)
        hashes.append({"key": hx(k), "seed": SEED, "hash": R().ref_bloom_hash(k, len(k))})
    with open(os.path.join(HERE, "hash.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (reference util/hash.cc)",
                   "cases": hashes}, f, indent=0)

    # ---------------- full filters ----------------
    full = []
    for n in [1, 2, 3, 7, 51, 52, 100, 1000, 4096]:
        keys = [dbkey(v) for v in range(n)]
        full.append({"name": f"dbbench_seq_{n}", "kind": "dbbench", "first": 0, "step": 1, "n": n,
                     "bpk": 10, "filter": hx(ref_full(keys))})
    for bpk in [1, 2, 5, 16, 20, 44, 50]:
        keys = [dbkey(v) for v in range(0, 3000, 3)]
        full.append({"name": f"dbbench_bpk{bpk}", "kind": "dbbench", "first": 0, "step": 3,
                     "n": 1000, "bpk": bpk, "filter": hx(ref_full(keys, bpk))})
    # variable-length keys incl. tails with bytes >= 0x80
    for n in [1, 5, 77, 1500]:
        keys = [bytes(rng.randrange(256) for _ in range(rng.randrange(0, 40))) for _ in range(n)]
        full.append({"name": f"varlen_{n}", "kind": "var", "keys": [hx(k) for k in keys],
                     "n": n, "bpk": 10, "filter": hx(ref_full(keys))})
    # dedup: a run of identical keys
    keys = [dbkey(7)] * 100
    full.append({"name": "dup_run_100", "kind": "var", "keys": [hx(k) for k in keys], "n": 100,
                 "bpk": 10, "filter": hx(ref_full(keys))})
    # dedup changing the line count: 52 keys with one adjacent repeat -> 51 distinct
    keys = [dbkey(v) for v in range(51)]
    keys.insert(20, keys[20])
    full.append({"name": "dup_changes_L_52", "kind": "var", "keys": [hx(k) for k in keys], "n": 52,
                 "bpk": 10, "filter": hx(ref_full(keys))})
    # non-adjacent repeat (not deduplicated by the reference)
    keys = [dbkey(v) for v in range(51)] + [dbkey(0)]
    full.append({"name": "dup_nonadjacent_52", "kind": "var", "keys": [hx(k) for k in keys],
                 "n": 52, "bpk": 10, "filter": hx(ref_full(keys))})
    # two distinct keys with the same BloomHash, adjacent (found by birthday
    # search over random 64-bit v: for v < 2^32 the 20-byte db_bench key hash is
    # a bijection of v, so sequential v never collide)
    vals = oracle.mt_values(4242, 1 << 64 - 1, 400_000)
    hs = np.empty(vals.size, dtype=np.uint32)
    kb = oracle.keys_from_values(vals, 20)
    for i in range(vals.size):
        hs[i] = oracle.bloom_hash(kb[i * 20:(i + 1) * 20].tobytes())
    order = np.argsort(hs, kind="stable")
    dup = np.nonzero(hs[order][1:] == hs[order][:-1])[0]
    pair = None
    for d in dup:
        a, b = int(vals[order[d]]), int(vals[order[d + 1]])
        if a != b:
            pair = (a, b)
            break
    assert pair is not None
    assert R().ref_bloom_hash(dbkey(pair[0]), 20) == R().ref_bloom_hash(dbkey(pair[1]), 20)
    a, b = pair
    keys = [dbkey(x) for x in range(40)] + [dbkey(a), dbkey(b)] + [dbkey(x) for x in range(100, 110)]
    full.append({"name": "hash_collision_adjacent", "kind": "var", "keys": [hx(k) for k in keys],
                 "n": len(keys), "bpk": 10, "collide_values": [a, b], "filter": hx(ref_full(keys))})
    # large: digests only (bytes too big to commit)
    digests = []
    for n in [153_846, 1_600_000]:
        keys_np = oracle.dbbench_keys(0, 1, n)
        data = keys_np.tobytes()
        keys = [data[i * 20:(i + 1) * 20] for i in range(n)]
        f = ref_full(keys)
        digests.append({"name": f"dbbench_seq_{n}", "first": 0, "step": 1, "n": n, "bpk": 10,
                        "len": len(f), "fnv1a64": oracle.fnv1a64(f)})
        lf = ref_legacy(keys)
        digests.append({"name": f"legacy_dbbench_seq_{n}", "first": 0, "step": 1, "n": n, "bpk": 10,
                        "len": len(lf), "fnv1a64": oracle.fnv1a64(lf), "format": "legacy"})
    # the 16 config-4 tables at 153,846 keys (v = 16 i + s)
    for s in [0, 5, 15]:
        n = 153_846
        data = oracle.dbbench_keys(s, 16, n).tobytes()
        keys = [data[i * 20:(i + 1) * 20] for i in range(n)]
        f = ref_full(keys)
        digests.append({"name": f"config4_table{s}_{n}", "first": s, "step": 16, "n": n, "bpk": 10,
                        "len": len(f), "fnv1a64": oracle.fnv1a64(f)})
    # filter blocks as FinishFilterBlock writes them (table_builder_computeside.cc:418-428):
    # filter + [type 0] + Fixed32(crc32c::Mask(crc32c::Extend(Value(filter), type)))
    blocks = []
    for c in full:
        if c["bpk"] != 10:
            continue
        fb = bytes.fromhex(c["filter"])
        crc = R().ref_crc32c_extend(R().ref_crc32c_extend(0, fb, len(fb)), b"\0", 1)
        blocks.append({"name": c["name"], "trailer": (b"\0" + R().ref_crc32c_mask(crc).to_bytes(4, "little")).hex()})
    for d in digests:
        if d.get("format") == "legacy":
            continue
        keys_np = oracle.dbbench_keys(d["first"], d["step"], d["n"]).tobytes()
        fb = ref_full([keys_np[i * 20:(i + 1) * 20] for i in range(d["n"])])
        crc = R().ref_crc32c_extend(R().ref_crc32c_extend(0, fb, len(fb)), b"\0", 1)
        d["block_trailer"] = (b"\0" + R().ref_crc32c_mask(crc).to_bytes(4, "little")).hex()
    crc_kats = []
    for data in [bytes(32), b"\xff" * 32, bytes(range(32)), bytes(range(31, -1, -1)), b"hello world", b"",
                 bytes([0x01, 0xc0] + [0] * 14 + [0x14, 0, 0, 0, 0, 0, 4, 0, 0, 0, 0, 0x14, 0, 0, 0, 0x18,
                                               0x28] + [0] * 7 + [2] + [0] * 7)]:
        crc_kats.append({"data": data.hex(), "crc": R().ref_crc32c_extend(0, data, len(data))})
    with open(os.path.join(HERE, "full.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (reference bloom_impl.h AddHash, crc32c.cc)",
                   "cases": full, "digests": digests, "blocks": blocks, "crc32c": crc_kats}, f, indent=0)

    # ---------------- legacy (util/bloom.cc) ----------------
    leg = []
    for n in [0, 1, 2, 3, 6, 7, 100, 1000]:
        keys = [dbkey(v) for v in range(n)]
        leg.append({"name": f"dbbench_seq_{n}", "kind": "dbbench", "first": 0, "step": 1, "n": n,
                    "bpk": 10, "filter": hx(ref_legacy(keys))})
    for n in [3, 200]:
        keys = [bytes(rng.randrange(256) for _ in range(rng.randrange(0, 30))) for _ in range(n)]
        leg.append({"name": f"varlen_{n}", "kind": "var", "keys": [hx(k) for k in keys], "n": n,
                    "bpk": 10, "filter": hx(ref_legacy(keys))})
    # bloom_test.cc Small: "hello","world"
    keys = [b"hello", b"world"]
    f = ref_legacy(keys)
    small = {"filter": hx(f), "queries": {}}
    for q in [b"hello", b"world", b"x", b"foo"]:
        small["queries"][q.decode()] = R().ref_legacy_may_match(q, len(q), f, len(f))
    # reader edge cases run through the reference KeyMayMatch
    edges = []
    base = bytearray(ref_legacy([dbkey(v) for v in range(10)]))
    for kb in [0, 1, 6, 30, 31, 100, 127, 128, 200, 255]:
        fb = bytes(base[:-1]) + bytes([kb])
        qs = []
        for v in range(0, 40):
            k = dbkey(v)
            qs.append(R().ref_legacy_may_match(k, 20, fb, len(fb)))
        edges.append({"filter": hx(fb), "k_byte": kb, "query_first": 0, "answers": qs})
    for fb in [b"", b"\x06"]:
        k = dbkey(1)
        edges.append({"filter": hx(fb), "query_first": 1, "answers": [R().ref_legacy_may_match(k, 20, fb, len(fb))]})
    with open(os.path.join(HERE, "legacy.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (reference util/bloom.cc)",
                   "cases": leg, "small": small, "edges": edges}, f, indent=0)

    # ---------------- probe booleans (full filters) ----------------
    probe = {"filters": [], "queries": {"first": 0, "step": 1, "n": 10_000}, "answers": []}
    specs = [(0, 2, 1000), (1, 2, 2500), (0, 1, 4096), (5000, 7, 600)]
    fl = []
    for first, step, n in specs:
        keys = [dbkey(first + i * step) for i in range(n)]
        f = ref_full(keys)
        fl.append(f)
        probe["filters"].append({"first": first, "step": step, "n": n, "bpk": 10, "filter": hx(f)})
    for f in fl:
        ans = bytearray()
        for v in range(10_000):
            k = dbkey(v)
            ans.append(R().ref_full_may_match(k, 20, f, len(f)))
        probe["answers"].append(hx(bytes(ans)))
    # the reader ctor's two accepted layouts (full_filter_block.cc:239-249):
    # num_lines * 64 == len (log2 line 6) and len % num_lines == 0 (log2 line
    # left at 0), random filter bodies, through the reference's probe
    rng = random.Random(20261017)
    branches = []
    for L, line_bytes, k in [(3, 32, 6), (5, 8, 4), (1, 7, 2), (7, 128, 6), (2, 1, 1), (9, 64, 6)]:
        body = bytes(rng.randrange(256) for _ in range(L * line_bytes))
        fb = body + bytes([k]) + L.to_bytes(4, "little")
        ans = bytearray()
        for v in range(5_000):
            kk = dbkey(v)
            r = R().ref_full_may_match_any(kk, 20, fb, len(fb))
            assert r in (0, 1)
            ans.append(r)
        branches.append({"num_lines": L, "line_bytes": line_bytes, "k": k, "filter": hx(fb),
                         "answers": hx(bytes(ans))})
    probe["reader_branches"] = {"queries": {"first": 0, "step": 1, "n": 5_000}, "cases": branches}
    with open(os.path.join(HERE, "probe.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (reference bloom_impl.h HashMayMatch)",
                   **probe}, f, indent=0)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
