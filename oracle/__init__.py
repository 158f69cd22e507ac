"""CPU oracle for the dLSM Bloom-filter hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker / the timed CPU baseline.
The product path (``dlsm_amd``) never imports it.

``liboracle.so`` is the plain-C restatement (``bloom_oracle.c``); ``_ref/libref.so``
is the reference compiled in place (this container only, see ``build_ref.sh``).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None

u8p = C.POINTER(C.c_uint8)
u64p = C.POINTER(C.c_uint64)


def build(quiet: bool = True) -> None:
    """Compile liboracle.so (and _ref/libref.so when the reference is mounted)."""
    out = subprocess.DEVNULL if quiet else None
    subprocess.run(["make", "-C", _HERE, "liboracle.so"], check=True, stdout=out)
    subprocess.run(["bash", os.path.join(_HERE, "build_ref.sh")], check=True, stdout=out)


def _ptr(a, t=u8p):
    if a is None:
        return None
    return a.ctypes.data_as(t)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.orc_hash.restype = C.c_uint32
        L.orc_hash.argtypes = [u8p, C.c_size_t, C.c_uint32]
        L.orc_bloom_hash.restype = C.c_uint32
        L.orc_bloom_hash.argtypes = [u8p, C.c_size_t]
        L.orc_full_num_probes.argtypes = [C.c_int]
        L.orc_legacy_num_probes.argtypes = [C.c_int]
        L.orc_full_filter_bytes.restype = C.c_uint64
        L.orc_full_filter_bytes.argtypes = [C.c_uint64, C.c_int, C.POINTER(C.c_uint32)]
        L.orc_full_dedup_count.restype = C.c_uint64
        L.orc_full_dedup_count.argtypes = [u8p, u64p, C.c_uint32, C.c_uint64]
        L.orc_full_build.restype = C.c_int64
        L.orc_full_build.argtypes = [u8p, u64p, C.c_uint32, C.c_uint64, C.c_int, u8p, C.c_uint64]
        L.orc_internal_keys_select.restype = C.c_int64
        L.orc_internal_keys_select.argtypes = [u8p, u64p, C.c_uint32, C.c_uint64, C.c_int,
                                               C.c_uint64, u8p, u64p]
        L.orc_version_probe.argtypes = [C.c_void_p, C.c_int, u8p, u64p, C.c_uint32, C.c_uint32,
                                        C.c_uint64, C.c_uint64, u64p, C.POINTER(C.c_uint32)]
        L.orc_filter_block_build.restype = C.c_int64
        L.orc_filter_block_build.argtypes = [u8p, u64p, C.c_uint32, C.c_uint64, u64p, u64p, C.c_int,
                                             C.c_int, C.c_int, u8p, C.c_uint64]
        L.orc_filter_block_key_may_match.argtypes = [u8p, C.c_uint64, C.c_uint64, u8p, C.c_size_t,
                                                     C.c_int]
        L.orc_full_reader_parse.argtypes = [u8p, C.c_uint64, C.POINTER(C.c_int),
                                            C.POINTER(C.c_uint32), C.POINTER(C.c_int)]
        L.orc_full_key_may_match.argtypes = [u8p, C.c_uint64, u8p, C.c_size_t]
        L.orc_legacy_filter_bytes.restype = C.c_uint64
        L.orc_legacy_filter_bytes.argtypes = [C.c_uint64, C.c_int]
        L.orc_legacy_build.restype = C.c_int64
        L.orc_legacy_build.argtypes = [u8p, u64p, C.c_uint32, C.c_uint64, C.c_int, u8p, C.c_uint64]
        L.orc_legacy_key_may_match.argtypes = [u8p, C.c_uint64, u8p, C.c_size_t]
        L.orc_gen_keys_arith.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, u8p]
        L.orc_gen_values_mt.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, u64p]
        L.orc_gen_keys_from_values.argtypes = [u64p, C.c_uint64, C.c_int, u8p]
        L.orc_fnv1a64.restype = C.c_uint64
        L.orc_fnv1a64.argtypes = [u8p, C.c_uint64]
        L.orc_full_build_many.argtypes = [C.POINTER(u8p), u64p, C.c_uint32, C.c_int, C.c_int,
                                          C.POINTER(u8p), u64p, C.POINTER(C.c_int64), C.c_int]
        L.orc_full_probe_many.argtypes = [C.POINTER(u8p), u64p, C.c_int, u8p, C.c_uint32,
                                          C.c_uint64, u8p, C.c_int]
        L.orc_full_probe_var.argtypes = [C.POINTER(u8p), u64p, C.c_int, u8p, u64p, C.c_uint32,
                                         C.c_uint64, u8p]
        L.orc_legacy_probe.argtypes = [u8p, C.c_uint64, u8p, u64p, C.c_uint32, C.c_uint64, u8p]
        L.orc_crc32c_extend.restype = C.c_uint32
        L.orc_crc32c_extend.argtypes = [C.c_uint32, u8p, C.c_uint64]
        L.orc_crc32c_mask.restype = C.c_uint32
        L.orc_crc32c_mask.argtypes = [C.c_uint32]
        _LIB = L
    return _LIB


def timed_cpu_baseline(kind: str, tables, n: int, filters: list, q: np.ndarray, nq: int, bpk: int,
                       threads: int, legacy_tables: int | None = None):
    """Time the CPU path on the host: kind "reference" = the reference's own
    code (oracle/_ref/libref.so: util/bloom_impl.h AddHash / HashMayMatch,
    util/hash.cc, util/bloom.cc), kind "port" = this oracle's C restatement.
    Cost structure of the reference: one SSTable per thread for the builds
    (hash -> vector -> scatter, FullFilterBlockBuilder), the lookups split over
    the threads with BloomHash recomputed per filter (FullFilterBlockReader::
    KeyMayMatch), and util/bloom.cc CreateFilter (the legacy FilterPolicy
    format) over the first `legacy_tables` tables.  Returns a dict of times
    (s) and outputs, or None for "reference" without libref.so."""
    import time
    from concurrent.futures import ThreadPoolExecutor

    R = ref_lib() if kind == "reference" else None
    if kind == "reference" and R is None:
        return None
    L = lib()
    offs = np.arange(n + 1, dtype=np.uint64) * 20
    cap = full_filter_bytes(n, bpk)[0] + 64
    lcap = int(L.orc_legacy_filter_bytes(n, bpk)) + 64

    def build_one(t):
        out = np.zeros(cap, dtype=np.uint8)
        if R is not None:
            ln = R.ref_full_build(t.ctypes.data_as(C.c_char_p), _ptr(offs, u64p), n, bpk, out.ctypes.data, cap)
        else:
            ln = L.orc_full_build(_ptr(t), None, 20, n, bpk, _ptr(out), cap)
        return out[:ln].tobytes()

    def legacy_one(t):
        out = np.zeros(lcap, dtype=np.uint8)
        if R is not None:
            ln = R.ref_legacy_create(t.ctypes.data_as(C.c_char_p), _ptr(offs, u64p), n, bpk, out.ctypes.data)
        else:
            ln = L.orc_legacy_build(_ptr(t), None, 20, n, bpk, _ptr(out), lcap)
        return out[:ln].tobytes()

    fa = [np.frombuffer(f, dtype=np.uint8) for f in filters]
    fp = (C.c_void_p * len(fa))(*[a.ctypes.data for a in fa])
    fpu = (u8p * len(fa))(*[_ptr(a) for a in fa])
    fl = np.array([a.size for a in fa], dtype=np.uint64)
    mask = np.zeros(max(nq, 1), dtype=np.uint8)

    def probe_part(r):
        lo, hi = nq * r // threads, nq * (r + 1) // threads
        if hi <= lo:
            return
        if R is not None:
            R.ref_full_probe_many(fp, _ptr(fl, u64p), len(fa), q[lo * 20:].ctypes.data_as(C.c_char_p),
                                  hi - lo, 20, mask[lo:].ctypes.data)
        else:
            L.orc_full_probe_many(fpu, _ptr(fl, u64p), len(fa), _ptr(q[lo * 20:]), 20, hi - lo,
                                  _ptr(mask[lo:]), 1)

    nl = len(tables) if legacy_tables is None else legacy_tables
    with ThreadPoolExecutor(max_workers=threads) as ex:  # ctypes calls release the GIL
        t0 = time.perf_counter()
        built = list(ex.map(build_one, tables))
        t1 = time.perf_counter()
        list(ex.map(probe_part, range(threads)))
        t2 = time.perf_counter()
        leg = list(ex.map(legacy_one, tables[:nl]))
        t3 = time.perf_counter()
    return {"build_s": t1 - t0, "probe_s": t2 - t1, "legacy_s": t3 - t2, "legacy_tables": nl,
            "built": built, "mask": mask[:nq], "legacy": leg}


def ref_lib():
    """The reference compiled in place, or None (GPU box / reference absent)."""
    global _REF
    if _REF is None:
        path = os.path.join(_HERE, "_ref", "libref.so")
        if not os.path.exists(path):
            return None
        R = C.CDLL(path)
        cp = C.c_char_p
        R.ref_hash.restype = C.c_uint32
        R.ref_hash.argtypes = [cp, C.c_size_t, C.c_uint32]
        R.ref_bloom_hash.restype = C.c_uint32
        R.ref_bloom_hash.argtypes = [cp, C.c_size_t]
        R.ref_legacy_create.restype = C.c_int64
        R.ref_legacy_create.argtypes = [cp, u64p, C.c_int, C.c_int, C.c_void_p]
        R.ref_legacy_may_match.argtypes = [cp, C.c_size_t, cp, C.c_size_t]
        R.ref_full_build.restype = C.c_int64
        R.ref_full_build.argtypes = [cp, u64p, C.c_uint64, C.c_int, C.c_void_p, C.c_uint64]
        R.ref_full_may_match.argtypes = [cp, C.c_size_t, cp, C.c_size_t]
        R.ref_full_may_match_any.argtypes = [cp, C.c_size_t, cp, C.c_size_t]
        R.ref_full_probe_many.restype = None
        R.ref_full_probe_many.argtypes = [C.POINTER(C.c_void_p), u64p, C.c_int, cp, C.c_uint64,
                                          C.c_uint32, C.c_void_p]
        R.ref_crc32c_extend.restype = C.c_uint32
        R.ref_crc32c_extend.argtypes = [C.c_uint32, cp, C.c_size_t]
        R.ref_crc32c_mask.restype = C.c_uint32
        R.ref_crc32c_mask.argtypes = [C.c_uint32]
        _REF = R
    return _REF


# ---------------------------------------------------------------------------
# Key sets.  A key set is (bytes: uint8[...], offsets: uint64[n+1] | None,
# stride: int, n: int).  Fixed-stride sets have offsets=None.
# ---------------------------------------------------------------------------

def dbbench_keys(first: int, step: int, n: int, key_size: int = 20) -> np.ndarray:
    """Keys v = first + i*step (db_bench GenerateKeyFromInt), packed [n, key_size]."""
    out = np.empty(n * key_size, dtype=np.uint8)
    lib().orc_gen_keys_arith(first, step, n, key_size, _ptr(out))
    return out


def mt_values(seed: int, modulus: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.uint64)
    lib().orc_gen_values_mt(seed, modulus, n, _ptr(out, u64p))
    return out


def keys_from_values(v: np.ndarray, key_size: int = 20) -> np.ndarray:
    v = np.ascontiguousarray(v, dtype=np.uint64)
    out = np.empty(v.size * key_size, dtype=np.uint8)
    lib().orc_gen_keys_from_values(_ptr(v, u64p), v.size, key_size, _ptr(out))
    return out


def pack_var(keys: list[bytes]):
    offs = np.zeros(len(keys) + 1, dtype=np.uint64)
    if keys:
        offs[1:] = np.cumsum([len(k) for k in keys])
    data = np.frombuffer(b"".join(keys) + b"\0", dtype=np.uint8).copy()
    return data, offs


def bloom_hash(key: bytes) -> int:
    a = np.frombuffer(key + b"\0", dtype=np.uint8)
    return int(lib().orc_bloom_hash(_ptr(a), len(key)))


def hash_seed(key: bytes, seed: int) -> int:
    a = np.frombuffer(key + b"\0", dtype=np.uint8)
    return int(lib().orc_hash(_ptr(a), len(key), seed))


def full_filter_bytes(n_dedup: int, bpk: int = 10):
    nl = C.c_uint32(0)
    b = lib().orc_full_filter_bytes(n_dedup, bpk, C.byref(nl))
    return int(b), int(nl.value)


def full_build(keys: np.ndarray, n: int, stride: int = 20, offsets=None, bpk: int = 10) -> bytes:
    if offsets is None:
        nd = n
    else:
        nd = n
    cap = full_filter_bytes(nd, bpk)[0]
    out = np.zeros(cap, dtype=np.uint8)
    r = lib().orc_full_build(_ptr(keys), _ptr(offsets, u64p), stride, n, bpk, _ptr(out), cap)
    if r < 0:
        raise RuntimeError(f"orc_full_build: {r}")
    return out[:r].tobytes()


def full_dedup_count(keys, n, stride=20, offsets=None) -> int:
    return int(lib().orc_full_dedup_count(_ptr(keys), _ptr(offsets, u64p), stride, n))


def internal_keys_select(keys: np.ndarray, n: int, policy: int, snapshot: int,
                         stride: int = 28, offsets=None):
    """Flush (policy 0) / compaction (1) selection over internal keys:
    returns (keep u8[n], n_kept or -1 when a flush aborts, first_corrupt)."""
    keep = np.zeros(max(n, 1), dtype=np.uint8)
    bad = np.zeros(1, dtype=np.uint64)
    r = lib().orc_internal_keys_select(_ptr(keys), _ptr(offsets, u64p), stride, n, policy, snapshot,
                                       _ptr(keep), _ptr(bad, u64p))
    return keep[:n], int(r), int(bad[0])


def internal_key(user_key: bytes, seq: int, vtype: int = 1) -> bytes:
    """user_key || Fixed64(seq << 8 | type) (db/dbformat.h:115-118, AppendInternalKey)."""
    return user_key + ((seq << 8) | vtype).to_bytes(8, "little")


class _VFile(C.Structure):  # same layout as dlsm_version_file
    _fields_ = [("smallest", C.c_void_p), ("smallest_len", C.c_uint64),
                ("largest", C.c_void_p), ("largest_len", C.c_uint64),
                ("largest_trailer", C.c_uint64), ("number", C.c_uint64),
                ("level", C.c_int32), ("reserved", C.c_int32),
                ("filter", C.c_void_p), ("filter_len", C.c_uint64)]


def version_probe(files, keys: np.ndarray, n: int, snapshot: int, stride: int = 20,
                  offsets=None, suffix: int = 0):
    """ForEachOverlapping + FindFile + the filter check, restated
    (orc_version_probe).  files: objects with level, number, smallest, largest,
    largest_trailer, filter (bytes or None).  Returns (mask u64[n], level_file u32[n, 5])."""
    arr = (_VFile * max(len(files), 1))()
    keep = []
    for j, f in enumerate(files):
        sm = np.frombuffer(bytes(f.smallest) + b"\0", dtype=np.uint8)
        lg = np.frombuffer(bytes(f.largest) + b"\0", dtype=np.uint8)
        keep += [sm, lg]
        fp, fl = None, 0
        if f.filter is not None:
            fa = np.frombuffer(bytes(f.filter), dtype=np.uint8)
            keep.append(fa)
            fp, fl = fa.ctypes.data, fa.size
        arr[j] = _VFile(sm.ctypes.data, len(f.smallest), lg.ctypes.data, len(f.largest),
                        f.largest_trailer, f.number, f.level, 0, fp, fl)
    mask = np.zeros(max(n, 1), dtype=np.uint64)
    lf = np.zeros((max(n, 1), 5), dtype=np.uint32)
    st = lib().orc_version_probe(arr, len(files), _ptr(keys), _ptr(offsets, u64p), stride, suffix, n,
                                 snapshot, _ptr(mask, u64p), lf.ctypes.data_as(C.POINTER(C.c_uint32)))
    assert st == 0, st
    return mask[:n], lf[:n]


def filter_block_build(keys: np.ndarray, n: int, block_key_end, block_end_offset,
                       stride: int = 20, offsets=None, policy: int = 0, bpk: int = 10) -> bytes:
    """FilterBlockBuilder driven like TableBuilder (orc_filter_block_build).
    policy 0 = BloomFilterPolicy, 1 = filter_block_test.cc's TestHashFilter."""
    ke = np.asarray(block_key_end, dtype=np.uint64)
    eo = np.asarray(block_end_offset, dtype=np.uint64)
    cap = 64 + 8 * (len(ke) + int(eo.max() // 2048 if len(eo) else 0) + 2) + 16 * n + n * bpk // 8 * 2 + 4096
    out = np.zeros(cap, dtype=np.uint8)
    r = lib().orc_filter_block_build(_ptr(keys), _ptr(offsets, u64p), stride, n, _ptr(ke, u64p),
                                     _ptr(eo, u64p), len(ke), policy, bpk, _ptr(out), cap)
    if r < 0:
        raise ValueError(f"orc_filter_block_build: {r}")
    return out[:r].tobytes()


def filter_block_key_may_match(block: bytes, block_offset: int, key: bytes, policy: int = 0) -> int:
    b = np.frombuffer(block + b"\0", dtype=np.uint8)
    k = np.frombuffer(key + b"\0", dtype=np.uint8)
    return lib().orc_filter_block_key_may_match(_ptr(b), len(block), block_offset, _ptr(k), len(key),
                                                policy)


def full_reader_parse(filt: bytes):
    a = np.frombuffer(filt + b"\0", dtype=np.uint8)
    k, L, lg = C.c_int(0), C.c_uint32(0), C.c_int(0)
    st = lib().orc_full_reader_parse(_ptr(a), len(filt), C.byref(k), C.byref(L), C.byref(lg))
    return st, k.value, L.value, lg.value


def full_probe(filters: list[bytes], keys: np.ndarray, n: int, stride: int = 20,
               offsets=None, nthreads: int = 1) -> np.ndarray:
    F = len(filters)
    fa = [np.frombuffer(f, dtype=np.uint8) for f in filters]
    fptrs = (u8p * F)(*[_ptr(a) for a in fa])
    flen = np.array([len(f) for f in filters], dtype=np.uint64)
    mb = (F + 7) // 8
    mask = np.zeros(n * mb, dtype=np.uint8)
    if offsets is None:
        st = lib().orc_full_probe_many(fptrs, _ptr(flen, u64p), F, _ptr(keys), stride, n,
                                       _ptr(mask), nthreads)
    else:
        st = lib().orc_full_probe_var(fptrs, _ptr(flen, u64p), F, _ptr(keys), _ptr(offsets, u64p),
                                      stride, n, _ptr(mask))
    if st:
        raise RuntimeError(f"orc probe status {st}")
    return mask


def full_key_may_match(filt: bytes, key: bytes) -> int:
    a = np.frombuffer(filt + b"\0", dtype=np.uint8)
    k = np.frombuffer(key + b"\0", dtype=np.uint8)
    return int(lib().orc_full_key_may_match(_ptr(a), len(filt), _ptr(k), len(key)))


def legacy_build(keys: np.ndarray, n: int, stride: int = 20, offsets=None, bpk: int = 10) -> bytes:
    cap = int(lib().orc_legacy_filter_bytes(n, bpk))
    out = np.zeros(cap, dtype=np.uint8)
    r = lib().orc_legacy_build(_ptr(keys), _ptr(offsets, u64p), stride, n, bpk, _ptr(out), cap)
    if r < 0:
        raise RuntimeError(f"orc_legacy_build: {r}")
    return out[:r].tobytes()


def legacy_probe(filt: bytes, keys: np.ndarray, n: int, stride: int = 20, offsets=None) -> np.ndarray:
    a = np.frombuffer(filt + b"\0", dtype=np.uint8)
    out = np.zeros(max(n, 1), dtype=np.uint8)
    lib().orc_legacy_probe(_ptr(a), len(filt), _ptr(keys), _ptr(offsets, u64p), stride, n, _ptr(out))
    return out[:n]


def legacy_key_may_match(filt: bytes, key: bytes) -> int:
    a = np.frombuffer(filt + b"\0", dtype=np.uint8)
    k = np.frombuffer(key + b"\0", dtype=np.uint8)
    return int(lib().orc_legacy_key_may_match(_ptr(a), len(filt), _ptr(k), len(key)))


def fnv1a64(data) -> int:
    a = np.frombuffer(bytes(data) + b"\0", dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    n = len(data) if not isinstance(data, np.ndarray) else data.size
    return int(lib().orc_fnv1a64(_ptr(np.ascontiguousarray(a, dtype=np.uint8)), n))


def crc32c(data: bytes, init: int = 0) -> int:
    a = np.frombuffer(data + b"\0", dtype=np.uint8)
    return int(lib().orc_crc32c_extend(init, _ptr(a), len(data)))


def crc32c_mask(crc: int) -> int:
    return int(lib().orc_crc32c_mask(crc))


def filter_block(filt: bytes) -> bytes:
    """The bytes FlushFilter RDMA-writes: filter + [type 0] + Fixed32(Mask(crc32c(filter||type)))
    (table/table_builder_computeside.cc:418-428)."""
    crc = crc32c(b"\0", crc32c(filt))
    m = crc32c_mask(crc)
    return filt + b"\0" + m.to_bytes(4, "little")


def full_build_many(tables: list[np.ndarray], ns: list[int], stride: int, bpk: int,
                    nthreads: int):
    """CPU baseline: build len(tables) full filters on `nthreads` threads."""
    T = len(tables)
    caps = np.array([full_filter_bytes(n, bpk)[0] for n in ns], dtype=np.uint64)
    outs = [np.zeros(int(c), dtype=np.uint8) for c in caps]
    kp = (u8p * T)(*[_ptr(t) for t in tables])
    op = (u8p * T)(*[_ptr(o) for o in outs])
    nn = np.array(ns, dtype=np.uint64)
    lens = (C.c_int64 * T)()
    lib().orc_full_build_many(kp, _ptr(nn, u64p), stride, T, bpk, op, _ptr(caps, u64p), lens,
                              nthreads)
    return [o[: lens[i]].tobytes() for i, o in enumerate(outs)]
