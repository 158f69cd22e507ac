"""dlsm_amd -- MI355X-native SSTable Bloom-filter engine for dLSM.

Python face of the C ABI (``include/dlsm_bloom.h``).  The compute path is the
hand-written gfx950 HIP library ``dlsm_amd/lib/libdlsm_bloom.so``; this package
only marshals buffers (numpy arrays for host memory, torch tensors for device
memory) and mirrors the reference's class surface:

* :class:`FullFilterBlockBuilder` / :class:`FullFilterBlockReader`
  (table/full_filter_block.h:33-94)
* :class:`BloomFilterPolicy` (include/TimberSaw/filter_policy.h:31-71,
  util/bloom.cc)

There is no CPU fallback: without the HIP library every call raises.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib as _L
from ._lib import DlsmError, check, dlsm_build_job, dlsm_keyset

__all__ = [
    "Keys", "Context", "FilterSet", "DlsmError", "device_available", "bloom_hash",
    "full_size", "legacy_size", "full_parse", "FullFilterBlockBuilder",
    "FullFilterBlockReader", "BloomFilterPolicy", "PATH_AUTO", "PATH_DIRECT", "PATH_SLICED",
    "crc32c", "crc32c_mask", "Version", "VersionFile",
]

PATH_AUTO, PATH_DIRECT, PATH_SLICED = 0, 1, 2
INTERNAL_KEY_TRAILER = 8  # dlsm_keyset.suffix_len for internal keys (db/dbformat.h:374-377)
SELECT_FLUSH, SELECT_COMPACTION = 0, 1  # dlsm_internal_keys_select_dev policies
OPT_PATH, OPT_PROBE_ROUND_KEYS, OPT_BUILD_GROUPS = 0, 1, 2  # dlsm_ctx_set_option
OPT_PROBE_CHUNK_LG, OPT_PROBE_SLICE_LG, OPT_BUILD_EXACT, OPT_PROBE_ROUND_SERIAL = 3, 4, 5, 6
OPT_FAULT_INJECT = 7  # test hook: builds / probes on the context return -value
OPT_VERSION_SLICE_BYTES, OPT_VERSION_PASS_SLICES = 8, 9  # sliced version probe: level threshold, slices per pass
OPT_PROBE_MULTI = 10  # multi-group filter sets: 1 one pass over every group (default), 0 a pass per group


def lib():
    return _L._lib()


def device_available() -> bool:
    n = C.c_int(0)
    try:
        lib().dlsm_device_count(C.byref(n))
    except OSError:
        return False
    return n.value > 0


def bloom_hash(key: bytes) -> int:
    """BloomHash (include/TimberSaw/filter_policy.h:26-28), host side."""
    b = C.create_string_buffer(bytes(key), len(key) + 1)
    return int(lib().dlsm_bloom_hash(b, len(key)))


class PinnedArray:
    """A page-locked host uint8 array (dlsm_host_alloc), freed on close()."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        check(lib().dlsm_host_alloc(nbytes, C.byref(p)), "host_alloc")
        self.ptr = p.value
        self.array = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(self.ptr))

    def close(self):
        if self.ptr:
            lib().dlsm_host_free(C.c_void_p(self.ptr))
            self.ptr = None
            self.array = None


def full_size(n_dedup: int, bits_per_key: int = 10):
    L = C.c_uint32(0)
    nb = C.c_uint64(0)
    check(lib().dlsm_bloom_full_size(n_dedup, bits_per_key, C.byref(L), C.byref(nb)))
    return int(nb.value), int(L.value)


def legacy_size(n: int, bits_per_key: int = 10) -> int:
    nb = C.c_uint64(0)
    check(lib().dlsm_bloom_legacy_size(n, bits_per_key, C.byref(nb)))
    return int(nb.value)


def full_parse(filt: bytes):
    """(status, num_probes, num_lines, log2_line) -- FullFilterBlockReader ctor."""
    b = C.create_string_buffer(bytes(filt), max(len(filt), 1))
    k, L, lg = C.c_int(0), C.c_uint32(0), C.c_int(0)
    st = lib().dlsm_bloom_full_parse(b, len(filt), C.byref(k), C.byref(L), C.byref(lg))
    return st, k.value, L.value, lg.value


def crc32c(data: bytes, init: int = 0) -> int:
    """crc32c::Extend(init, data) (util/crc32c.h:17-22), host helper."""
    b = C.create_string_buffer(bytes(data), len(data) + 1)
    return int(lib().dlsm_crc32c_extend(init, b, len(data)))


def hash_batch(keys: "Keys", out: Optional[np.ndarray] = None, threads: int = 0) -> np.ndarray:
    """BloomHash of every key of a host key set on the host's cores
    (dlsm_bloom_hash_batch): uint32[n], numpy or a pinned torch CPU tensor's
    storage passed as ``out``."""
    if out is None:
        out = np.empty(max(keys.n, 1), dtype=np.uint32)
    if isinstance(out, np.ndarray):
        ok = out.itemsize == 4 and out.size >= keys.n and out.flags["C_CONTIGUOUS"]
    else:  # a torch CPU tensor
        ok = out.element_size() == 4 and out.numel() >= keys.n and out.is_contiguous() and not out.is_cuda
    if not ok:
        raise ValueError("hash_batch: `out` must be contiguous host memory of >= n 4-byte elements")
    ks = keys.c()
    check(lib().dlsm_bloom_hash_batch(C.byref(ks), _ptr(out), threads), "hash_batch")
    return out[: keys.n] if isinstance(out, np.ndarray) else out


def host_read_bytes(buf, threads: int = 0) -> int:
    """Stream a host buffer (numpy array or CPU torch tensor, size a multiple
    of 8 bytes) on the host-hash pool, NUMA-placed like hash_batch
    (dlsm_host_read_bytes); returns the XOR fold of its 64-bit words."""
    n = buf.nbytes if isinstance(buf, np.ndarray) else buf.numel() * buf.element_size()
    fold = C.c_uint64(0)
    check(lib().dlsm_host_read_bytes(_ptr(buf), n, threads, C.byref(fold)), "host_read_bytes")
    return int(fold.value)


def crc32c_mask(crc: int) -> int:
    return int(lib().dlsm_crc32c_mask(crc))


def _ptr(x) -> Optional[int]:
    """Address of a numpy array or torch tensor (host or device)."""
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    return int(x.data_ptr())


def _nbytes(x) -> int:
    """Bytes of a numpy array or torch tensor (0 for None)."""
    if x is None:
        return 0
    if isinstance(x, np.ndarray):
        return int(x.nbytes)
    return int(x.numel()) * int(x.element_size())


def _need(x, nbytes: int, what: str):
    """The binding's guard: a buffer the library writes or reads through a raw
    pointer must hold at least nbytes (a short device buffer would be written
    past its end by the kernels)."""
    if _nbytes(x) < nbytes:
        raise ValueError(f"{what}: buffer of {_nbytes(x)} bytes, {nbytes} needed")


def cu_subset(per_xcd: int, n_cus: int = 256, n_xcds: int = 8) -> list:
    """per_xcd compute units on each XCD under both CU-mask numberings a
    multi-XCD part may use (bit i on XCD i // (n_cus / n_xcds), or on XCD
    i % n_xcds): i = (n_cus / n_xcds) x + n_xcds j + x, j < per_xcd <= 4."""
    per = n_cus // n_xcds
    if not 1 <= per_xcd <= per // n_xcds:
        raise ValueError(f"per_xcd must be in [1, {per // n_xcds}]")
    return sorted(per * x + n_xcds * j + x for x in range(n_xcds) for j in range(per_xcd))


def cu_mask_stream(device: int, cus, n_cus: int = 256):
    """A torch ExternalStream over a new hipStream_t restricted to the CUs in
    `cus` (dlsm_stream_create_cu_mask).  The stream lives as long as the process."""
    import torch

    words = (C.c_uint32 * ((n_cus + 31) // 32))()
    for i in cus:
        words[i // 32] |= 1 << (i % 32)
    raw = C.c_void_p()
    check(lib().dlsm_stream_create_cu_mask(device, words, len(words), C.byref(raw)), "cu_mask_stream")
    return torch.cuda.ExternalStream(raw.value, device=torch.device("cuda", device))


@dataclass
class Keys:
    """A packed key set: ``data`` (uint8) + ``offsets`` (uint64[n+1]) or fixed ``key_len``.

    ``data``/``offsets`` are numpy arrays (host) or torch tensors (device)."""
    data: object
    n: int
    key_len: int = 20
    offsets: object = None
    suffix_len: int = 0  # INTERNAL_KEY_TRAILER: internal keys, hashed as ExtractUserKey(key)

    def c(self) -> dlsm_keyset:
        if self.offsets is None:
            _need(self.data, self.n * self.key_len, "Keys.data")
        else:
            _need(self.offsets, 8 * (self.n + 1), "Keys.offsets")
            # host offsets: the data must also hold the bytes they index (key
            # n-1 ends at offsets[n]); device offsets are not read back here (a
            # synchronising copy per call), the caller vouches for them
            if isinstance(self.offsets, np.ndarray) and self.n:
                _need(self.data, int(self.offsets[self.n]), "Keys.data")
        return dlsm_keyset(_ptr(self.data), _ptr(self.offsets), self.key_len, self.suffix_len, self.n)

    @staticmethod
    def pack(keys: Sequence[bytes]) -> "Keys":
        offs = np.zeros(len(keys) + 1, dtype=np.uint64)
        if keys:
            offs[1:] = np.cumsum([len(k) for k in keys])
        data = np.frombuffer(b"".join(keys) + b"\0" * 16, dtype=np.uint8).copy()
        return Keys(data, len(keys), 0, offs)


@dataclass
class VersionFile:
    """One SSTable of a version (RemoteMemTableMetaData's smallest / largest /
    number + its full filter).  ``largest_trailer`` = seq << 8 | type of the
    largest internal key; ``filter`` = bytes (host) or a device uint8 tensor,
    or None for a table without a filter."""
    level: int
    number: int
    smallest: bytes
    largest: bytes
    largest_trailer: int
    filter: object = None


class Version:
    """A version's files and filters resident on one device (search order:
    level-0 newest first, then one candidate per level 1..5)."""
    NUM_LEVELS = 6

    def __init__(self, ctx: "Context", files: Sequence[VersionFile], on_device: bool = False):
        n = len(files)
        arr = (_L.dlsm_version_file * max(n, 1))()
        keep = []
        for j, f in enumerate(files):
            sm = np.frombuffer(bytes(f.smallest) + b"\0", dtype=np.uint8)
            lg = np.frombuffer(bytes(f.largest) + b"\0", dtype=np.uint8)
            keep += [sm, lg]
            if f.filter is None:
                fp, fl = None, 0
            elif on_device:
                fp, fl = _ptr(f.filter), int(f.filter.numel())
            else:
                fa = np.frombuffer(bytes(f.filter), dtype=np.uint8)
                keep.append(fa)
                fp, fl = fa.ctypes.data, fa.size
            arr[j] = _L.dlsm_version_file(sm.ctypes.data, len(f.smallest), lg.ctypes.data,
                                          len(f.largest), f.largest_trailer, f.number, f.level, 0,
                                          fp, fl)
        h = C.c_void_p()
        check(lib().dlsm_version_create(ctx.h, arr, n, 1 if on_device else 0, C.byref(h)),
              "version_create")
        self.h = h
        a, b = C.c_int(), C.c_int()
        check(lib().dlsm_version_slots(h, C.byref(a), C.byref(b)), "version_slots")
        self.n_l0, self.n_slots = a.value, b.value

    def close(self):
        if getattr(self, "h", None):
            lib().dlsm_version_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


class FilterSet:
    """F parsed full filters resident on one device (FullFilterBlockReader state)."""

    def __init__(self, ctx: "Context", filters, on_device: bool = False):
        self.ctx = ctx
        F = len(filters)
        if on_device:
            ptrs = [_ptr(f) for f in filters]
            lens = [int(f.numel()) for f in filters]
            self._keep = list(filters)
        else:
            arrs = [np.frombuffer(bytes(f), dtype=np.uint8) for f in filters]
            ptrs = [a.ctypes.data for a in arrs]
            lens = [a.size for a in arrs]
            self._keep = arrs
        self.n_filters = F
        self.lens = lens
        h = C.c_void_p()
        pa = (C.c_void_p * F)(*ptrs)
        la = (C.c_uint64 * F)(*lens)
        check(lib().dlsm_filterset_create(ctx.h, pa, la, F, 1 if on_device else 0, C.byref(h)),
              "filterset_create")
        self.h = h
        self._keep = None

    @property
    def mask_bytes(self) -> int:
        return (self.n_filters + 7) // 8

    def close(self):
        if getattr(self, "h", None):
            lib().dlsm_filterset_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One device + one HIP stream + workspace (``dlsm_ctx``)."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check(lib().dlsm_ctx_create(device, C.byref(h)), "ctx_create")
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            lib().dlsm_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- plumbing -----------------------------------------------------------
    def sync(self):
        check(lib().dlsm_ctx_sync(self.h), "sync")

    def set_path(self, path: int):
        check(lib().dlsm_ctx_set_path(self.h, path), "set_path")

    def set_option(self, option: int, value: int):
        check(lib().dlsm_ctx_set_option(self.h, option, value), "set_option")

    def set_probe_round(self, keys: int):
        """Keys per pipelined probe round (0 = one round)."""
        self.set_option(OPT_PROBE_ROUND_KEYS, keys)

    def set_probe_serial(self, serial: bool):
        """Probe rounds one after another on this context's stream (DLSM_OPT_PROBE_ROUND_SERIAL)."""
        self.set_option(OPT_PROBE_ROUND_SERIAL, 1 if serial else 0)

    def set_build_groups(self, groups: int):
        """Job groups of a pipelined build (0 = auto, 1..4)."""
        self.set_option(OPT_BUILD_GROUPS, groups)

    def set_build_exact(self, mode: int):
        """0 auto, 1 count distinct hashes before bucketing, 2 never (DLSM_OPT_BUILD_EXACT)."""
        self.set_option(OPT_BUILD_EXACT, mode)

    def get_option(self, option: int) -> int:
        v = C.c_uint64()
        check(lib().dlsm_ctx_get_option(self.h, option, C.byref(v)), "get_option")
        return int(v.value)

    def set_probe_shape(self, chunk_lg: int, slice_lg: int):
        """Sliced probe shape: 2^chunk_lg keys per partition chunk (12..14),
        2^slice_lg stacked lines per LDS slice (7 = 64 KiB, 8 = 128 KiB)."""
        self.set_option(OPT_PROBE_CHUNK_LG, chunk_lg)
        self.set_option(OPT_PROBE_SLICE_LG, slice_lg)

    def set_stream(self, stream=None):
        """Run on a torch.cuda.Stream (or its raw handle); None = own stream."""
        raw = None if stream is None else (stream if isinstance(stream, int) else stream.cuda_stream)
        check(lib().dlsm_ctx_set_stream(self.h, raw), "set_stream")

    def set_partition_stream(self, stream=None, cus: int = 0):
        """Partition passes on `stream` (a CU-masked stream: cu_mask_stream),
        slice / unpermute passes on the context stream; None = one stream."""
        raw = None if stream is None else (stream if isinstance(stream, int) else stream.cuda_stream)
        check(lib().dlsm_ctx_set_partition_stream(self.h, raw, cus if raw else 0), "set_partition_stream")

    @property
    def stream_handle(self) -> int:
        return int(lib().dlsm_ctx_stream(self.h) or 0)

    def reserve(self, max_keys: int, max_jobs: int):
        check(lib().dlsm_ctx_reserve(self.h, max_keys, max_jobs), "reserve")

    def stats(self):
        """(device allocations made so far, workspace bytes held)."""
        n, b = C.c_uint64(), C.c_uint64()
        check(lib().dlsm_ctx_stats(self.h, C.byref(n), C.byref(b)), "stats")
        return int(n.value), int(b.value)

    # -- full filter build --------------------------------------------------
    @staticmethod
    def _jobs(tables: Sequence[Keys], outs, caps):
        n = len(tables)
        arr = (dlsm_build_job * max(n, 1))()
        for j, t in enumerate(tables):
            arr[j].keys = t.c()
            arr[j].out = _ptr(outs[j])
            arr[j].out_cap = caps[j]
        return arr

    def full_build(self, tables: Sequence[Keys], bits_per_key: int = 10, caps=None) -> list:
        """Host keys -> host filter bytes (synchronous).  One filter per table."""
        n = len(tables)
        if caps is None:
            caps = [full_size(t.n, bits_per_key)[0] for t in tables]
        outs = [np.zeros(max(c, 1), dtype=np.uint8) for c in caps]
        jobs = self._jobs(tables, outs, caps)
        lens = (C.c_uint64 * max(n, 1))()
        check(lib().dlsm_bloom_full_build(self.h, jobs, n, bits_per_key, lens), "full_build")
        return [outs[j][: lens[j]].tobytes() for j in range(n)]

    def full_build_dev(self, tables: Sequence[Keys], outs, out_lens, bits_per_key: int = 10):
        """Device keys (torch tensors) -> device slots; asynchronous on this ctx's stream."""
        _need(out_lens, 8 * len(tables), "full_build_dev out_lens")
        caps = [int(o.numel()) for o in outs]
        jobs = self._jobs(tables, outs, caps)
        check(lib().dlsm_bloom_full_build_dev(self.h, jobs, len(tables), bits_per_key,
                                              _ptr(out_lens)), "full_build_dev")

    def bind_full_build_dev(self, tables: Sequence[Keys], outs, out_lens, bits_per_key: int = 10):
        """full_build_dev with its arguments marshalled once: returns a
        zero-argument callable (one ctypes call per invocation; the GIL is
        released inside it), for per-step loops on several host threads."""
        _need(out_lens, 8 * len(tables), "bind_full_build_dev out_lens")
        caps = [int(o.numel()) for o in outs]
        jobs = self._jobs(tables, outs, caps)
        fn, h, n, lp = lib().dlsm_bloom_full_build_dev, self.h, len(tables), _ptr(out_lens)
        keep = (jobs, list(tables), list(outs), out_lens)

        def call():
            st = fn(h, jobs, n, bits_per_key, lp)
            if st:
                check(st, "full_build_dev")

        call.keep = keep
        return call

    def full_build_hashed(self, hash_sets, bits_per_key: int = 10, caps=None) -> list:
        """Filters from BloomHash values (numpy uint32 arrays, AddKey order;
        consecutive equal hashes are dropped like AddKey) -- host in/out."""
        sets = [np.ascontiguousarray(h, dtype=np.uint32) for h in hash_sets]
        tables = [Keys(h if h.size else np.zeros(1, dtype=np.uint32), h.size, 4) for h in sets]
        if caps is None:
            caps = [full_size(h.size, bits_per_key)[0] for h in sets]
        outs = [np.zeros(max(c, 1), dtype=np.uint8) for c in caps]
        jobs = self._jobs(tables, outs, caps)
        n = len(tables)
        lens = (C.c_uint64 * max(n, 1))()
        check(lib().dlsm_bloom_full_build_hashed(self.h, jobs, n, bits_per_key, lens), "full_build_hashed")
        return [outs[j][: lens[j]].tobytes() for j in range(n)]

    def full_build_hashed_dev(self, hash_sets, outs, out_lens, bits_per_key: int = 10):
        """Device form: hash_sets are device uint32 tensors."""
        _need(out_lens, 8 * len(hash_sets), "full_build_hashed_dev out_lens")
        tables = [Keys(h, int(h.numel()), 4) for h in hash_sets]
        caps = [int(o.numel()) for o in outs]
        jobs = self._jobs(tables, outs, caps)
        check(lib().dlsm_bloom_full_build_hashed_dev(self.h, jobs, len(tables), bits_per_key, _ptr(out_lens)),
              "full_build_hashed_dev")

    def full_build_block(self, tables: Sequence[Keys], bits_per_key: int = 10, caps=None) -> list:
        """Filter + 5-byte block trailer (FinishFilterBlock), host in/out."""
        n = len(tables)
        if caps is None:
            caps = [full_size(t.n, bits_per_key)[0] + 5 for t in tables]
        outs = [np.zeros(max(c, 1), dtype=np.uint8) for c in caps]
        jobs = self._jobs(tables, outs, caps)
        lens = (C.c_uint64 * max(n, 1))()
        check(lib().dlsm_bloom_full_build_block(self.h, jobs, n, bits_per_key, lens), "full_build_block")
        return [outs[j][: lens[j]].tobytes() for j in range(n)]

    def full_build_block_dev(self, tables: Sequence[Keys], outs, out_lens, bits_per_key: int = 10):
        caps = [int(o.numel()) for o in outs]
        jobs = self._jobs(tables, outs, caps)
        check(lib().dlsm_bloom_full_build_block_dev(self.h, jobs, len(tables), bits_per_key,
                                                    _ptr(out_lens)), "full_build_block_dev")

    def crc32c_dev(self, bufs) -> list:
        """crc32c::Value of device tensors (uint8), computed on the GPU."""
        n = len(bufs)
        ptrs = (C.c_void_p * max(n, 1))(*[_ptr(b) for b in bufs])
        lens = (C.c_uint64 * max(n, 1))(*[int(b.numel()) for b in bufs])
        out = (C.c_uint32 * max(n, 1))()
        check(lib().dlsm_crc32c_dev(self.h, ptrs, lens, n, out), "crc32c_dev")
        return [int(out[j]) for j in range(n)]

    # -- internal keys: flush / compaction selection, user-key gather --------
    def internal_keys_select_dev(self, keys: Keys, policy: int, smallest_snapshot: int, keep):
        """keep (device uint8[n]) <- 1 for every key the flush / compaction loop
        passes to TableBuilder::Add.  Returns (n_kept, kept_user_key_bytes,
        first_corrupt or None).  A flush over a corrupt key raises DlsmError
        (DLSM_E_CORRUPT) like the reference's IOError."""
        ks = keys.c()
        nk, nb, bad = C.c_uint64(), C.c_uint64(), C.c_uint64()
        st = lib().dlsm_internal_keys_select_dev(self.h, C.byref(ks), policy, smallest_snapshot,
                                                 _ptr(keep), C.byref(nk), C.byref(nb), C.byref(bad))
        check(st, "internal_keys_select_dev")
        return int(nk.value), int(nb.value), (None if bad.value == 2**64 - 1 else int(bad.value))

    def user_keys_gather_dev(self, keys: Keys, keep, out, offsets=None):
        """Pack ExtractUserKey(key) of the kept keys into `out` (device uint8);
        variable-length keys also fill `offsets` (device uint64[n_kept+1])."""
        ks = keys.c()
        check(lib().dlsm_user_keys_gather_dev(self.h, C.byref(ks), _ptr(keep), _ptr(out), _ptr(offsets)),
              "user_keys_gather_dev")

    # -- legacy block-based filter block (table/filter_block.cc) -------------
    def filter_block_build_dev(self, keys: Keys, block_key_end, block_end_offset,
                               bits_per_key: int = 10, out=None):
        """FilterBlockBuilder over a table's keys (data block b ends at key
        block_key_end[b], then StartBlock(block_end_offset[b])).  Returns the
        block as a device uint8 tensor (or fills `out` and returns its length)."""
        import torch

        ke = np.ascontiguousarray(block_key_end, dtype=np.uint64)
        eo = np.ascontiguousarray(block_end_offset, dtype=np.uint64)
        nb = C.c_uint64()
        check(lib().dlsm_filter_block_size(_ptr(ke), _ptr(eo), len(ke), keys.n,
                                           bits_per_key, C.byref(nb)), "filter_block_size")
        ret = out is None
        if out is None:
            out = torch.empty(nb.value, dtype=torch.uint8, device=f"cuda:{self.device}")
        ln = C.c_uint64()
        ks = keys.c()
        check(lib().dlsm_filter_block_build_dev(self.h, C.byref(ks), _ptr(ke), _ptr(eo),
                                                len(ke), bits_per_key, _ptr(out), int(out.numel()),
                                                C.byref(ln)), "filter_block_build_dev")
        return out[: ln.value] if ret else ln.value

    def filter_block_probe_dev(self, block, keys: Keys, block_offsets, out):
        """FilterBlockReader::KeyMayMatch(block_offsets[i], key i) -> out[i] (device)."""
        ks = keys.c()
        check(lib().dlsm_filter_block_probe_dev(self.h, _ptr(block), int(block.numel()), C.byref(ks),
                                                _ptr(block_offsets), _ptr(out)), "filter_block_probe_dev")

    # -- MultiGet-style probe of a version -------------------------------------
    def version(self, files: Sequence[VersionFile], on_device: bool = False) -> Version:
        return Version(self, files, on_device)

    def version_probe_dev(self, v: Version, keys: Keys, snapshot: int, slot_mask, level_file=None):
        """slot_mask (device uint64[n]): bit s = search slot s is a file Version::Get
        visits and whose filter passes the key; level_file (device int32/uint32
        [n, 5], optional): per level the candidate file's index in the level."""
        ks = keys.c()
        check(lib().dlsm_version_probe_dev(self.h, v.h, C.byref(ks), snapshot, _ptr(slot_mask),
                                           _ptr(level_file)), "version_probe_dev")

    # -- full filter probe --------------------------------------------------
    def filterset(self, filters, on_device: bool = False) -> FilterSet:
        return FilterSet(self, filters, on_device)

    def full_probe(self, fs: FilterSet, keys: Keys) -> np.ndarray:
        mask = np.zeros(max(keys.n * fs.mask_bytes, 1), dtype=np.uint8)
        ks = keys.c()
        check(lib().dlsm_bloom_full_probe(self.h, fs.h, C.byref(ks), mask.ctypes.data), "full_probe")
        return mask[: keys.n * fs.mask_bytes]

    def full_probe_hashed_dev(self, fs: FilterSet, hashes, mask, n: Optional[int] = None):
        """Probe from BloomHash values (device uint32 tensor); asynchronous."""
        n = int(hashes.numel()) if n is None else n
        _need(mask, n * fs.mask_bytes, "full_probe_hashed_dev mask")
        ks = Keys(hashes, n, 4).c()
        check(lib().dlsm_bloom_full_probe_hashed_dev(self.h, fs.h, C.byref(ks), _ptr(mask)),
              "full_probe_hashed_dev")

    def full_probe_dev(self, fs: FilterSet, keys: Keys, mask):
        _need(mask, keys.n * fs.mask_bytes, "full_probe_dev mask")
        ks = keys.c()
        check(lib().dlsm_bloom_full_probe_dev(self.h, fs.h, C.byref(ks), _ptr(mask)),
              "full_probe_dev")

    def bind_full_probe_dev(self, fs: FilterSet, keys: Keys, mask):
        """full_probe_dev with its arguments marshalled once (see bind_full_build_dev)."""
        _need(mask, keys.n * fs.mask_bytes, "bind_full_probe_dev mask")
        ks = keys.c()
        fn, h, fh, kp, mp = lib().dlsm_bloom_full_probe_dev, self.h, fs.h, C.byref(ks), _ptr(mask)
        keep = (ks, fs, keys, mask)

        def call():
            st = fn(h, fh, kp, mp)
            if st:
                check(st, "full_probe_dev")

        call.keep = keep
        return call

    # -- legacy FilterPolicy format -----------------------------------------
    def legacy_build(self, tables: Sequence[Keys], bits_per_key: int = 10) -> list:
        n = len(tables)
        caps = [legacy_size(t.n, bits_per_key) for t in tables]
        outs = [np.zeros(c, dtype=np.uint8) for c in caps]
        jobs = self._jobs(tables, outs, caps)
        lens = (C.c_uint64 * max(n, 1))()
        check(lib().dlsm_bloom_legacy_build(self.h, jobs, n, bits_per_key, lens), "legacy_build")
        return [outs[j][: lens[j]].tobytes() for j in range(n)]

    def legacy_build_dev(self, tables: Sequence[Keys], outs, out_lens, bits_per_key: int = 10):
        _need(out_lens, 8 * len(tables), "legacy_build_dev out_lens")
        caps = [int(o.numel()) for o in outs]
        jobs = self._jobs(tables, outs, caps)
        check(lib().dlsm_bloom_legacy_build_dev(self.h, jobs, len(tables), bits_per_key,
                                                _ptr(out_lens)), "legacy_build_dev")

    def legacy_probe(self, filt: bytes, keys: Keys) -> np.ndarray:
        fa = np.frombuffer(bytes(filt) + b"\0", dtype=np.uint8)
        out = np.zeros(max(keys.n, 1), dtype=np.uint8)
        ks = keys.c()
        check(lib().dlsm_bloom_legacy_probe(self.h, fa.ctypes.data if len(filt) else None, len(filt),
                                            C.byref(ks), out.ctypes.data), "legacy_probe")
        return out[: keys.n]

    def legacy_probe_dev(self, filt_dev, length: int, keys: Keys, out):
        _need(filt_dev, length, "legacy_probe_dev filter")
        _need(out, keys.n, "legacy_probe_dev out")
        ks = keys.c()
        check(lib().dlsm_bloom_legacy_probe_dev(self.h, _ptr(filt_dev), length, C.byref(ks),
                                                _ptr(out)), "legacy_probe_dev")


from .filter_block import BloomFilterPolicy, FullFilterBlockBuilder, FullFilterBlockReader  # noqa: E402
