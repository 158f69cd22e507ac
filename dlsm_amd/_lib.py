"""ctypes binding of the C ABI in include/dlsm_bloom.h.

Loads the in-tree gfx950 library ``dlsm_amd/lib/libdlsm_bloom.so`` (built by
``make`` / ``__graft_entry__.build()``).  There is no fallback: if the library is
missing, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libdlsm_bloom.so")
# A/B tuning only: $DLSM_LIB_VARIANT=<tag> loads the in-tree build
# dlsm_amd/lib/variants/libdlsm_bloom_<tag>.so (``make variant``) instead.
if os.environ.get("DLSM_LIB_VARIANT"):
    LIB_PATH = os.path.join(_HERE, "lib", "variants",
                            f"libdlsm_bloom_{os.environ['DLSM_LIB_VARIANT']}.so")

DLSM_OK = 0
DLSM_E_ARG = -1
DLSM_E_CAPACITY = -2
DLSM_E_CORRUPT = -3
DLSM_E_DEVICE = -4
DLSM_E_NOMEM = -5
DLSM_E_BUSY = -6


class dlsm_keyset(C.Structure):
    _fields_ = [("bytes", C.c_void_p), ("offsets", C.c_void_p), ("key_len", C.c_uint32),
                ("suffix_len", C.c_uint32), ("n", C.c_uint64)]


class dlsm_build_job(C.Structure):
    _fields_ = [("keys", dlsm_keyset), ("out", C.c_void_p), ("out_cap", C.c_uint64)]


class dlsm_device_work(C.Structure):
    _fields_ = [("probe_ctx", C.c_void_p), ("build_ctx", C.c_void_p), ("jobs", C.c_void_p),
                ("n_jobs", C.c_int), ("out_len_dev", C.c_void_p), ("fs", C.c_void_p),
                ("keys", dlsm_keyset), ("mask_dev", C.c_void_p)]


class dlsm_version_file(C.Structure):
    _fields_ = [("smallest_user_key", C.c_void_p), ("smallest_len", C.c_uint64),
                ("largest_user_key", C.c_void_p), ("largest_len", C.c_uint64),
                ("largest_trailer", C.c_uint64), ("number", C.c_uint64),
                ("level", C.c_int32), ("reserved", C.c_int32),
                ("filter", C.c_void_p), ("filter_len", C.c_uint64)]


class DlsmError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        msg = _lib().dlsm_strerror(status).decode() if _LIB is not None else str(status)
        super().__init__(f"{what}: {msg} ({status})" if what else f"{msg} ({status})")


# Exported symbols and their signatures: (name, restype, argtypes).
_VP = C.c_void_p
_U64P = C.POINTER(C.c_uint64)
SIGNATURES = [
    ("dlsm_strerror", C.c_char_p, [C.c_int]),
    ("dlsm_abi_version", C.c_int, []),
    ("dlsm_bloom_hash", C.c_uint32, [_VP, C.c_size_t]),
    ("dlsm_bloom_full_num_probes", C.c_int, [C.c_int]),
    ("dlsm_bloom_full_size", C.c_int, [C.c_uint64, C.c_int, C.POINTER(C.c_uint32), _U64P]),
    ("dlsm_bloom_legacy_size", C.c_int, [C.c_uint64, C.c_int, _U64P]),
    ("dlsm_bloom_full_parse", C.c_int, [_VP, C.c_uint64, C.POINTER(C.c_int),
                                        C.POINTER(C.c_uint32), C.POINTER(C.c_int)]),
    ("dlsm_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("dlsm_ctx_create", C.c_int, [C.c_int, C.POINTER(_VP)]),
    ("dlsm_ctx_destroy", C.c_int, [_VP]),
    ("dlsm_thread_ctx", C.c_int, [C.POINTER(_VP)]),
    ("dlsm_thread_ctx_bind", C.c_int, [_VP]),
    ("dlsm_thread_ctx_stats", C.c_int, [_U64P, _U64P, _U64P]),
    ("dlsm_fallback_note", None, [_VP]),
    ("dlsm_fallback_stats", C.c_int, [_VP, _U64P, _U64P]),
    ("dlsm_ctx_set_stream", C.c_int, [_VP, _VP]),
    ("dlsm_ctx_stream", _VP, [_VP]),
    ("dlsm_ctx_sync", C.c_int, [_VP]),
    ("dlsm_ctx_set_partition_stream", C.c_int, [_VP, _VP, C.c_uint32]),
    ("dlsm_stream_create_cu_mask", C.c_int, [C.c_int, C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(_VP)]),
    ("dlsm_stream_destroy", C.c_int, [_VP]),
    ("dlsm_ctx_reserve", C.c_int, [_VP, C.c_uint64, C.c_uint32]),
    ("dlsm_ctx_stats", C.c_int, [_VP, _U64P, _U64P]),
    ("dlsm_ctx_set_path", C.c_int, [_VP, C.c_int]),
    ("dlsm_ctx_set_option", C.c_int, [_VP, C.c_int, C.c_uint64]),
    ("dlsm_ctx_get_option", C.c_int, [_VP, C.c_int, _U64P]),
    ("dlsm_host_register", C.c_int, [_VP, C.c_size_t]),
    ("dlsm_host_unregister", C.c_int, [_VP]),
    ("dlsm_host_alloc", C.c_int, [C.c_size_t, C.POINTER(_VP)]),
    ("dlsm_host_free", C.c_int, [_VP]),
    ("dlsm_host_pool_acquire", C.c_int, [C.c_uint64, C.POINTER(_VP), _U64P]),
    ("dlsm_host_pool_release", C.c_int, [_VP]),
    ("dlsm_host_pool_trim", C.c_int, []),
    ("dlsm_ctx_host_buffer_claim", C.c_int, [_VP, _VP]),
    ("dlsm_ctx_host_buffer_release", C.c_int, [_VP, _VP]),
    ("dlsm_ctx_host_buffer", C.c_int, [_VP, C.c_uint64, C.c_uint64, C.POINTER(_VP), _U64P]),
    ("dlsm_bloom_full_build_dev", C.c_int, [_VP, C.POINTER(dlsm_build_job), C.c_int, C.c_int, _VP]),
    ("dlsm_bloom_full_build", C.c_int, [_VP, C.POINTER(dlsm_build_job), C.c_int, C.c_int, _U64P]),
    ("dlsm_bloom_full_build_block_dev", C.c_int, [_VP, C.POINTER(dlsm_build_job), C.c_int, C.c_int, _VP]),
    ("dlsm_bloom_full_build_block", C.c_int, [_VP, C.POINTER(dlsm_build_job), C.c_int, C.c_int, _U64P]),
    ("dlsm_crc32c_dev", C.c_int, [_VP, C.POINTER(_VP), _U64P, C.c_int, C.POINTER(C.c_uint32)]),
    ("dlsm_crc32c_extend", C.c_uint32, [C.c_uint32, _VP, C.c_size_t]),
    ("dlsm_crc32c_mask", C.c_uint32, [C.c_uint32]),
    ("dlsm_filterset_create", C.c_int, [_VP, C.POINTER(_VP), _U64P, C.c_int, C.c_int,
                                        C.POINTER(_VP)]),
    ("dlsm_filterset_destroy", C.c_int, [_VP]),
    ("dlsm_filterset_size", C.c_int, [_VP, C.POINTER(C.c_int), _U64P]),
    ("dlsm_bloom_full_probe_dev", C.c_int, [_VP, _VP, C.POINTER(dlsm_keyset), _VP]),
    ("dlsm_internal_keys_select_dev", C.c_int, [_VP, C.POINTER(dlsm_keyset), C.c_int, C.c_uint64,
                                                _VP, _U64P, _U64P, _U64P]),
    ("dlsm_user_keys_gather_dev", C.c_int, [_VP, C.POINTER(dlsm_keyset), _VP, _VP, _VP]),
    ("dlsm_filter_block_size", C.c_int, [_VP, _VP, C.c_int, C.c_uint64, C.c_int, _U64P]),
    ("dlsm_filter_block_build_dev", C.c_int, [_VP, C.POINTER(dlsm_keyset), _VP, _VP, C.c_int,
                                              C.c_int, _VP, C.c_uint64, _U64P]),
    ("dlsm_filter_block_probe_dev", C.c_int, [_VP, _VP, C.c_uint64, C.POINTER(dlsm_keyset), _VP, _VP]),
    ("dlsm_filter_block_build", C.c_int, [_VP, C.POINTER(dlsm_keyset), _VP, _VP, C.c_int, C.c_int,
                                          _VP, C.c_uint64, _U64P]),
    ("dlsm_filter_block_probe", C.c_int, [_VP, _VP, C.c_uint64, C.POINTER(dlsm_keyset), _VP, _VP]),
    ("dlsm_version_create", C.c_int, [_VP, C.POINTER(dlsm_version_file), C.c_int, C.c_int,
                                      C.POINTER(_VP)]),
    ("dlsm_version_destroy", C.c_int, [_VP]),
    ("dlsm_version_slots", C.c_int, [_VP, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("dlsm_version_probe_dev", C.c_int, [_VP, _VP, C.POINTER(dlsm_keyset), C.c_uint64, _VP, _VP]),
    ("dlsm_bloom_full_probe", C.c_int, [_VP, _VP, C.POINTER(dlsm_keyset), _VP]),
    ("dlsm_bloom_full_probe_hashed_dev", C.c_int, [_VP, _VP, C.POINTER(dlsm_keyset), _VP]),
    ("dlsm_bloom_hash_batch", C.c_int, [C.POINTER(dlsm_keyset), _VP, C.c_int]),
    ("dlsm_host_read_bytes", C.c_int, [_VP, C.c_uint64, C.c_int, C.POINTER(C.c_uint64)]),
    ("dlsm_bloom_legacy_build_dev", C.c_int, [_VP, C.POINTER(dlsm_build_job), C.c_int, C.c_int, _VP]),
    ("dlsm_bloom_legacy_build", C.c_int, [_VP, C.POINTER(dlsm_build_job), C.c_int, C.c_int, _U64P]),
    ("dlsm_bloom_legacy_probe_dev", C.c_int, [_VP, _VP, C.c_uint64, C.POINTER(dlsm_keyset), _VP]),
    ("dlsm_bloom_legacy_probe", C.c_int, [_VP, _VP, C.c_uint64, C.POINTER(dlsm_keyset), _VP]),
    ("dlsm_bloom_full_build_hashed_dev", C.c_int, [_VP, C.POINTER(dlsm_build_job), C.c_int, C.c_int, _VP]),
    ("dlsm_bloom_full_build_hashed", C.c_int, [_VP, C.POINTER(dlsm_build_job), C.c_int, C.c_int, _U64P]),
    ("dlsm_stream_kernel", C.c_int, [_VP, C.c_int, C.c_int, _VP, _VP, C.c_uint64, C.c_uint32]),
    ("dlsm_ctx_device", C.c_int, [_VP]),
    ("dlsm_batcher_create", C.c_int, [C.c_int, C.c_int, C.c_uint32, C.c_uint32, C.POINTER(_VP)]),
    ("dlsm_batcher_destroy", C.c_int, [_VP]),
    ("dlsm_batcher_full_build", C.c_int, [_VP, C.POINTER(dlsm_build_job), C.c_int, _U64P]),
    ("dlsm_batcher_full_build_hashed", C.c_int, [_VP, C.POINTER(dlsm_build_job), C.c_int, _U64P]),
    ("dlsm_batcher_submit", C.c_int, [_VP, C.POINTER(dlsm_build_job), C.c_int, C.c_int, _U64P]),
    ("dlsm_batcher_stats", C.c_int, [_VP, _U64P, _U64P, _U64P]),
    ("dlsm_multi_device_run", C.c_int, [C.POINTER(dlsm_device_work), C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.POINTER(C.c_double), C.POINTER(C.c_float)]),
    ("dlsm_multi_device_run_sampled", C.c_int, [C.POINTER(dlsm_device_work), C.c_int, C.c_int, C.c_int, C.c_int,
                                               C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_float)]),
    ("dlsm_multi_device_run_timed", C.c_int, [C.POINTER(dlsm_device_work), C.c_int, C.c_int, C.c_int, C.c_int,
                                             C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_float),
                                             C.POINTER(C.c_double)]),
]

_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        # One HIP runtime per process: torch ships its own libamdhip64 (soname
        # libamdhip64.so.7, but its users NEED the unversioned name).  Loading
        # torch first makes our NEEDED libamdhip64.so.7 bind to that same copy;
        # loading ours first would put two runtimes in the process and torch
        # then sees no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"dlsm_amd: HIP library not built ({LIB_PATH} missing); run `make` or "
                "__graft_entry__.build() -- there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def check(status: int, what: str = "") -> int:
    if status != DLSM_OK:
        raise DlsmError(status, what)
    return status
