"""Every shape of the library's streaming kernels (dlsm_stream_kernel) on this
box: read-only, copy and the probe partition's byte shape (20 B in, 6 B out
per key), each plain / non-temporal x grid-stride / one contiguous range per
workgroup x 512..4096 workgroups of 512 threads.  Diagnostic, run by hand on
a GPU box; prints one JSON line (recorded under profiles/).

    python tests/diag/run_stream_variants.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch

    import dlsm_amd

    fn = dlsm_amd.lib().dlsm_stream_kernel
    nbytes = 2_000_000_000  # the probe's 100 M 20-byte keys
    src = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    raw = ctypes.c_void_p(s.cuda_stream)
    rows = []
    for kind, name, factor in ((0, "read", 1.0), (1, "copy", 2.0), (2, "partition shape", 1.3)):
        for variant in range(4):
            for blocks in (512, 1024, 2048, 4096):
                args = (raw, kind, variant, ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                        ctypes.c_uint64(nbytes), ctypes.c_uint32(blocks))
                assert fn(*args) == 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(5):
                    fn(*args)
                e1.record(s)
                s.synchronize()
                ms = e0.elapsed_time(e1) / 5
                rows.append({"kind": name, "nt": bool(variant & 1), "chunked": bool(variant & 2), "blocks": blocks,
                             "us": round(ms * 1e3, 1), "TBs": round(nbytes * factor / (ms * 1e-3) / 1e12, 3)})
                print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"bytes_read": nbytes, "runs": rows}))


if __name__ == "__main__":
    main()
