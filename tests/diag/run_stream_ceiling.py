"""HBM streaming ceilings of the box (diagnostic, run by hand on a GPU box;
output recorded under profiles/): read-only, copy, and the probe partition's
byte shape (20 B read, 4 + 2 B written per key) at several grid sizes.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared \
        tests/diag/stream_ceiling.hip -o tests/diag/libstream_ceiling.so
    python tests/diag/run_stream_ceiling.py
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    import torch

    lib = ctypes.CDLL(os.path.join(HERE, "libstream_ceiling.so"))
    lib.stream_ceiling_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
    keys = 100_000_000
    nbytes = keys * 20  # the probe's 100 M 20-byte keys
    src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    src.random_(0, 256)
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    ent = torch.empty(keys * 4, dtype=torch.uint8, device="cuda")
    pos = torch.empty(keys * 2, dtype=torch.uint8, device="cuda")
    sink = torch.empty(4096 * 512, dtype=torch.int32, device="cuda")
    out = {"bytes_in": nbytes, "runs": []}
    reps = 10
    for kind, name in ((0, "read"), (1, "copy"), (2, "partition shape")):
        for blocks in (512, 1024, 2048, 4096):
            for unroll in ((4, 8) if kind < 2 else (1, 2)):
                args = {0: (src.data_ptr(), sink.data_ptr(), 0),
                        1: (src.data_ptr(), dst.data_ptr(), 0),
                        2: (src.data_ptr(), ent.data_ptr(), pos.data_ptr())}[kind]
                for _ in range(2):
                    lib.stream_ceiling_launch(kind, *args, nbytes, blocks, unroll)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(reps):
                    rc = lib.stream_ceiling_launch(kind, *args, nbytes, blocks, unroll)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
                moved = {0: nbytes, 1: 2 * nbytes, 2: nbytes + keys * 6}[kind]
                r = {"kind": name, "blocks": blocks, "threads": 512, "unroll": unroll, "rc": rc,
                     "us": round(ms * 1e3, 1), "TBs": round(moved / (ms * 1e-3) / 1e12, 3)}
                out["runs"].append(r)
                print(json.dumps(r), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
