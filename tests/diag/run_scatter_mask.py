"""Scattered final-mask stores vs bucket-order answer stores (diagnostic for
VERDICT r2 "next" 2b, run by hand on a GPU box; output under profiles/).

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared \
        tests/diag/scatter_mask.hip -o tests/diag/libscatter_mask.so
    python tests/diag/run_scatter_mask.py [--keys 100000000]

Builds the probe's bucket layout for `keys` lookups (8,192-key chunks, 123
slices of a 31,251-line filter set, buckets padded to 16-byte units), then
times the slice-pass walk storing (a) each key's byte at its own position in
its chunk (the cut that would drop the position array and the unpermute pass)
and (b) 4 answers per lane as one dword in bucket order (today).  Prints one
JSON line.
"""
import argparse
import ctypes
import json
import os
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def layout(keys, C, S, seed=1):
    """run_off[nC][S+1] (16-byte units) and idx[nC][CR] (in-chunk key index
    in bucket order, 0xffff = padding), slices uniform at random."""
    nC = (keys + C - 1) // C
    CR = C + 4 * 256
    rng = np.random.default_rng(seed)
    run_off = np.zeros((nC, S + 1), dtype=np.uint32)
    idx = np.full((nC, CR), 0xFFFF, dtype=np.uint16)
    step = 512  # chunks per batch (bounded host memory)
    for c0 in range(0, nC, step):
        c1 = min(nC, c0 + step)
        n = c1 - c0
        sl = rng.integers(0, S, size=(n, C), dtype=np.int32)
        valid = (np.arange(C)[None, :] + (np.arange(c0, c1) * C)[:, None]) < keys
        sl = np.where(valid, sl, S)  # past the last key: a bucket that is never walked
        order = np.argsort(sl, axis=1, kind="stable")
        ssort = np.take_along_axis(sl, order, axis=1)
        cnt = np.zeros((n, S + 1), dtype=np.int64)
        np.add.at(cnt, (np.repeat(np.arange(n), C), sl.ravel()), 1)
        padded = (cnt[:, :S] + 3) // 4 * 4
        start_u = np.zeros((n, S + 1), dtype=np.int64)
        start_u[:, 1:] = np.cumsum(padded, axis=1) // 4
        run_off[c0:c1] = start_u
        unp = np.zeros((n, S + 1), dtype=np.int64)
        unp[:, 1:] = np.cumsum(cnt[:, :S], axis=1)
        j = np.arange(C)[None, :]
        s_of = np.minimum(ssort, S - 1)
        rank = j - np.take_along_axis(unp, s_of, axis=1)
        dest = np.take_along_axis(start_u * 4, s_of, axis=1) + rank
        ok = ssort < S
        rows = np.repeat(np.arange(n), C).reshape(n, C)
        idx[c0:c1][rows[ok], dest[ok]] = order[ok].astype(np.uint16)
        if c0 % (step * 8) == 0:
            print(f"layout: chunk {c0} of {nC}", flush=True)
    return run_off, idx, nC, CR


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch

    C, S, parts = 8192, 123, 2
    t0 = time.time()
    run_off, idx, nC, CR = layout(args.keys, C, S)
    print(f"layout in {time.time() - t0:.1f}s", flush=True)
    lib = ctypes.CDLL(os.path.join(HERE, "libscatter_mask.so"))
    lib.scatter_mask_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_int]
    d_ro = torch.from_numpy(run_off.view(np.int32)).cuda()
    d_ix = torch.from_numpy(idx.view(np.int16)).cuda()
    out_s = torch.zeros(nC * C, dtype=torch.uint8, device="cuda")
    out_c = torch.zeros(nC * CR, dtype=torch.uint8, device="cuda")
    res = {"keys": args.keys, "chunk": C, "slices": S, "parts": parts}
    for name, sc, out in (("bucket_order_dword_stores", 0, out_c), ("scattered_byte_stores", 1, out_s)):
        call = lambda: lib.scatter_mask_launch(sc, d_ro.data_ptr(), d_ix.data_ptr(), out.data_ptr(),  # noqa: E731
                                               S, nC, C, CR, parts)
        for _ in range(2):
            assert call() == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        res[name + "_us"] = round(e0.elapsed_time(e1) / args.reps * 1e3, 1)
    # every key's byte written exactly once by the scattered walk
    nz = int(torch.count_nonzero(out_s[: args.keys]).item())
    res["scattered_bytes_written_nonzero"] = nz
    res["delta_us"] = round(res["scattered_byte_stores_us"] - res["bucket_order_dword_stores_us"], 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
