"""Reproduce the sliced-probe corruption fixed by commit 1c7c4c6 in isolation
(diagnostic, run by hand on a GPU box; output recorded under profiles/).

Runs the pre-fix probe slice kernel (tests/diag/old_probe_slice.hip, the
kernel exactly as it stood) on synthetic 4,096-key chunk buckets against a
random stacked image, in several builds (launch bound, windows per lane, LDS
per workgroup: see old_slice_launch) and compares every answer byte with numpy.
Mismatches are reported per wave of the 1,024-thread workgroup (wave w walks
64-chunk groups w, w + 16, ... of its part).  Buffers carry >4 GiB of slack
past the chunk regions so that even a wrapped 32-bit offset stays in bounds.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared \
        tests/diag/old_probe_slice.hip -o tests/diag/libold_slice.so
    python tests/diag/run_old_slice.py
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
CHUNK = 4096
L = 31_251  # the bench filter's line count (1.6 M keys, 10 bits/key)
S = (L + 127) // 128
NC = 2048
PARTS = min(max(1, (512 + S // 2) // S), max(1, NC // 1024))  # the pre-fix launch
SLACK = (1 << 32) + 64 * CHUNK + (1 << 20)


def expected_answers(x, stacked):
    line = (x % L).astype(np.int64)
    delta = ((x >> np.uint32(17)) | (x << np.uint32(15))).astype(np.uint32)
    acc = np.full(x.size, 0xFF, dtype=np.uint8)
    h = x.copy()
    img = stacked.reshape(-1, 64, 8)  # [line][word][filter]
    for _ in range(6):
        bp = (h & np.uint32(511)).astype(np.int64)
        byte = img[line, bp >> 3]  # [n, 8]: filter f's byte of the line
        bit = (byte >> (bp & 7)[:, None].astype(np.uint8)) & np.uint8(1)
        acc &= np.bitwise_or.reduce(bit << np.arange(8, dtype=np.uint8)[None, :], axis=1).astype(np.uint8)
        h = (h + delta).astype(np.uint32)
    # the kernel packs byte f's bit 0 with (acc * 0x0102040810204080) >> 56:
    # filter f lands in bit f
    return acc


def main():
    import torch

    rng = np.random.default_rng(20261016)
    n = NC * CHUNK
    x = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    sl = ((x % L) >> 7).astype(np.int64)
    chunk = np.arange(n, dtype=np.int64) // CHUNK
    order = np.lexsort((sl, chunk))  # stable: by chunk, then slice
    ent = x[order]
    slc = sl[order].reshape(NC, CHUNK)
    tab = np.zeros((NC, S + 1), dtype=np.uint16)
    for c in range(NC):
        tab[c] = np.searchsorted(slc[c], np.arange(S + 1), side="left")
    stacked = rng.integers(0, 256, size=S * 128 * 512, dtype=np.uint8)
    want = expected_answers(ent, stacked[: L * 512])

    lib = ctypes.CDLL(os.path.join(HERE, "libold_slice.so"))
    lib.old_slice_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.c_int]
    dev = torch.device("cuda", 0)
    d_st = torch.from_numpy(stacked).to(dev)
    d_ent = torch.zeros(n + SLACK, dtype=torch.int32, device=dev)
    d_ent[:n] = torch.from_numpy(ent.view(np.int32)).to(dev)
    d_tab = torch.from_numpy(tab.view(np.int16)).to(dev)
    d_mask = torch.empty(n + SLACK, dtype=torch.uint8, device=dev)
    out = {"L": L, "S": S, "chunks": NC, "parts": PARTS, "keys": n, "variants": {}}
    runs = ((1, "launch_bounds(1024), U=8: no spill, 1 WG/CU"),
            (0, "launch_bounds(1024, 8), U=8: 1 VGPR spilled, 2 WG/CU (pre-fix)"),
            (0, "launch_bounds(1024, 8), U=8: 1 VGPR spilled, 2 WG/CU (pre-fix), again"),
            (2, "launch_bounds(1024, 8), U=8, +24 KiB LDS: 1 VGPR spilled, 1 WG/CU"),
            (3, "launch_bounds(1024, 8), U=6: no spill, 2 WG/CU"))
    for variant, name in runs:
        d_mask.fill_(0xEE)
        torch.cuda.synchronize()
        rc = lib.old_slice_launch(d_st.data_ptr(), L, S, NC, d_ent.data_ptr(), d_tab.data_ptr(),
                                  d_mask.data_ptr(), PARTS, variant)
        got = d_mask[:n].cpu().numpy()
        outside = int((d_mask[n:] != 0xEE).sum().item())
        bad = np.nonzero(got != want)[0]
        c_bad = bad // CHUNK
        part = (c_bad * PARTS) // NC
        c_lo = (part * NC) // PARTS
        wave = ((c_bad - c_lo) // 64) % 16
        out["variants"][name] = {
            "rc": rc, "mismatched_answers": int(bad.size), "writes_outside_regions": outside,
            "unwritten_0xEE_where_answer_differs": int(np.count_nonzero(got[bad] == 0xEE)),
            "mismatches_per_wave": np.bincount(wave, minlength=16).tolist(),
        }
        print(name, json.dumps(out["variants"][name]), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
