"""Per-phase time of the persistent probe partition from in-kernel s_memtime
stamps (diagnostic; needs the stamps build):

    make variant TAG=stamps VFLAGS=-DDLSM_STAMPS=1
    DLSM_LIB_VARIANT=stamps python scripts/partition_stamps.py

Runs the bench's probe (100 M lookups vs 8 stacked 1.6 M-key filters) a few
times, then reads wave 0's stamps of every workgroup and chunk iteration and
prints the median and mean cycles of each phase of a chunk:
  0->1 hash unit 0 (tiles: LDS store, barrier, hash)   1->2 rank unit 0
  2->3 hash unit 1                                      3->4 rank unit 1
  4->5 pad + scan                                       5->6 tab row, pads, scatter
  6->7 entry / position stores + barrier                7->0' to the next chunk
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

WGS, ITERS, PH = 1024, 64, 8


def main():
    import torch

    import dlsm_amd
    from dlsm_amd import sharding as SH

    ctx = dlsm_amd.Context(0)
    stream = torch.cuda.Stream()
    ctx.set_stream(stream)
    work = SH.plan(0, 1, 16, 1_600_000, 100_000_000, "strong")
    inp = SH.make_inputs(ctx, work, 1_600_000, 8, 10, torch.device("cuda", 0), stream=stream)
    torch.cuda.synchronize()
    for _ in range(3):
        ctx.full_probe_dev(inp.fs, inp.lookups, inp.mask)
    ctx.sync()
    buf = np.zeros(WGS * ITERS * PH, dtype=np.uint64)
    lib = dlsm_amd.lib()
    rc = lib.dlsm_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(buf.size))
    assert rc == 0, rc
    st = buf.reshape(WGS, ITERS, PH).astype(np.int64)
    valid = (st != 0).all(axis=2)
    d = np.diff(st, axis=2)  # phases 0->1 .. 6->7
    nxt = st[:, 1:, 0] - st[:, :-1, 7]  # 7 -> next chunk's 0
    names = ["hash u0", "rank u0", "hash u1", "rank u1", "pad+scan", "tab+pads+scatter", "stores+barrier"]
    out = {"workgroups": int(valid.any(axis=1).sum()), "chunk_iters": int(valid.sum()), "phases": {}}
    for i, nm in enumerate(names):
        v = d[:, :, i][valid]
        out["phases"][nm] = {"median": float(np.median(v)), "mean": float(v.mean())}
    v = nxt[valid[:, 1:] & valid[:, :-1]]
    out["phases"]["to next chunk"] = {"median": float(np.median(v)), "mean": float(v.mean())}
    tot = (st[:, :, 7] - st[:, :, 0])[valid]
    out["chunk_total"] = {"median": float(np.median(tot)), "mean": float(tot.mean())}
    out["unit"] = "s_memtime ticks"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
