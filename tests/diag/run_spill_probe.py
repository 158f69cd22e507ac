"""Minimal reproducer for the commit-1c7c4c6 failure (diagnostic, run by hand
on a GPU box; output recorded under profiles/): in 1,024-thread workgroups at 8
waves per SIMD, with two workgroups per CU (64 KiB LDS each) and with one (24
KiB of extra dynamic LDS), (0) a value spilled to scratch and reloaded, and
(1) the pre-fix kernel's wave scan through ds_bpermute with its lane
addresses spilled and reloaded.  Prints the count of lanes that got a wrong
value.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared \
        tests/diag/spill_probe.hip -o tests/diag/libspill_probe.so
    python tests/diag/run_spill_probe.py
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    import torch

    lib = ctypes.CDLL(os.path.join(HERE, "libspill_probe.so"))
    lib.spill_probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int]
    blocks, iters = 4096, 2000
    n = blocks * 1024
    g = torch.Generator().manual_seed(7)
    vin = torch.randint(0, 1 << 31, (n,), generator=g, dtype=torch.int64).to(torch.int32).cuda()
    bad = torch.empty(n, dtype=torch.int32, device="cuda")
    out = {"blocks": blocks, "threads": 1024, "iters": iters, "runs": []}
    for kind, extra, label in ((0, 24, "spilled value, 1 WG/CU (88 KiB LDS)"),
                               (0, 0, "spilled value, 2 WG/CU (64 KiB LDS)"),
                               (1, 24, "spilled scan addresses, 1 WG/CU"),
                               (1, 0, "spilled scan addresses, 2 WG/CU"),
                               (1, 0, "spilled scan addresses, 2 WG/CU again")):
        bad.fill_(-1)
        torch.cuda.synchronize()
        rc = lib.spill_probe_launch(vin.data_ptr(), bad.data_ptr(), blocks, iters if kind == 0 else 200, extra,
                                    kind)
        b = (bad & 0x7FFFFFFF).cpu()
        lanes = int((b != 0).sum())
        waves_hit = int(((b.view(-1, 64) != 0).any(dim=1)).sum())
        r = {"config": label, "rc": rc, "lanes_with_bad_reload": lanes, "bad_reloads": int(b.sum()),
             "waves_hit": waves_hit, "waves": n // 64}
        out["runs"].append(r)
        print(json.dumps(r), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
