"""Times K bench steps issued by tests/diag/step_loop_lib.cc (one C call)
from a torch process, beside the same K steps issued per call from Python
(as bench.py does).  Prints one JSON line.  Build the helper on the box:
g++ -shared -fPIC -I include tests/diag/step_loop_lib.cc -o bin/libstep_loop.so
-L dlsm_amd/lib -ldlsm_bloom"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch

    import dlsm_amd
    from dlsm_amd import _lib as L
    from dlsm_amd import sharding as SH

    dev = torch.device("cuda", 0)
    ctx = dlsm_amd.Context(0)
    st = torch.cuda.Stream(device=dev)
    ctx.set_stream(st)
    work = SH.plan(0, 1, 16, 1_600_000, 100_000_000, "strong")
    inp = SH.make_inputs(ctx, work, 1_600_000, 8, 10, dev, stream=st, dist=None)
    torch.cuda.synchronize()
    lib = C.CDLL(os.path.join(ROOT, "bin", "libstep_loop.so"))
    lib.step_loop_run.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                  C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    tabs, outs, lens, fs, qk, mask = inp.tables, inp.outs, inp.lens, inp.fs, inp.lookups, inp.mask
    jobs = ctx._jobs(tabs, outs, [int(o.numel()) for o in outs])
    ks = qk.c()
    K = 50
    res = {}
    for rep in range(2):
        for mode in ("python_per_call", "c_loop"):
            for _ in range(5):
                ctx.full_build_dev(tabs, outs, lens, 10)
                ctx.full_probe_dev(fs, qk, mask)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if mode == "c_loop":
                rc = lib.step_loop_run(ctx.h, jobs, len(tabs), 10, lens.data_ptr(), ctx.h, fs.h, C.byref(ks),
                                       mask.data_ptr(), K)
                assert rc == 0, rc
            else:
                for _ in range(K):
                    ctx.full_build_dev(tabs, outs, lens, 10)
                    ctx.full_probe_dev(fs, qk, mask)
            torch.cuda.synchronize()
            res[f"{mode}_{rep}_ms_per_step"] = round((time.perf_counter() - t0) / K * 1e3, 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
