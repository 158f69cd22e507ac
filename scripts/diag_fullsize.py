import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import dlsm_amd, oracle
ctx = dlsm_amd.Context(0)
n = 1_600_000
tabs = [dlsm_amd.Keys(oracle.dbbench_keys(f, 8, n), n, 20) for f in range(8)]
want = [oracle.full_build(t.data, n) for t in tabs]
for path in (1, 2):
    ctx.set_path(path)
    got = ctx.full_build(tabs, 10)
    print("build path", path, [g == w for g, w in zip(got, want)], flush=True)
ctx.set_path(0)
fs = ctx.filterset(want)
for path in (1, 2):
    ctx.set_path(path)
    for f in range(2):
        m = ctx.full_probe(fs, tabs[f])
        bad = np.nonzero(((m >> f) & 1) == 0)[0]
        print("probe path", path, "filter", f, "false negatives", bad.size, bad[:10], flush=True)
    q = oracle.keys_from_values(oracle.mt_values(5, 25_600_000, 3_000_000))
    m = ctx.full_probe(fs, dlsm_amd.Keys(q, 3_000_000, 20))
    w = oracle.full_probe(want, q, 3_000_000, nthreads=8)
    d = np.nonzero(m != w)[0]
    print("probe path", path, "random mismatches", d.size, d[:10], flush=True)
