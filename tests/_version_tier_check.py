"""Helper for test_gpu_version_tiers_forced: run under DLSM_VERSION_LDS=<m>
(read once per process) and check random versions -- from one file up to a
few hundred -- against the oracle in that table tier.  Prints 'ok N'."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

import dlsm_amd  # noqa: E402
import oracle  # noqa: E402
from test_version_probe import K, build_filter, random_version  # noqa: E402
from dlsm_amd import VersionFile  # noqa: E402


def main():
    ctx = dlsm_amd.Context(0)
    t = (1 << 8) | 1
    shapes = [[VersionFile(1, 1, K(100), K(200), t, build_filter(np.arange(100, 201, 3)))],
              [VersionFile(0, 2, K(0), K(50), t, build_filter(np.arange(0, 51, 2))),
               VersionFile(2, 3, K(10), K(20), t), VersionFile(2, 4, K(30), K(90), t)]]
    rng = np.random.default_rng(11)
    for n_l0 in (0, 5, 30):
        shapes.append(random_version(rng, n_l0, 1_000_000))
    done = 0
    for files in shapes:
        n = 100_003
        v_ = np.concatenate([rng.integers(0, 1_100_000, n - 2), [0, 1 << 40]]).astype(np.uint64)
        q = oracle.keys_from_values(v_)
        snap = int(rng.integers(1, 1 << 52))
        want, want_lf = oracle.version_probe(files, q, n, snapshot=snap)
        v = ctx.version(files)
        mask = torch.zeros(n, dtype=torch.uint64, device="cuda")
        lf = torch.zeros((n, 5), dtype=torch.int32, device="cuda")
        ctx.version_probe_dev(v, dlsm_amd.Keys(torch.from_numpy(q).cuda(), n, 20), snap, mask, lf)
        ctx.sync()
        assert np.array_equal(mask.cpu().numpy().view(np.uint64), want), (len(files), n_l0)
        assert np.array_equal(lf.cpu().numpy().view(np.uint32), want_lf), len(files)
        v.close()
        done += 1
    ctx.close()
    print("ok", done)


if __name__ == "__main__":
    main()
