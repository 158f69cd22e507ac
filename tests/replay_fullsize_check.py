"""Config 5 at its stated size, sample-checked against the oracle (test
infrastructure; run by hand on a GPU box, output recorded under profiles/):

    python tests/replay_fullsize_check.py [--num 6250000 --threads 16]

Runs dbbench_replay.run (100 M fillrandom writes -> flushes + leveled
compactions, every filter built on the GPU from host keys; 100 M readrandom
Gets over the final version) and checks every `--every`-th built filter and the
first `--gets` Gets' filter answers against the oracle.  Prints one JSON line:
the replay's record plus the check counts.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_check(num=6_250_000, threads=16, every=97, gets=2_000_000, progress=None):
    """The replay at `num` writes per thread with oracle sampling; returns the
    replay record with an "oracle_check" entry.  `progress`: a callable given a
    line every ~20 s (a long run must show activity)."""
    import dbbench_replay as R
    import oracle

    chk = {"filters_checked": 0, "filters_bad": 0, "gets_checked": 0, "gets_bad": 0, "builds_seen": 0}
    t_last = [time.time()]
    say = progress or (lambda m: print(m, file=sys.stderr, flush=True))

    def on_build(values, filters):
        for v, f in zip(values, filters):
            chk["builds_seen"] += 1
            if chk["builds_seen"] % every == 1:
                chk["filters_checked"] += 1
                if f != oracle.full_build(oracle.keys_from_values(v), v.size):
                    chk["filters_bad"] += 1
        if time.time() - t_last[0] > 20:  # progress for the hang detector
            t_last[0] = time.time()
            say(f"[replay] {chk['builds_seen']} filters built")

    def on_read(b0, vals, masks, files):
        if b0 == 0:
            n = min(gets, vals.size)
            fo = [type("F", (), dict(level=f.level, number=f.number, smallest=f.smallest, largest=f.largest,
                                     largest_trailer=f.largest_trailer, filter=f.filter)) for f in files]
            want, _ = oracle.version_probe(fo, oracle.keys_from_values(vals[:n]), n, (1 << 56) - 1)
            chk["gets_checked"] = n
            chk["gets_bad"] = int(np.count_nonzero(want != masks[:n]))
        say(f"[replay] reads from {b0}")

    res, _ = R.run(num, threads, 10, on_build=on_build, on_read=on_read)
    res["oracle_check"] = chk
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num", type=int, default=6_250_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--every", type=int, default=97)
    ap.add_argument("--gets", type=int, default=2_000_000)
    args = ap.parse_args()
    res = run_check(args.num, args.threads, args.every, args.gets)
    chk = res["oracle_check"]
    print(json.dumps(res), flush=True)
    if chk["filters_bad"] or chk["gets_bad"]:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
