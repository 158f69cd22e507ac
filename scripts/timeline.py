"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV.

Usage: python scripts/timeline.py DIR_OR_CSV [--steps K]

Takes the library's kernels (dlsm::...) of the last K steps, groups them by
stream, and prints per kernel kind: mean duration and mean idle gap before it
on its stream; then the mean step span (first start to last end per step) and
the fraction of that span with at least one dlsm kernel running.
"""
import argparse
import csv
import glob
import os
import re
import statistics as st


def short(name):
    m = re.search(r"(\w+_kernel)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def load(path):
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        if not cands:
            raise SystemExit(f"no kernel_trace.csv under {path}")
        path = cands[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if "dlsm::" not in r["Kernel_Name"]:
                continue
            stream = r.get("Stream_Id") or r.get("Queue_Id")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), stream, short(r["Kernel_Name"])))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--first", default="full_partition_kernel", help="kernel that starts a step")
    a = ap.parse_args()
    rows = load(a.path)
    starts = [i for i, r in enumerate(rows) if r[3].startswith(a.first)]
    if len(starts) < a.steps + 1:
        raise SystemExit(f"only {len(starts)} steps found")
    lo = starts[-a.steps - 1]
    sel = rows[lo:]
    last_end = {}
    per = {}
    for s, e, q, k in sel:
        gap = s - last_end[q] if q in last_end else None
        last_end[q] = e
        d = per.setdefault((q, k), {"dur": [], "gap": []})
        d["dur"].append(e - s)
        if gap is not None:
            d["gap"].append(gap)
    print(f"{'stream':>8} {'kernel':<48} {'n':>4} {'mean us':>9} {'min us':>8} {'gap before us':>14}")
    for (q, k), d in sorted(per.items(), key=lambda x: (x[0][0], -st.mean(x[1]["dur"]))):
        g = st.mean(d["gap"]) / 1e3 if d["gap"] else float("nan")
        print(f"{q:>8} {k[:48]:<48} {len(d['dur']):>4} {st.mean(d['dur'])/1e3:>9.1f} {min(d['dur'])/1e3:>8.1f} {g:>14.1f}")
    t0, t1 = sel[0][0], max(r[1] for r in sel)
    span = t1 - t0
    # busy = union of kernel intervals
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in sel:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    n = len(starts) - starts.index(lo) - 0
    steps = sum(1 for r in sel if r[3].startswith(a.first))
    print(f"steps {steps}: span {span/1e3/steps:.1f} us/step, some kernel running {busy/span:.3f} of it")


if __name__ == "__main__":
    main()
