"""Per-kernel durations of the timed steps whose passes bench.py times.

Usage: python scripts/sampled_kernel_stats.py TRACE_DIR_OR_CSV STEPS

bench.py brackets the passes of every event_stride(STEPS)-th timed step with
HIP events, and those steps run their two passes one after the other, alone
on the GPU (the other steps overlap the build with the probe on two streams).
rocprofv3 --stats averages every launch, overlapped ones included; this
script reads the kernel trace of the same bench command and averages, per
library kernel, only the launches of the sampled steps (the last STEPS
launches of each step kernel are the timed steps, in order), then the probe
pass = partition + slice + unpermute, comparable with the bench line's
probe ms.
"""
import csv
import glob
import os
import re
import statistics as st
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def short(name):
    m = re.search(r"(\w+_kernel)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    from dlsm_amd.multigpu import event_stride

    every = event_stride(steps)
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    launches = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if "dlsm::" in r["Kernel_Name"]:
                launches.setdefault(short(r["Kernel_Name"]), []).append(
                    (int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    print(f"timed steps {steps}, passes timed on every {every}-th step (i % {every} == {every - 1})")
    print(f"{'kernel':<52} {'sampled us':>11} {'all timed us':>13}")
    probe = 0.0
    for k, v in sorted(launches.items()):
        if len(v) < steps:
            continue  # set-up kernels (the filter set's build, stacking)
        v = sorted(v)[-steps:]
        durs = [(e - s) / 1e3 for s, e in v]
        samp = [d for i, d in enumerate(durs) if i % every == every - 1]
        print(f"{k[:52]:<52} {st.mean(samp):>11.1f} {st.mean(durs):>13.1f}")
        if k.startswith(("probe_partition", "probe_slice", "probe_unpermute")):
            probe += st.mean(samp)
    print(f"probe pass (partition + slice + unpermute) on the sampled steps: {probe:.1f} us")


if __name__ == "__main__":
    main()
