"""Shrink a GPU session's outputs before they travel back (gpurun merges at
most 64 MiB): summarise rocprofv3 --pmc passes (pmc_summary.py) and kernel
traces (dlsm kernels only), then drop the raw CSVs whose rows carry the full
names of every torch kernel.

    python3 scripts/shrink_outputs.py OUTDIR
"""
import csv
import glob
import os
import shutil
import subprocess
import sys

d = sys.argv[1]
here = os.path.dirname(os.path.abspath(__file__))
if os.path.isdir(os.path.join(d, "pmc")):
    with open(os.path.join(d, "pmc_summary.txt"), "w") as f:
        subprocess.run([sys.executable, os.path.join(here, "pmc_summary.py"), os.path.join(d, "pmc")], stdout=f,
                       check=False)
    shutil.rmtree(os.path.join(d, "pmc"))
for tr in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    rows = [r for r in csv.DictReader(open(tr)) if "dlsm" in r["Kernel_Name"]]
    if rows:
        with open(tr[:-4] + "_dlsm.csv", "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
    os.remove(tr)
