"""Median per-launch PMC values of the one-pass probe's kernels from the
passes of scripts/diag_mg_pmc.sh: python scripts/mg_pmc_summary.py OUT"""
import csv
import glob
import re
import statistics
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(f"{sys.argv[1]}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        m = re.search(r"::([a-z_]+_kernel)", r["Kernel_Name"])
        if m and ("probe_m" in m.group(1) or "probe_slice" in m.group(1)):
            vals[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in vals.items():
    print(k)
    for c, x in sorted(v.items()):
        print(f"  {c:24s} {statistics.median(x):.4g}")
