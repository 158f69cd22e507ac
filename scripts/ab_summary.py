"""Median build/probe ms per label of a scripts/gpu_ab.sh directory."""
import glob
import json
import re
import statistics
import sys
from collections import defaultdict

rows = defaultdict(list)
for f in sorted(glob.glob(f"{sys.argv[1]}/*.json")):
    m = re.match(r"(.*)_(\d+)\.json$", f.split("/")[-1])
    if not m:
        continue
    d = json.load(open(f))
    rows[m.group(1)].append((d["value"], d["build"]["ms"], d["probe"]["ms"]))
for k, v in rows.items():
    print(f"{k:14s} n={len(v)} value={statistics.median(x[0] for x in v):10.1f} "
          f"build_ms={statistics.median(x[1] for x in v):.4f} probe_ms={statistics.median(x[2] for x in v):.4f}")
