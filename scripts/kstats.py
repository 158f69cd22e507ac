"""Per-kernel rocprofv3 --stats summary: kstats.py <prof dir> [all].

Prints the dlsm kernels (every kernel with a second argument) and, when the
directory also holds a bench.json, its headline value."""
import csv
import json
import os
import sys

d = sys.argv[1]
rows = list(csv.DictReader(open(f'{d}/run_kernel_stats.csv')))
for r in rows:
    n = r['Name']
    if 'dlsm' not in n and len(sys.argv) < 3:
        continue
    print(f"{n[:80]:80s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:9.1f} min_us={float(r['MinNs'])/1e3:9.1f}")
if os.path.exists(f'{d}/bench.json'):
    b = json.load(open(f'{d}/bench.json'))
    print('value', b['value'], 'build', b['build'], 'probe', b['probe'])
