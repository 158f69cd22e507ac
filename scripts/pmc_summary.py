import csv, sys, collections, glob, re
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f'{d}/p*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name']
        if 'dlsm' not in n: continue
        m = re.search(r'::([a-z_]+_kernel)(<[^>]*>)?\(', n)
        short = (m.group(1) + (m.group(2) or '')) if m else n[:60]
        agg[short][r['Counter_Name']].append(float(r['Counter_Value']))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        v2 = sorted(v)
        print(f"   {c:24s} n={len(v):3d} median={v2[len(v2)//2]:.4g} max={v2[-1]:.4g}")
