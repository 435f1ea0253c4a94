"""Summarise a tools/profile.sh output directory: per-kernel average of every counter."""
import csv, collections, sys, glob, os
d = sys.argv[1]
for f in glob.glob(os.path.join(d, 'kt', '*kernel_stats.csv')):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:70]:70s} calls={r['Calls']:>4} avg_ms={float(r['AverageNs'])/1e6:.4f}")
agg = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, '*', '*counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name']
        if 'ipp' not in n and 'k_' not in n: continue
        short = n.split('(')[0].split('::')[-1][:40]
        agg[(short, r['Counter_Name'])].append(float(r['Counter_Value']))
for (k, c), v in sorted(agg.items()):
    print(f"{k:40s} {c:28s} {sum(v)/len(v):14.5g}  (n={len(v)})")
