"""Summarise a tools/profile.sh output directory: kernel-trace stats, then the
per-dispatch average of every PMC counter per kernel."""
import collections
import csv
import glob
import os
import re
import sys


def short(name: str) -> str:
    m = re.search(r"(k_\w+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name[:40]


d = sys.argv[1]
for f in glob.glob(os.path.join(d, "kt", "*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        print(f"{short(r['Name']):40s} calls={r['Calls']:>5} avg_ms={float(r['AverageNs']) / 1e6:.4f}")
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "k_" not in r["Kernel_Name"]:
            continue
        key = (short(r["Kernel_Name"]), r["Counter_Name"])
        agg[key][r.get("Dispatch_Id", "")] += float(r["Counter_Value"])
for (k, c), v in sorted(agg.items()):
    print(f"{k:40s} {c:24s} {sum(v.values()) / len(v):14.5g}  (n={len(v)})")
