"""Median per-dispatch PMC values by kernel from rocprofv3 --pmc passes: python tools/pmc_summary.py DIR [substr]"""
import collections
import csv
import glob
import statistics
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            agg[(r["Kernel_Name"][:60], r["Counter_Name"])][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
for (k, c), v in sorted(agg.items()):
    print(f"{k:60s} {c:36s} n={len(v):4d} median={statistics.median(v.values()):.4g}")
