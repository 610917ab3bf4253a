#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per-dispatch mean of each counter for one kernel."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "k_env_step"
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{d}/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    v = sorted(v)
    print(f"{k:28s} n={len(v):3d} median={v[len(v)//2]:.4g} mean={sum(v)/len(v):.4g}")
