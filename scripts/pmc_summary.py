#!/usr/bin/env python3
"""Summarise rocprofv3 PMC CSVs: mean counter value per kernel per dispatch."""
import collections
import csv
import glob
import sys

tag = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/prof_{tag}_pmc_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        agg[(kn, r["Counter_Name"])].append(float(r["Counter_Value"]))
kernels = sorted({k for k, _ in agg})
for kn in kernels:
    if "k_" not in kn:
        continue
    print(kn)
    for (k, c), v in sorted(agg.items()):
        if k == kn:
            print(f"   {c:24s} n={len(v):2d} mean={sum(v)/len(v):.4g}")
