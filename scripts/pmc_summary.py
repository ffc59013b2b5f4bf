#!/usr/bin/env python3
"""Summarise rocprofv3 PMC CSVs: mean counter value per kernel per dispatch,
and per-agent HBM bytes of each sizing kernel.

usage: pmc_summary.py TAG AGENTS [OUT_JSON]

HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE
are KiB from the L2's memory-side request counters; on gfx950 FETCH_SIZE
reports half the bytes of a wide streaming read, so it is doubled.  Our loads
are 16 B/lane but not coalesced across lanes and our stores are 4 B/lane, an
access width the guide lists as uncalibrated -- the json carries the raw
counters beside the corrected total."""
import collections
import csv
import glob
import json
import os
import sys

tag, agents = sys.argv[1], int(sys.argv[2])
# k_hourly_batt runs as HB_LAUNCHES month-segment launches per sizing call
# (dgen_set_hourly_segment): its per-agent bytes sum the per-launch means
HB_LAUNCHES = int(os.environ.get("HB_LAUNCHES", "12"))
out_json = sys.argv[3] if len(sys.argv) > 3 else f"gpurun_out/prof_{tag}_pmc_bytes.json"
agg = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/prof_{tag}_pmc_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0]
        agg[(kn, r["Counter_Name"])].append(float(r["Counter_Value"]))
kernels = sorted({k for k, _ in agg})
res = {}
for kn in kernels:
    if not kn.startswith("k_"):
        continue
    print(kn)
    means = {}
    for (k, c), v in sorted(agg.items()):
        if k == kn:
            means[c] = sum(v) / len(v)
            print(f"   {c:24s} n={len(v):2d} mean={means[c]:.4g}")
    if "FETCH_SIZE" in means and "WRITE_SIZE" in means:
        per_call = HB_LAUNCHES if kn == "k_hourly_batt" else 1
        rd = 2.0 * means["FETCH_SIZE"] * 1024.0 * per_call
        wr = means["WRITE_SIZE"] * 1024.0 * per_call
        res[kn] = {"fetch_size_kib": means["FETCH_SIZE"], "write_size_kib": means["WRITE_SIZE"],
                   "hbm_read_bytes": rd, "hbm_write_bytes": wr,
                   "hbm_bytes_per_agent": (rd + wr) / agents, "agents": agents,
                   "launches_per_call": per_call,
                   "correction": "2 x FETCH_SIZE (gfx950 half-count) + WRITE_SIZE"}
        print(f"   -> HBM bytes/agent {(rd + wr) / agents:.1f} (read {rd / agents:.1f}, write {wr / agents:.1f})")
json.dump(res, open(out_json, "w"), indent=1)
print("wrote", out_json)
