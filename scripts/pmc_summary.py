#!/usr/bin/env python3
"""Summarise rocprofv3 PMC CSVs of one workload: per-agent HBM bytes and VALU
activity of each sizing kernel family, summed over its template
instantiations.

usage: pmc_summary.py 'DIR_GLOB' AGENTS OUT_JSON [CALLS]
  DIR_GLOB  rocprofv3 -d directories of the workload's PMC passes (one pass
            per counter group; each pass runs the same bench command)
  AGENTS    agents per sizing call
  OUT_JSON  e.g. profiles/pmc/<workload>.json (read by bench.py --pmc-dir)
  CALLS     sizing calls per pass (bench --steps + --warmup); measured from
            the dispatches of the k_size_w instantiations when omitted

Accounting (round 6).  A kernel family (k_hourly_batt, k_size_w, ...) runs
several instantiations per call -- national: k_hourly_batt<NB>, <TS> and the
bins-only scan, with different dispatch counts and very different sizes.  Each
instantiation is keyed by its FULL name (template arguments included); its
counters are averaged over its own dispatches and multiplied by its own
dispatches per call; the family figure is the sum over instantiations.
(Round 5 averaged over all instantiations by base name and multiplied by one
dispatch count, which undercounted national k_hourly_batt.)

HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE
are KiB from the L2's memory-side request counters; on gfx950 FETCH_SIZE
reports half the bytes of a wide streaming read, so it is doubled.  The json
keeps the raw per-instantiation counters beside the corrected totals."""
from __future__ import annotations

import collections
import csv
import glob
import json
import re
import sys

SIMDS = 256 * 4          # MI355X: 256 CUs x 4 SIMDs
XCDS = 8


def inst_name(kernel_name: str) -> str:
    """'void (anonymous namespace)::k_size_w<32, false>(dgen_tables, ...)' ->
    'k_size_w<32, false>' (template arguments kept, parameter list dropped)."""
    s = kernel_name.replace("(anonymous namespace)::", "").replace("dgen_srch::", "")
    s = re.sub(r"^void ", "", s.strip())
    depth, cut = 0, len(s)
    for i, ch in enumerate(s):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    return s[:cut].strip()


def family(inst: str) -> str:
    return inst.split("<")[0]


def summarize(files, agents: int, calls: float | None = None) -> dict:
    vals = collections.defaultdict(list)          # (inst, counter) -> values
    disp = collections.defaultdict(set)           # (file, inst) -> dispatch ids
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                inst = inst_name(r["Kernel_Name"])
                if not inst.startswith("k_"):
                    continue
                vals[(inst, r["Counter_Name"])].append(float(r["Counter_Value"]))
                disp[(f, inst)].add(r["Dispatch_Id"])
    # sizing calls per pass: given, or the largest k_size_w instantiation count
    # (each present instantiation launches once per call and pipeline chunk)
    per_file_calls = {}
    for f in files:
        if calls is not None:
            per_file_calls[f] = float(calls)
        else:
            ks = [len(ids) for (ff, i), ids in disp.items() if ff == f and family(i) == "k_size_w"]
            if ks:
                per_file_calls[f] = float(max(ks))
    per_call = collections.defaultdict(list)      # inst -> dispatches per call, per pass
    for (f, inst), ids in disp.items():
        if per_file_calls.get(f):
            per_call[inst].append(len(ids) / per_file_calls[f])
    insts = sorted({i for i, _ in vals})
    res = {}
    for fam in sorted({family(i) for i in insts}):
        members = {}
        tot = collections.defaultdict(float)      # family counters per call
        for inst in (i for i in insts if family(i) == fam):
            means = {c: sum(v) / len(v) for (i, c), v in vals.items() if i == inst}
            dpc = (sum(per_call[inst]) / len(per_call[inst])) if per_call.get(inst) else 1.0
            members[inst] = {"counters_per_dispatch": means, "dispatches_per_call": round(dpc, 4)}
            for c, m in means.items():
                tot[c] += m * dpc
        rec = {"instantiations": members, "counters_per_call": dict(tot),
               "dispatches_per_call": round(sum(m["dispatches_per_call"] for m in members.values()), 4),
               "agents": agents}
        if "FETCH_SIZE" in tot and "WRITE_SIZE" in tot:
            rd = 2.0 * tot["FETCH_SIZE"] * 1024.0
            wr = tot["WRITE_SIZE"] * 1024.0
            rec.update({"hbm_read_bytes_per_call": rd, "hbm_write_bytes_per_call": wr,
                        "hbm_bytes_per_agent": (rd + wr) / agents,
                        "hbm_read_bytes_per_agent": rd / agents, "hbm_write_bytes_per_agent": wr / agents,
                        "correction": "sum over instantiations of (2 x FETCH_SIZE (gfx950 half-count) + "
                                      "WRITE_SIZE) x its dispatches per call"})
        if "SQ_INSTS_VALU" in tot:
            rec["valu_wave_insts_per_agent"] = tot["SQ_INSTS_VALU"] / agents
        if tot.get("SQ_ACTIVE_INST_ANY"):
            rec["valu_share_of_active"] = tot.get("SQ_ACTIVE_INST_VALU", 0.0) / tot["SQ_ACTIVE_INST_ANY"]
        if "SQ_INSTS_VALU" in tot and tot.get("GRBM_GUI_ACTIVE"):
            # VALU issue share of the family's dispatches: a wave64 VALU
            # instruction holds its SIMD 4 cycles (16 lanes / clock, fp64 and
            # 32-bit alike on CDNA4); GRBM_GUI_ACTIVE sums the busy clocks of
            # the 8 XCDs (PMC passes serialise dispatches)
            rec["valu_busy_frac"] = tot["SQ_INSTS_VALU"] * 4.0 / (SIMDS * tot["GRBM_GUI_ACTIVE"] / XCDS)
            rec["valu_busy_note"] = "sum SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x sum GRBM_GUI_ACTIVE / 8)"
        res[fam] = rec
    return res


def main(argv):
    pattern, agents, out_json = argv[1], int(argv[2]), argv[3]
    calls = float(argv[4]) if len(argv) > 4 else None
    files = []
    for d in sorted(glob.glob(pattern)):
        files += sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True))
    res = summarize(files, agents, calls)
    for fam, rec in res.items():
        print(fam, {k: (round(v, 4) if isinstance(v, float) else v) for k, v in rec.items()
                    if k not in ("instantiations", "counters_per_call")})
        for inst, m in rec["instantiations"].items():
            print(f"   {inst:70s} x{m['dispatches_per_call']}")
    with open(out_json, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", out_json, "from", len(files), "csv files")


if __name__ == "__main__":
    main(sys.argv)
