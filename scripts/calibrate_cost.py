#!/usr/bin/env python3
"""Measure the partition's per-path device cost (dgen_amd/partition.py
PATH_COST_NS) on one MI355X.

A national population is drawn against the shared tables; its agents are
split by billing path (engine.path_class: 0 bins / NEM, 1 net billing from the
scan-built split, 2 other hourly) and sector, and each class is sized alone
(warmup, then --reps timed calls, kernel times from the C-ABI's HIP events).
Per class: scan = (k_hourly_batt + k_batt_finance) ns per agent, per_eval =
k_size ns per agent / mean Brent evaluations (outputs["nfev"]).  Prints one
JSON line; the per-agent model is cost = scan + per_eval x E(L), E(L) the
Brent-depth bound (the partition only needs relative costs).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=100_000, help="agents per class")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    from dgen_amd import partition as P
    from dgen_amd.engine import Engine, path_class, profile_order
    from dgen_amd.synth import national_tables, make_population
    T = national_tables()
    eng = Engine(0)
    eng.load_profiles(T.shapes, T.cfs, T.wholesale)
    eng.set_tariffs(T.tt.array())
    eng.set_switches(T.switches)
    naep_row = T.cfs.astype(np.float64).sum(axis=1) / 1e6
    pool = make_population("national_mixed", 12 * args.agents, tables=T, agent_seed=20267000,
                           state_mix="census")
    pc = path_class(pool.cols)
    res = (pool.cols["flags"] & 1) != 0
    out_rows = {}
    for p in (0, 1, 2):
        for r in (True, False):
            idx = np.flatnonzero((pc == p) & (res == r))[: args.agents]
            if idx.size < 2000:
                continue
            cols = {k: np.asarray(v)[idx] for k, v in pool.cols.items()}
            batch = eng.upload_agents(cols, order=profile_order(cols))
            out = eng.alloc_outputs(batch.n, hourly=True)
            co = eng.c_outputs(out)
            eng.size(batch, out, co)
            torch.cuda.synchronize()
            eng.kernel_times()
            for _ in range(args.reps):
                eng.size(batch, out, co)
            torch.cuda.synchronize()
            ks, kh, kf, cnt = eng.kernel_times()
            nfev = out["nfev"].double().mean().item()
            E = P.brent_depth(cols["load_kwh"], naep_row[cols["cf_row"]]).mean()
            n = idx.size
            out_rows[f"{p},{int(r)}"] = {
                "path": p, "res": bool(r), "agents": int(n), "k_size_ms": ks, "k_hourly_batt_ms": kh,
                "k_batt_finance_ms": kf, "mean_nfev": nfev, "mean_E_bound": float(E),
                "scan_ns": (kh + kf) * 1e6 / n, "per_eval_ns": ks * 1e6 / n / max(E, 1e-9),
                "total_ns": (ks + kh + kf) * 1e6 / n}
            del batch, out, co
            torch.cuda.empty_cache()
    print(json.dumps({"calibration": out_rows}), flush=True)


if __name__ == "__main__":
    main()
