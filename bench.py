#!/usr/bin/env python3
"""Benchmark: agents sized per second on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one resident batch: for every agent,
the bounded-Brent PV search (each evaluation = sticky rate switch + 25-year
Utilityrate5 bills + Cashloan cash flow / NPV / payback), then one PV+battery
forward run (sizing, 8760-h peak-shaving dispatch, battery-case bills and cash
flow) and the three 8760-h hourly output planes.  Inputs are resident in HBM
before timing starts.

Multi-GPU (torch.distributed.run, one rank per GPU): agents shard with no
data-path collective (weak scaling: --agents per GPU); a barrier + device sync
brackets the timed region and the slowest rank's time is reported.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "agents sized/sec (8760-h bill+NPV) at 1/2/4/8 GPU; % HBM roofline"
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md chip table (spec)
NH = 8760
# algorithmic bytes per agent of k_hourly_batt: read the agent's
# load-shape row (f32) and cf row (i32), write baseline / PV-only / with-battery
# hourly planes (f32), plus the bins and scalars it reads / writes
BYTES_HOURLY = NH * 4 * 2 + NH * 4 * 3 + 2 * 144 * 8 + 16 * 8
# k_size: row slot sums for the agent (load + cf, f64) + 4 yearly planes x 51 x 8 B
# + the bins it builds (2 x 12 P x 8 B, P<=12) + ~24 scalars in/out
BYTES_SIZE = 576 * 8 * 2 + 4 * 51 * 8 + 2 * 144 * 8 + 24 * 8
# k_batt_finance: battery bins (2 x 144 x 8) + 3 yearly planes + scalars
BYTES_FIN = 2 * 144 * 8 + 3 * 51 * 8 + 24 * 8


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--agents", type=int, default=1_000_000, help="agents per GPU")
    ap.add_argument("--config", default="res_1m_nem_tou")
    ap.add_argument("--no-hourly", action="store_true", help="on-device reduction mode")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--chunks", type=int, default=None,
                    help="size() pipeline depth (default: the library's DGEN_DEFAULT_CHUNKS)")
    ap.add_argument("--hb-months", type=int, default=None,
                    help="months per k_hourly_batt launch (default: the library's)")
    ap.add_argument("--order-major", default="load", choices=["cf", "load"],
                    help="profile_order grouping: by (cf_row, load_row) or (load_row, cf_row)")
    ap.add_argument("--caller-order", action="store_true",
                    help="keep the generator's agent order on device (no profile_order grouping)")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_bytes_per_agent.json"))
    return ap.parse_args()


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def cpu_baseline(pop, seconds: float, threads: int):
    """Time the CPU oracle ('port' of the reference semantics) on a bounded
    sample of the same workload (first agents of rank 0's shard)."""
    from oracle import oracle as orc
    from tests.helpers import oracle_population
    from dgen_amd.config import EngineConfig
    cfg = orc.make_cfg(**EngineConfig().oracle_kwargs())
    try:
        avail = len(os.sched_getaffinity(0))
    except Exception:
        avail = os.cpu_count() or 1
    threads = max(1, min(threads, avail))
    chunk = max(64, 32 * threads)
    n_take = min(pop.cols["load_kwh"].size, 200_000)
    sub = {k: v[:n_take] for k, v in pop.cols.items()}
    opop = oracle_population(sub, pop.tariffs, pop.switches, pop.shapes, pop.cfs, pop.wholesale,
                             demand=pop.demand)
    done, t0 = 0, time.perf_counter()
    while True:
        idx = list(range(done % n_take, min(done % n_take + chunk, n_take)))
        _, bad = opop.run_batch_timed(cfg, threads, idx)
        done += len(idx)
        el = time.perf_counter() - t0
        if el >= seconds or done >= n_take:
            break
    return {"value": done / el, "unit": "agents/s", "cores": threads, "kind": "port",
            "sample": f"{done} agents of the same synthetic workload ({pop.config}), "
                      f"oracle/orc.c full per-agent driver, OpenMP x{threads}, {el:.1f} s"}


def main():
    args = parse()
    ws, rank, local = dist_env()
    import torch
    import torch.distributed as dist
    if ws > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from dgen_amd.config import EngineConfig
    from dgen_amd.engine import Engine, profile_order
    from dgen_amd.synth import make_population

    pop = make_population(args.config, args.agents, seed=20260000 + 3 + 7919 * rank)
    # demand-charge configs run the extension mode; every other config the
    # reference's switch (SKIP_DEMAND_CHARGES = True, ff:35)
    eng = Engine(local if ws > 1 else 0, EngineConfig(skip_demand_charges=pop.skip_demand_charges))
    if args.chunks is not None:
        eng.set_pipeline(args.chunks)
    if args.hb_months is not None:
        eng.set_hourly_segment(args.hb_months)
    eng.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
    eng.set_tariffs(pop.tariffs, pop.demand)
    eng.set_switches(pop.switches)
    order = None if args.caller_order else profile_order(pop.cols, args.order_major)
    batch = eng.upload_agents(pop.cols, pop.n_scratch, order=order)
    out = eng.alloc_outputs(batch.n, hourly=not args.no_hourly)
    c_out = eng.c_outputs(out)
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        eng.size(batch, out, c_out)
    torch.cuda.synchronize()
    eng.kernel_times()                      # drop warmup events

    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.size(batch, out, c_out)
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if ws > 1:
        t = torch.tensor([el], dtype=torch.float64, device=eng.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ms_size, ms_hourly, ms_fin, cnt = eng.kernel_times()

    st = out["status"].cpu().numpy()
    n_bad = int(((st & 0x3B) != 0).sum())
    total_agents = args.agents * ws * args.steps
    value = total_agents / el

    kern = {"k_size": (ms_size, BYTES_SIZE), "k_hourly_batt": (ms_hourly, BYTES_HOURLY),
            "k_batt_finance": (ms_fin, BYTES_FIN)}
    dom = max(kern, key=lambda k: kern[k][0])
    hb_ms = ms_hourly
    bytes_launch = BYTES_HOURLY * args.agents if not args.no_hourly else (NH * 8 + 2 * 144 * 8) * args.agents
    achieved = bytes_launch / (hb_ms * 1e-3) / 1e9 if hb_ms > 0 else None
    traffic = None
    if os.path.exists(args.pmc):
        try:
            with open(args.pmc) as f:
                pm = json.load(f)
            traffic = float(pm["k_hourly_batt"]["hbm_bytes_per_agent"]) * args.agents
        except Exception:
            traffic = None
    n_launch = -(-12 // eng.hb_months) * eng.chunks
    roof = {"bound": "hbm", "kernel": "k_hourly_batt", "achieved": achieved, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
            # traffic and algorithmic bytes per launch (the year's bytes split evenly
            # over the month launches); the per-step totals beside them
            "traffic": (traffic / n_launch) if traffic else None,
            "algorithmic_bytes_per_launch": bytes_launch / n_launch,
            "traffic_per_step": traffic, "algorithmic_bytes_per_step": bytes_launch,
            "kernel_ms": {"k_size": ms_size, "k_hourly_batt": ms_hourly, "k_batt_finance": ms_fin},
            "dominant_kernel": dom, "event_samples": cnt,
            # k_hourly_batt sweeps the year in month segments: kernel_ms is the
            # per-step sum over these launches (rocprof reports per launch)
            "hourly_launches_per_step": n_launch}

    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu:
        try:
            cpu = cpu_baseline(pop, args.cpu_seconds, args.cpu_threads)
        except Exception as e:  # the baseline never blocks the GPU number
            cpu = {"value": None, "unit": "agents/s", "cores": 0, "kind": "port",
                   "sample": f"unavailable: {type(e).__name__}: {e}"}

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "agents/s", "n_gpus": ws,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (numpy PCG64 population per SURVEY 8d; no DB / agent files offline)",
            "config": {"workload": args.config, "agents_per_gpu": args.agents,
                       "global_agents": args.agents * ws,
                       "hourly_outputs": not args.no_hourly,
                       "demand_charges": not pop.skip_demand_charges,
                       "pipeline_chunks": eng.chunks, "hourly_months_per_launch": eng.hb_months,
                       "device_order": "caller" if args.caller_order else
                       ("profile (cf_row, load_row)" if args.order_major == "cf" else "profile (load_row, cf_row)"),
                       "parallelism": f"dp{ws} (agent shards, no collective in the step)",
                       "agents_with_status_errors": n_bad},
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
