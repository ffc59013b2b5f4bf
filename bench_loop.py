#!/usr/bin/env python3
"""Benchmark of the device model-year loop (BASELINE config C5: national
synthetic population, 2026-2050 diffusion loop with RCCL state totals).

Per model year, on every rank's resident shard (state pieces of one national
population, dgen_amd.partition: cut to equal predicted device cost, a state
split across ranks where balance needs it): per-year inputs, dgen_size_agents
(Brent PV sizing + PV+battery run), max market share, Bass diffusion,
largest-remainder battery attachment (split states' groups gathered and
allocated whole), per-state 8760-h export (in place from the sizing planes,
or by re-running the scan in chunks with --hourly-chunk for shards whose
planes do not fit), per-state totals, and one all-reduce of the per-state
totals + 8760-h rows (RCCL over xGMI for N > 1).  The line reports every
rank's measured time and sizing device time.

Launch like bench.py (python bench_loop.py, or torch.distributed.run with one
rank per GPU).  Weak scaling: --agents per GPU.  Prints ONE JSON line on rank 0:
value = agents x model years / slowest rank's time for the timed years.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--agents", type=int, default=1_000_000, help="agents per GPU")
    ap.add_argument("--config", default="national_mixed",
                    help="national_mixed (C5) or de_res (C1: Delaware residential, one GPU)")
    ap.add_argument("--first-year", type=int, default=2026)
    ap.add_argument("--step", type=int, default=1,
                    help="years between model years (C1: 2; the Bass step is teq + 2 either way, "
                         "diffusion_functions_elec.py:285)")
    ap.add_argument("--years", type=int, default=25, help="timed model years (2026-2050)")
    ap.add_argument("--no-batt", action="store_true", help="PV-only variant (no PV+battery forward run)")
    ap.add_argument("--exact", type=int, default=-1, choices=[-1, 0, 1, 2],
                    help="certified Brent paths (dgen_set_exact; bench.py --exact): -1 = the engine's default")
    ap.add_argument("--warmup", type=int, default=1, help="untimed model years, then reset")
    ap.add_argument("--hourly-chunk", type=int, default=None,
                    help="re-size chunks of this many agents for the state export")
    ap.add_argument("--no-export", action="store_true", help="skip the per-state hourly export")
    ap.add_argument("--export", default="auto", choices=["auto", "with_batt", "planes", "chunked"],
                    help="how the per-state rows are made (YearLoop export; auto: the with-battery plane alone "
                         "where it fits, else --hourly-chunk's re-run scans)")
    ap.add_argument("--cut-tol", type=float, default=0.02,
                    help="plan_partition tol: a rank cut snaps to a state boundary within this share of "
                         "the per-rank cost (0: cut inside states wherever balance puts the cut)")
    args = ap.parse_args()
    # --gpus N without torch.distributed.run: start N rank children before any
    # GPU call (dgen_amd.launch); under torchrun, WORLD_SIZE must equal --gpus
    from dgen_amd.launch import maybe_launch
    st = maybe_launch(args.gpus, __file__, sys.argv[1:])
    if st is not None:
        sys.exit(st)
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    # one rank per GPU (RCCL); DGEN_DIST_BACKEND=gloo rehearses the N > 1 flow
    # with several ranks on one GPU (device = LOCAL_RANK mod the visible GPUs)
    backend = os.environ.get("DGEN_DIST_BACKEND", "nccl")
    if ws > 1:
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    from dgen_amd import partition as P
    from dgen_amd.engine import Engine
    from dgen_amd.synth import STATES, make_population, national_tables, shard_population, split_state_members
    from dgen_amd.year_loop import LoopTables, YearLoop, loop_agents

    t_setup = time.perf_counter()
    cnum = 1 if args.config == "de_res" else 5
    n_global = args.agents * ws
    plan = None
    if args.config == "de_res":
        pop = make_population(args.config, args.agents, seed=20260000 + cnum + 7919 * rank,
                              state_pool=[STATES.index("DE")])
        ag = loop_agents(pop, agent_id0=rank * 2 * args.agents)
        sg = None
        n_rank = args.agents
    else:
        # national population by pieces (dgen_amd.partition): census state
        # sizes, the states cut into equal measured device cost per rank (the
        # per-path cost model over a per-state sample; a state is split across
        # ranks where balance needs it), every rank drawing its own pieces
        T = national_tables(args.config)
        naep_row = T.cfs.astype(np.float64).sum(axis=1) / 1e6
        sizes = P.census_sizes(n_global)
        cost = np.zeros(len(STATES))
        for s in range(len(STATES)):
            smp = make_population(args.config, 2000, tables=T, agent_seed=20268000 + s, state_pool=[s])
            cost[s] = P.cost_per_agent(smp.cols, naep_row[smp.cols["cf_row"]]).mean()
        plan = P.plan_partition(sizes, cost, ws, tol=args.cut_tol)
        pop, ag = shard_population(T, plan, rank)
        secs, ids = split_state_members(args.config, plan)
        sg = P.split_groups(plan, rank, secs, ids)
        n_rank = len(ag["agent_id"])
    from dgen_amd.config import EngineConfig
    eng = Engine(local if ws > 1 else 0, EngineConfig(exact_brent=args.exact))
    if args.no_batt:
        eng.set_battery(False)
    eng.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
    eng.set_tariffs(pop.tariffs)
    eng.set_switches(pop.switches)
    loop = YearLoop(eng, pop, ag, LoopTables.synthetic(), first_year=args.first_year,
                    hourly_export=not args.no_export, hourly_chunk=args.hourly_chunk, plan=plan, split=sg,
                    export=args.export)
    del pop
    setup_s = time.perf_counter() - t_setup
    for k in range(args.warmup):
        loop.run_year(args.first_year + k * args.step)
    loop.reset()
    eng.kernel_times()
    years = list(range(args.first_year, args.first_year + args.years * args.step, args.step))
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = [loop.run_year(y) for y in years]
    torch.cuda.synchronize()
    own = time.perf_counter() - t0                  # this rank's own time, before the barrier
    if ws > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    ms_size, ms_hourly, ms_fin, cnt = eng.kernel_times()
    # sizing device time per year of this rank (HIP events of the sizing kernels)
    dev_ms = (ms_size + ms_hourly + ms_fin) * (cnt / max(len(years), 1) if cnt else 0.0)
    n_total = n_rank
    per_rank = [[own, dev_ms, float(n_rank)]]
    if ws > 1:
        dev = eng.dev if backend == "nccl" else "cpu"
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        c = torch.tensor([float(n_rank)], dtype=torch.float64, device=dev)
        dist.all_reduce(c)
        n_total = int(c.item())
        g = torch.zeros((ws, 3), dtype=torch.float64, device=dev)
        g[rank] = torch.tensor(per_rank[0], dtype=torch.float64, device=dev)
        dist.all_reduce(g)
        per_rank = g.cpu().tolist()
    last = res[-1].totals.cpu().numpy()
    if rank == 0:
        line = {
            "metric": "agent-years/sec (national diffusion loop: sizing + diffusion + attachment "
                      "+ state export + all-reduced state totals)",
            "exchange_backend": (None if ws == 1 else ("RCCL" if backend == "nccl" else backend)),
            "value": n_total * len(years) / el, "unit": "agent-years/s", "n_gpus": ws,
            "steps": len(years), "warmup": args.warmup, "ms_per_step": el / len(years) * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic national population (numpy PCG64; synthetic Bass / max-market-share "
                    "/ attachment tables; no DB offline)",
            "config": {"workload": "national_loop" if args.config == "national_mixed" else f"{args.config}_loop",
                       "population": args.config, "year_step": args.step, "battery_run": not args.no_batt,
                       "certified_brent_paths": eng.cfg.exact_mode(),
                       "agents_per_gpu": args.agents,
                       "global_agents": n_total, "years": [years[0], years[-1]],
                       "state_mix": "census" if plan is not None else "DE",
                       "rank_partition": (None if plan is None else
                                          {"pieces_per_rank": [len(p_) for p_ in plan.pieces],
                                           "split_states": [STATES[s_] for s_ in plan.split_states()],
                                           "predicted_cost_max_over_mean": plan.imbalance()}),
                       "per_rank": {"seconds": [r_[0] for r_ in per_rank],
                                    "sizing_device_ms_per_year": [r_[1] for r_ in per_rank],
                                    "agents": [int(r_[2]) for r_ in per_rank],
                                    "measured_max_over_mean": (max(r_[0] for r_ in per_rank) /
                                                               (sum(r_[0] for r_ in per_rank) / len(per_rank)))},
                       "state_export": not args.no_export, "hourly_chunk": args.hourly_chunk,
                       "export_mode": loop.export_mode,
                       "parallelism": f"dp{ws} (state pieces per rank; split groups gathered, one all-reduce of state rows per year)"},
            "sizing_kernel_ms_per_call": {"k_size": ms_size, "k_hourly_batt": ms_hourly,
                                          "k_batt_finance": ms_fin, "launch_samples": cnt},
            "final_year": {"adopters": float(last[:, 3].sum()), "system_mw": float(last[:, 0].sum() / 1e3),
                           "batt_mw": float(last[:, 1].sum() / 1e3), "agents": float(last[:, 4].sum())},
            "setup_s": setup_s,
        }
        print(json.dumps(line), flush=True)
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
