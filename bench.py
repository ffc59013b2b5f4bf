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
ROW_BYTES = NH * 4              # one f32 load-shape row or one i32 cf row
PLANE_BYTES = NH * 4            # one f32 hourly output plane per agent
SYS_BYTES = NH * 8              # the battery case's f64 system-output plane per agent


MAXP, DCP = 12, 8                 # include/dgen_hip.h DGEN_MAXP / DGEN_DCP
DCR_HEAD = 2 * 12 * DCP * 8 + 64  # a demand record's per-(month, period) max load + lower bound


def scratch_paths(cols, recs, tariff_final, *, battery=True, skip_dc=True, nb_scan=True,
                  dcr_on=True, has_wholesale=True, ts_scan=False):
    """Which scratch-slot agents move the battery case's f64 system-output
    plane and which hand k_batt_finance a compact record instead, per agent in
    the order of `cols` (dgen_hip.hip k_hourly_batt: put_sys / put_nb / put_dcr
    / skip_plane).  `tariff_final` is the battery case's tariff (after the
    storage switch, outputs["tariff_final"]); `recs` the engine's tariff
    records (Engine.tariff_records).  Returns (plane, nb_rec, dcr_rec, mo2, P)
    boolean / int arrays.  Agents whose record overflowed (the repair pass
    writes their plane) are counted as record agents: a lower bound.
    ts_scan: the TS sell-rate agents' split is built in their own scan
    (k_hourly_batt<TS>; dgen_size_agents' ts_split), so they hand a record too."""
    tf = np.asarray(tariff_final, np.int64)
    sl = np.asarray(cols["scratch_slot"]) >= 0
    mo, dc, unit = recs["mo"][tf], recs["dc"][tf], recs["unit"][tf]
    P = recs["P"][tf].astype(np.int64)
    mo2 = (mo == 2) | (mo == 3)
    has_dc = (dc > 0) & ((not skip_dc) | (unit == 1) | (unit == 3))
    ca = (np.asarray(cols["flags"]) & 2) != 0
    ts_on = (mo == 2) & ~ca & (np.asarray(cols["wholesale_row"]) >= 0) & bool(has_wholesale)
    put_sys = (mo2 | has_dc) & sl & bool(battery)
    put_nb = put_sys & mo2 & (~ts_on | bool(ts_scan)) & bool(nb_scan)
    put_dcr = put_sys & has_dc & bool(dcr_on)
    skip = (put_nb & ~has_dc) | (put_dcr & ~mo2)
    return put_sys & ~skip, put_nb, put_dcr, mo2, P


def algorithmic_bytes(cols, hourly: bool, battery: bool, paths=None, recs=None, ts_rows: int = 0):
    """ALGORITHMIC HBM bytes per step of each sizing kernel for this population
    (DESIGN.md section 5): the bytes the step cannot avoid moving.  Profile
    rows are shared: every distinct load-shape / cf row the batch uses is read
    once (a per-agent re-read that hits L2 / MALL is not HBM traffic);
    per-agent inputs and outputs are moved once each.
      k_size          the distinct rows' 576 (month, daytype, hour) slot sums
                      (f64, both tables), ~24 scalars and 4 yearly output
                      arrays of N+1 f64 per agent; the agents whose search
                      bills hourly imports (net billing, demand charges) also
                      read their distinct rows once.  Intermediate records
                      (the search's net-billing split, the demand envelopes)
                      are not counted: they are this implementation's, not
                      the algorithm's
      k_hourly_batt   the distinct rows, the agent's 12 x P (load, system)
                      bin pairs (NEM agents) + scalars, the three f32 hourly
                      planes when requested; the f64 system-output plane only
                      for the agents that write it (`scratch_paths`), and the
                      (month, period) sums / maxima of the compact records for
                      the agents that hand one to the finance kernel instead
                      (their variable hour entries are not counted: a lower
                      bound)
      k_batt_finance  bins + scalars + 3 yearly arrays per agent; the plane
                      agents read their plane and their distinct load rows,
                      the record agents their record's sums / maxima
    `paths` = scratch_paths(...) after a run; without it every scratch-slot
    agent is taken to write and read the plane (an upper bound).  `ts_rows`:
    the distinct TS rows the scan reads for the agents whose split it builds
    with the hourly sell rate (f64, 70 KB each)."""
    n = len(cols["load_kwh"])
    lr, cr = np.asarray(cols["load_row"]), np.asarray(cols["cf_row"])
    yearly = 8.0 * (np.asarray(cols["econ_life"], np.int64) + 1).sum()
    sl = np.asarray(cols["scratch_slot"]) >= 0
    if paths is None:
        plane, nbr, dcr, mo2 = sl, np.zeros(n, bool), np.zeros(n, bool), sl
        P = np.full(n, MAXP, np.int64)
    else:
        plane, nbr, dcr, mo2, P = paths
    distinct = lambda m, a: np.unique(a[m]).size if m.any() else 0
    rows = (np.unique(lr).size + np.unique(cr).size) * ROW_BYTES
    # the search bills hourly imports for the scratch-slot agents (initial tariff)
    rows_h = (distinct(sl, lr) + distinct(sl, cr)) * ROW_BYTES
    slots = (np.unique(lr).size + np.unique(cr).size) * 576 * 8
    k_size = slots + n * 24 * 8 + 4 * yearly + rows_h
    bins = float((12 * P * 16)[~mo2].sum())              # NEM agents' (load, system) pairs
    recb = float((12 * P * 4 * 8)[nbr].sum() + 64 * nbr.sum() + DCR_HEAD * dcr.sum())
    k_hourly = rows + n * 16 * 8 + bins + recb + int(ts_rows) * 8 * 8760
    if hourly:
        k_hourly += n * 3 * PLANE_BYTES
    if battery:
        k_hourly += plane.sum() * SYS_BYTES
    k_fin = (n * 24 * 8 + bins + 3 * yearly + recb + plane.sum() * SYS_BYTES +
             distinct(plane, lr) * ROW_BYTES) if battery else 0.0
    return {"k_size": float(k_size), "k_hourly_batt": float(k_hourly), "k_batt_finance": float(k_fin)}


def pmc_traffic(pmc_dir: str, workload: str):
    """Per-agent HBM bytes and VALU-busy fraction per kernel measured by
    rocprofv3 PMC on THIS workload (profiles/pmc/<workload>.json, written by
    scripts/pmc_summary.py): ({kernel: bytes}, {kernel: valu_busy}, source)."""
    path = os.path.join(pmc_dir, f"{workload}.json")
    if not os.path.exists(path):
        return {}, {}, None
    try:
        with open(path) as f:
            pm = json.load(f)
        key = lambda k: k[:-2] if k.endswith("_w") else k
        return ({key(k): float(v["hbm_bytes_per_agent"]) for k, v in pm.items() if "hbm_bytes_per_agent" in v},
                {key(k): float(v["valu_busy_frac"]) for k, v in pm.items() if "valu_busy_frac" in v},
                os.path.relpath(path, REPO))
    except Exception:
        return {}, {}, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=120)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--agents", type=int, default=1_000_000, help="agents per GPU")
    ap.add_argument("--config", default="res_1m_nem_tou")
    ap.add_argument("--no-hourly", action="store_true", help="on-device reduction mode")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="OpenMP threads of the CPU baseline (0 = every core this process may run on, "
                         "capped by OMP_NUM_THREADS when the environment sets it: the GPU box's CPU share)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--chunks", type=int, default=None,
                    help="size() pipeline depth (default: the library's DGEN_DEFAULT_CHUNKS)")
    ap.add_argument("--hb-months", type=int, default=None,
                    help="months per k_hourly_batt launch (default: the library's)")
    ap.add_argument("--hb-split", type=int, default=None, choices=[1, 2, 3, 4],
                    help="parts of k_hourly_batt's scan, each on its own stream (default the library's, 2; A/B; DGEN_HB_SPLIT)")
    ap.add_argument("--hb-nem", type=int, default=None, choices=[0, 1],
                    help="batches without scratch slots run the bins-only scan (1, default) or the general one "
                         "(0; A/B; DGEN_HB_NEM)")
    ap.add_argument("--order-major", default="load", choices=["cf", "load"],
                    help="profile_order grouping: by (cf_row, load_row) or (load_row, cf_row)")
    ap.add_argument("--caller-order", action="store_true",
                    help="keep the generator's agent order on device (no profile_order grouping)")
    ap.add_argument("--replan-hours", type=int, default=24, choices=[24, 1],
                    help="peak-shaving re-plan interval: 24 = a plan per day, 1 = re-planned every hour "
                         "over the next 24 h (DESIGN.md section 3)")
    ap.add_argument("--no-batt", action="store_true",
                    help="PV-only variant: no PV+battery forward run (SURVEY 8(d)); the reference always runs it")
    ap.add_argument("--exact", type=int, default=-1, choices=[-1, 0, 1, 2],
                    help="certified Brent paths (dgen_set_exact): 1 = re-run in the oracle's arithmetic the agents "
                         "a device / oracle difference bound does not settle, 0 = off, 2 = every agent; -1 (default) "
                         "= the engine's default (1 in the reference's mode, 0 with demand charges)")
    ap.add_argument("--pmc-dir", default=os.path.join(REPO, "profiles", "pmc"),
                    help="per-workload PMC summaries (traffic field); none -> traffic null")
    return ap.parse_args()


def _lib_default_split() -> int:
    from dgen_amd import _lib
    return _lib.DEFAULT_HOURLY_SPLIT


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def cpu_baseline(pop, seconds: float, threads: int, replan_hours: int = 24):
    """Time the CPU oracle ('port' of the reference semantics) on a bounded
    sample of the same workload (first agents of rank 0's shard), on every
    host core this process may run on (len(os.sched_getaffinity(0)), SURVEY
    8(d)(ii)): `value`.  The box's OMP_NUM_THREADS share (its CPU allotment
    for one GPU) is timed beside it as a secondary figure.  Each timed window
    cycles over the sample until `seconds` have passed."""
    from oracle import oracle as orc
    from tests.helpers import oracle_population
    from dgen_amd.config import EngineConfig
    cfg = orc.make_cfg(**EngineConfig(batt_update_hours=replan_hours).oracle_kwargs())
    try:
        avail = len(os.sched_getaffinity(0))
    except Exception:
        avail = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    share = min(avail, omp) if omp > 0 else avail
    threads = avail if threads <= 0 else max(1, min(threads, avail))
    n_take = min(pop.cols["load_kwh"].size, 200_000)
    sub = {k: v[:n_take] for k, v in pop.cols.items()}
    opop = oracle_population(sub, pop.tariffs, pop.switches, pop.shapes, pop.cfs, pop.wholesale,
                             demand=pop.demand)

    def window(nt, secs):
        chunk = max(64, 32 * nt)
        done, t0 = 0, time.perf_counter()
        while True:
            lo = done % n_take
            idx = list(range(lo, min(lo + chunk, n_take)))
            opop.run_batch_timed(cfg, nt, idx)
            done += len(idx)
            el = time.perf_counter() - t0
            if el >= secs:
                return done, el
    quota = cgroup_cpus()
    done, el = window(threads, seconds)
    runs = {threads: (done, el)}
    # the box's CPU allotment (cgroup quota / OMP_NUM_THREADS) can be far below
    # its affinity set: time that thread count too and report the faster one
    alt = min(x for x in (share, quota or share) if x)
    if alt != threads:
        runs[alt] = window(alt, max(5.0, seconds / 3))
    best = max(runs, key=lambda k: runs[k][0] / runs[k][1])
    d, e = runs[best]
    res = {"value": d / e, "unit": "agents/s", "cores": best, "kind": "port",
           "host_cpus": os.cpu_count(), "affinity_cpus": avail, "cgroup_cpu_quota": quota,
           "omp_num_threads_env": omp or None,
           "by_threads": {str(k): {"agents_per_s": v[0] / v[1], "agents": v[0], "seconds": round(v[1], 2)}
                          for k, v in runs.items()},
           "sample": f"{d} agent sizings over the first {n_take} agents of the same synthetic workload "
                     f"({pop.config}), oracle/orc.c full per-agent driver, OpenMP x{best} (the faster of "
                     f"{sorted(runs)} threads: all {avail} affinity CPUs and the box's CPU allotment), {e:.1f} s"}
    return res


def cgroup_cpus():
    """CPUs the cgroup quota allows (cpu.max quota / period), or None."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, per = f.read().split()[:2]
            if q != "max":
                return max(1, int(round(int(q) / int(per))))
        except Exception:
            pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        if q > 0:
            return max(1, int(round(q / per)))
    except Exception:
        pass
    return None


def timed_region(step, steps: int, sync, dist_mod=None, device=None) -> float:
    """The contract's timed region: barrier + device sync on both sides of
    exactly `steps` calls of `step`, then the MAX over ranks (one all-reduce;
    gloo on CPU in tests/test_dist.py, RCCL on GPU tensors here)."""
    if dist_mod is not None:
        dist_mod.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if dist_mod is not None:
        dist_mod.barrier()
    el = time.perf_counter() - t0
    if dist_mod is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64, device=device)
        dist_mod.all_reduce(t, op=dist_mod.ReduceOp.MAX)
        el = float(t.item())
    return el


def main():
    args = parse()
    # --gpus N without torch.distributed.run: start N rank children before any
    # GPU call (dgen_amd.launch); under torchrun, WORLD_SIZE must equal --gpus
    from dgen_amd.launch import maybe_launch
    st = maybe_launch(args.gpus, __file__, sys.argv[1:])
    if st is not None:
        sys.exit(st)
    ws, rank, local = dist_env()
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
    from dgen_amd.config import EngineConfig
    from dgen_amd.engine import Engine, profile_order
    from dgen_amd.synth import make_population

    if args.hb_nem is not None:
        os.environ["DGEN_HB_NEM"] = str(args.hb_nem)              # read by dgen_open
    if args.hb_split is not None:
        os.environ["DGEN_HB_SPLIT"] = str(args.hb_split)          # read by dgen_open
    pop = make_population(args.config, args.agents, seed=20260000 + 3 + 7919 * rank)
    # demand-charge configs run the extension mode; every other config the
    # reference's switch (SKIP_DEMAND_CHARGES = True, ff:35)
    eng = Engine(local if ws > 1 else 0, EngineConfig(skip_demand_charges=pop.skip_demand_charges,
                                                      batt_update_hours=args.replan_hours,
                                                      exact_brent=args.exact))
    if args.chunks is not None:
        eng.set_pipeline(args.chunks)
    if args.hb_months is not None:
        eng.set_hourly_segment(args.hb_months)
    if args.no_batt:
        eng.set_battery(False)
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

    el = timed_region(lambda: eng.size(batch, out, c_out), args.steps, torch.cuda.synchronize,
                      dist if ws > 1 else None, eng.dev if backend == "nccl" else "cpu")
    ms_size, ms_hourly, ms_fin, cnt = eng.kernel_times()
    if os.environ.get("DGEN_PHASE_PROF") and hasattr(eng.lib, "dgen_phase_read"):   # ablation builds only
        import ctypes
        ph = (ctypes.c_uint64 * 16)()
        if eng.lib.dgen_phase_read(ph, 0) == 0:
            print(json.dumps({"phase_cycles": list(ph)}), file=sys.stderr, flush=True)
    if hasattr(eng.lib, "dgen_clk_read"):      # clock-stamp ablation builds only (scripts/make_ablations.py)
        import ctypes
        import numpy as _np
        ck = (ctypes.c_uint64 * (4 * 8192))()
        if eng.lib.dgen_clk_read(ck) == 0:
            a = _np.frombuffer(ck, dtype=_np.uint64).reshape(4, 8192).astype(_np.float64)
            ok = (a[3] > a[1]) & (a[2] > a[0])
            ghz = (a[2][ok] - a[0][ok]) / (a[3][ok] - a[1][ok]) * 0.1
            if ghz.size:
                print(json.dumps({"hourly_clock_ghz": {"median": float(_np.median(ghz)), "p10": float(_np.percentile(ghz, 10)),
                                                       "p90": float(_np.percentile(ghz, 90)), "blocks": int(ghz.size)}}),
                      file=sys.stderr, flush=True)

    st = out["status"].cpu().numpy()
    n_bad = int(((st & 0x3B) != 0).sum())
    # agents the last timed call re-ran in the oracle's arithmetic (certified
    # Brent paths, dgen_set_exact; their cost is inside k_size's time)
    n_exact = eng.exact_count()
    total_agents = args.agents * ws * args.steps
    value = total_agents / el

    # which scratch-slot agents moved the f64 system-output plane and which a
    # compact record (the battery case's final tariff, the batch's switches)
    dcols = pop.cols if batch.perm is None else {k: np.asarray(v)[batch.perm] for k, v in pop.cols.items()}
    recs = eng.tariff_records
    # the record forms the kernels took in the last timed call (dgen_last_paths),
    # not a restatement of dgen_size_agents' gates
    lp = eng.last_paths()
    nb_on, dcr_on, ts_scan = bool(lp["nb_scan"]), bool(lp["dcr_on"]), bool(lp["ts_split"])
    tf_dev = out["tariff_final"].cpu().numpy()
    paths = scratch_paths(dcols, recs, tf_dev, battery=not args.no_batt,
                          skip_dc=pop.skip_demand_charges, nb_scan=nb_on, dcr_on=dcr_on,
                          has_wholesale=bool(eng.tables.wholesale), ts_scan=ts_scan)
    ts_rows = 0
    if ts_scan:
        wr = np.asarray(dcols["wholesale_row"])
        ts_ag = paths[1] & (recs["mo"][tf_dev] == 2) & ((np.asarray(dcols["flags"]) & 2) == 0) & (wr >= 0)
        ts_rows = int(np.unique(wr[ts_ag]).size) if ts_ag.any() else 0
    nbytes = algorithmic_bytes(dcols, not args.no_hourly, not args.no_batt, paths, ts_rows=ts_rows)
    traffic_pa, valu_busy, traffic_src = pmc_traffic(args.pmc_dir, args.config)
    # launches per step: k_hourly_batt sweeps the year in month-segment launches
    # per pipeline chunk; the year-lane kernels launch once per chunk
    launches = {"k_size": eng.chunks, "k_hourly_batt": -(-12 // eng.hb_months) * eng.chunks,
                "k_batt_finance": eng.chunks if not args.no_batt else 0}
    kms = {"k_size": ms_size, "k_hourly_batt": ms_hourly, "k_batt_finance": ms_fin}
    per_kernel = {}
    for k, t in kms.items():
        gbs = nbytes[k] / (t * 1e-3) / 1e9 if t > 0 else None
        per_kernel[k] = {"ms_per_step": t, "launches_per_step": launches[k],
                         "algorithmic_bytes_per_step": nbytes[k], "achieved_gbs": gbs,
                         "hbm_frac": (gbs / HBM_PEAK_GBS) if gbs else None,
                         "traffic_per_step": (traffic_pa[k] * args.agents) if k in traffic_pa else None,
                         "valu_busy_frac_pmc": valu_busy.get(k)}
    dom = max(kms, key=lambda k: kms[k])
    d = per_kernel[dom]
    nl = max(launches[dom], 1)
    # the roofline follows the dominant kernel's limiter: k_hourly_batt streams
    # its rows and hourly planes (HBM); the year-lane kernels (k_size,
    # k_batt_finance) re-bill per evaluation from LDS / registers and are
    # bound by fp64 VALU issue, so their line reports the PMC VALU-busy share
    # of this workload (profiles/pmc/<workload>.json) with the HBM fraction
    # kept as a secondary field
    valu_bound = dom != "k_hourly_batt" and valu_busy.get(dom) is not None
    if valu_bound:
        head = {"bound": "valu", "kernel": dom, "achieved": valu_busy[dom], "peak": 1.0,
                "unit": "VALU-busy fraction", "frac": valu_busy[dom]}
    else:
        head = {"bound": "hbm", "kernel": dom, "achieved": d["achieved_gbs"], "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": d["hbm_frac"]}
    roof = {**head, "hbm_frac": d["hbm_frac"], "hbm_achieved_gbs": d["achieved_gbs"],
            # per launch, like rocprof's per-dispatch durations (bytes / launches)
            "traffic": (d["traffic_per_step"] / nl) if d["traffic_per_step"] is not None else None,
            "algorithmic_bytes_per_launch": nbytes[dom] / nl, "launches_per_step": nl,
            "kernel_ms": kms, "per_kernel": per_kernel, "dominant_kernel": dom, "event_samples": cnt,
            "traffic_source": traffic_src if dom in traffic_pa else None,
            # the VALU side of the same kernel (PMC of this workload): share of
            # its dispatch the SIMDs spend issuing VALU (scripts/pmc_summary.py)
            "valu_busy_frac": valu_busy.get(dom),
            "note": ("k_hourly_batt streams its rows and planes (HBM roofline) and is co-limited by fp64 "
                     "VALU (valu_busy_frac)" if dom == "k_hourly_batt"
                     else (f"{dom} is fp64-VALU / latency bound (the year lanes re-bill per evaluation): "
                           "bound/frac are its PMC VALU-busy share; hbm_frac is secondary") if valu_bound
                     else f"{dom}: no PMC summary for this workload, HBM fraction only")}

    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu:
        try:
            cpu = cpu_baseline(pop, args.cpu_seconds, args.cpu_threads, args.replan_hours)
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
                       "battery_run": not args.no_batt,
                       "battery_replan_hours": args.replan_hours,
                       "pipeline_chunks": eng.chunks, "hourly_months_per_launch": eng.hb_months,
                       "hourly_scan_streams": int(os.environ.get("DGEN_HB_SPLIT", _lib_default_split())),
                       "device_order": "caller" if args.caller_order else
                       ("profile (cf_row, load_row)" if args.order_major == "cf" else "profile (load_row, cf_row)"),
                       "parallelism": f"dp{ws} (agent shards, no collective in the step)",
                       "agents_with_status_errors": n_bad,
                       "certified_brent_paths": {"mode": eng.cfg.exact_mode(),
                                                 "exact_reruns_per_step": n_exact}},
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
