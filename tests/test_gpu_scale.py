"""Oracle checks at the configurations' per-GPU sizes (VERDICT r02 item 3,
r05 item 1): C2 (CA-like net billing + storage, 200k agents), national mix
(200k), C3 (1M residential NEM TOU), C4 (commercial, demand charges + battery,
1M agents = 8M / 8 GPUs) and a C5 model-year loop (national, 2.5M agents =
20M / 8 GPUs, three years, chunked hourly export).

At these sizes the batch exercises what small parity populations do not:
net-billing split records near their capacity, envelope overflow fallbacks,
the two-agent demand-charge build, chunked re-sizing for the state export.
Each test sizes the whole batch on the GPU in the bench's device order, then

* checks the Brent path of a 20 000-agent sample against the oracle (its
  OpenMP batch driver): every agent's nfev, system kW and last x (to 1e-9),
  sticky tariff state and NPV -- no allowance: the certified paths
  (dgen_set_exact) put every agent on the oracle's path;
* checks 150 of them in full (bills, payback, battery case, hourly planes)."""
import numpy as np
import pytest
import torch

from dgen_amd.engine import profile_order
from dgen_amd.synth import make_population
from oracle import oracle as orc
from tests import helpers

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

SAMPLE = 150
PATH_SAMPLE = 20_000
PATH_KEYS = ("system_kw", "x_last", "nfev", "npv", "tariff_final", "switched", "status", "payback_period")


def _check_sample(pop, out, idx, cfg, demand=None, hourly=True, tag="", search_tariff=None):
    opop = helpers.oracle_population({k: v[idx] for k, v in pop.cols.items()}, pop.tariffs, pop.switches,
                                     pop.shapes, pop.cfs, pop.wholesale, demand=demand)
    ref = opop.run(cfg, hourly=hourly)
    o = {k: out[k].cpu().numpy()[idx] for k in ("system_kw", "npv", "nfev", "payback_period", "batt_kwh",
                                                 "annual_kwh", "npv_pv_batt", "status", "x_last",
                                                 "tariff_final", "switched")}
    hp = {}
    if hourly:
        ti = torch.as_tensor(idx, device=out["baseline"].device)
        hp = {k: out[k].index_select(1, ti).permute(1, 0, 2).reshape(len(idx), -1).double().cpu().numpy()
              for k in ("baseline", "net_pvonly", "net_with_batt")}
    naep = pop.cfs.astype(np.float64).sum(axis=1) / 1e6
    for n_j, (j, r) in enumerate(zip(idx, ref)):
        assert o["status"][n_j] == 0 and r["status"] == 0, (tag, j)
        if search_tariff is not None and not helpers.same_path(o, n_j, r):
            # the fast search alone: compared where its search ended (its
            # sticky tariff state before the battery run's storage switch)
            xa = helpers.xatol_of(pop.cols["load_kwh"][j], naep[pop.cols["cf_row"][j]])
            o_s = dict(o, tariff_final=search_tariff)
            r = helpers.at_device_point(o_s, n_j, opop, n_j, cfg, r, xa, hourly=hourly)
        else:
            assert helpers.same_path(o, n_j, r), (tag, j, o["nfev"][n_j], r["nfev"])
        assert np.isclose(o["npv"][n_j], r["npv"], rtol=1e-6, atol=1e-6), (tag, j)
        assert o["payback_period"][n_j] == r["payback_period"], (tag, j)
        assert np.isclose(o["annual_kwh"][n_j], r["annual_kwh"], rtol=1e-9), (tag, j)
        assert np.isclose(o["batt_kwh"][n_j], r["batt_kwh"], rtol=1e-9), (tag, j)
        assert np.isclose(o["npv_pv_batt"][n_j], r["npv_pv_batt"], rtol=1e-6, atol=1e-6), (tag, j)
        for k_o, k_r in (("baseline", "baseline_net_hourly"), ("net_pvonly", "adopter_net_hourly_pvonly"),
                         ("net_with_batt", "adopter_net_hourly_with_batt")):
            if k_o in hp:
                ref_h = np.asarray(r[k_r], dtype=np.float64)
                assert np.allclose(hp[k_o][n_j], ref_h, rtol=2e-6,
                                   atol=2e-6 * max(1.0, np.abs(ref_h).max())), (tag, j, k_o)


def _path_sample(pop, o, idx, cfg, demand=None, tag=""):
    """The Brent path of every sampled agent against the oracle's OpenMP
    batch driver (o: the sample's device outputs, host arrays).  Returns the
    divergent agents (the callers require none)."""
    opop = helpers.oracle_population({k: v[idx] for k, v in pop.cols.items()}, pop.tariffs, pop.switches,
                                     pop.shapes, pop.cfs, pop.wholesale, demand=demand)
    ref = opop.run_parallel(cfg)
    div = []
    for n_j, r in enumerate(ref):
        assert o["status"][n_j] == 0 and r["status"] == 0, (tag, idx[n_j])
        if not (helpers.same_path(o, n_j, r) and o["tariff_final"][n_j] == r["tariff_final"]
                and o["switched"][n_j] == r["switched"]
                and np.isclose(o["npv"][n_j], r["npv"], rtol=1e-6, atol=1e-6)
                and o["payback_period"][n_j] == r["payback_period"]):
            div.append(int(idx[n_j]))
    print(f"\n{tag}: {len(ref)} sampled agents, Brent-path divergences {len(div)}: {div[:20]}", flush=True)
    return div


def _device_sample(out, dev_idx, hourly=True):
    ti = torch.as_tensor(np.asarray(dev_idx, np.int64), device=out["npv"].device)
    sub = {k: out[k].index_select(0, ti) for k in ("system_kw", "npv", "nfev", "payback_period", "batt_kwh",
                                                   "annual_kwh", "npv_pv_batt", "status", "x_last",
                                                   "tariff_final", "switched")}
    if hourly:
        sub.update({k: out[k].index_select(1, ti) for k in ("baseline", "net_pvonly", "net_with_batt")})
    return sub


def _size_at_scale(eng, pop, hourly=True, demand=None):
    """The whole population sized in the bench's device order; returns
    (device-order outputs, caller -> device row map, agents listed for the
    exact re-run)."""
    eng.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
    eng.set_tariffs(pop.tariffs, demand)
    eng.set_switches(pop.switches)
    batch = eng.upload_agents(pop.cols, pop.n_scratch, order=profile_order(pop.cols))
    out = eng.alloc_outputs(batch.n, hourly=hourly)
    eng.size(batch, out)
    torch.cuda.synchronize()
    n_ex = eng.exact_count()
    assert (out["status"].cpu().numpy() == 0).all()
    inv = np.empty(batch.n, np.int64)
    inv[batch.perm] = np.arange(batch.n)
    print(f"\n{batch.n} agents: {n_ex} re-run in the oracle's arithmetic ({100.0 * n_ex / batch.n:.3f} %)",
          flush=True)
    return out, inv, batch


def _path_check(pop, out, inv, seed, tag, demand=None, extra=None):
    from dgen_amd.synth import subset
    n = len(pop.cols["load_kwh"])
    rng = np.random.default_rng(seed)
    idx = rng.choice(n, PATH_SAMPLE, replace=False)
    if extra is not None:
        idx = np.concatenate([idx, extra])
    idx = np.unique(idx)
    ti = torch.as_tensor(inv[idx], device=out["npv"].device)
    o = {k: out[k].index_select(0, ti).cpu().numpy() for k in PATH_KEYS}
    return _path_sample(subset(pop, idx), o, np.arange(idx.size), orc.make_cfg(), demand=demand, tag=tag), idx


def test_c2_ca_like_200k_sample_vs_oracle(engine):
    """C2 (CA-like, net billing with the NEM3 sell rate, storage) at 200k in
    the bench's device order; the battery-case split built in the scan."""
    from dgen_amd.synth import subset
    n = 200_000
    pop = make_population("ca_res_storage", n, seed=20260000 + 2 + 101)
    out, inv, batch = _size_at_scale(engine, pop)
    assert batch.nb_scan
    div, _ = _path_check(pop, out, inv, 22, "C2 200k")
    assert not div, div
    idx = np.sort(np.random.default_rng(12).choice(n, SAMPLE, replace=False))
    sample = _device_sample(out, inv[idx])
    del out, batch
    torch.cuda.empty_cache()
    _check_sample(subset(pop, idx), sample, np.arange(SAMPLE), orc.make_cfg(), tag="C2")


def test_national_200k_sample_vs_oracle(engine):
    """The national mix at 200k with hourly planes, in the bench's device
    order: NEM bins, the scan-built net-billing split (CA and no-TS agents)
    and the TS sell-rate agents' own scan (k_hourly_batt<TS>) in one batch; a
    20 000-agent path sample and 150 agents in full (50 on the TS path)."""
    from dgen_amd.engine import path_class
    from dgen_amd.synth import subset
    n = 200_000
    pop = make_population("national_mixed", n, seed=20260000 + 5 + 211)
    out, inv, batch = _size_at_scale(engine, pop)
    assert batch.nb_scan and batch.ts_rows[1] > batch.ts_rows[0]
    div, _ = _path_check(pop, out, inv, 25, "national 200k")
    assert not div, div
    rng = np.random.default_rng(15)
    ts = np.flatnonzero(path_class(pop.cols) == 2)
    idx = np.unique(np.concatenate([rng.choice(n, SAMPLE - 50, replace=False), rng.choice(ts, 50, replace=False)]))
    sample = _device_sample(out, inv[idx])
    del out, batch
    torch.cuda.empty_cache()
    _check_sample(subset(pop, idx), sample, np.arange(idx.size), orc.make_cfg(), tag="national")


def test_c3_1m_path_sample_vs_oracle(engine):
    """C3 (the bench workload: 1M residential NEM TOU agents) in the bench's
    device order: a 20 000-agent Brent-path sample against the oracle."""
    n = 1_000_000
    pop = make_population("res_1m_nem_tou", n, seed=20260000 + 3)
    out, inv, batch = _size_at_scale(engine, pop, hourly=False)
    div, _ = _path_check(pop, out, inv, 33, "C3 1M")
    del out, batch
    torch.cuda.empty_cache()
    assert not div, div


# C4 Brent-path divergences of the fast search alone (the extension mode's
# default: certified paths off) in the 20 000-agent sample, pinned
C4_FAST_DIVERGENCES_MAX = 60


def test_c4_commercial_dc_1m_sample_vs_oracle(engine_dc):
    """C4 per GPU (8M commercial agents over 8 GPUs): demand charges billed
    (extension mode), battery run, as the bench runs it -- the fast search
    alone (certified paths off, the mode's default).  A 20 000-agent Brent-path
    sample against the oracle: the divergent agents are counted, printed and
    pinned; 1000 agents in full, each compared at the device's own point when
    its path left the oracle's (the outputs equal the oracle's driver there,
    kW within scipy's xatol)."""
    from dgen_amd.synth import subset
    eng = engine_dc
    eng.set_exact(0)
    try:
        n = 1_000_000
        pop = make_population("com_dc_batt", n, seed=20260000 + 4 + 101)
        out, inv, batch = _size_at_scale(eng, pop, demand=pop.demand)
        div, _ = _path_check(pop, out, inv, 44, "C4 1M (fast search alone)", demand=pop.demand)
        assert len(div) <= C4_FAST_DIVERGENCES_MAX, len(div)
        k = 1000
        idx = np.sort(np.random.default_rng(13).choice(n, k, replace=False))
        sample = _device_sample(out, inv[idx])
        del out, batch                       # the 1M-agent planes (105 GB) before the next test
        torch.cuda.empty_cache()
        # the sample's search-end tariff state: the same agents sized alone
        # with the battery run off (agents are independent of their batch)
        sp = subset(pop, idx)
        eng.set_battery(False)
        try:
            b2 = eng.upload_agents(sp.cols, sp.n_scratch)
            o2 = eng.alloc_outputs(b2.n, hourly=False)
            eng.size(b2, o2)
            torch.cuda.synchronize()
            st = o2["tariff_final"].cpu().numpy()
            assert np.array_equal(o2["nfev"].cpu().numpy(), sample["nfev"].cpu().numpy())
        finally:
            eng.set_battery(True)
        _check_sample(sp, sample, np.arange(k), orc.make_cfg(), demand=pop.demand, tag="C4",
                      search_tariff=st)
    finally:
        eng.set_exact(1)


def test_c5_loop_2p5m_sample_vs_oracle(engine):
    """C5 per GPU (20M national agents over 8 GPUs): three model years of the
    resident loop with the chunked hourly export; each year a sample's sizing
    (with the year's gathered inputs) and Bass step against the oracle."""
    from dgen_amd.year_loop import LoopTables, YearLoop, loop_agents
    from dgen_amd.synth import STATES, subset
    from oracle import diffusion as od
    import gc
    gc.collect()
    torch.cuda.empty_cache()
    n = 2_500_000
    pop = make_population("national_mixed", n, seed=20260000 + 5 + 101, state_mix="census")
    engine.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
    engine.set_tariffs(pop.tariffs)
    engine.set_switches(pop.switches)
    ag = loop_agents(pop, agent_id0=0)
    tabs = LoopTables.synthetic()
    loop = YearLoop(engine, pop, ag, tabs, first_year=2026, hourly_export=True, hourly_chunk=500_000)
    inv = np.empty(n, np.int64)
    inv[loop.perm] = np.arange(n)
    idx = np.sort(np.random.default_rng(14).choice(n, SAMPLE, replace=False))
    di = torch.as_tensor(inv[idx], device=engine.dev)
    bass = tabs.bass.set_index(["state_abbr", "sector_abbr"])
    sec = ["res" if s == 0 else "com" for s in ag["sector"][idx]]
    st = [STATES[s] for s in ag["state"][idx]]
    p = np.array([bass.loc[(a, b), "bass_param_p"] for a, b in zip(st, sec)])
    q = np.array([bass.loc[(a, b), "bass_param_q"] for a, b in zip(st, sec)])
    t1 = np.array([bass.loc[(a, b), "teq_yr1"] for a, b in zip(st, sec)])
    m = tabs.mms_df
    for y in (2026, 2027, 2028):
        r = loop.run_year(y, keep_per_agent=True)
        assert np.isfinite(r.hourly.cpu().numpy()).all()
        # the sample's gathered inputs for this year -> the oracle's sizing
        cols = {k: v.index_select(0, di).cpu().numpy() for k, v in loop.batch.cols.items()}
        sp = subset(pop, idx)
        sp.cols.update({k: cols[k] for k in sp.cols if k in cols and k != "scratch_slot"})
        ref = helpers.oracle_population(sp.cols, pop.tariffs, pop.switches, pop.shapes, pop.cfs,
                                        pop.wholesale).run(orc.make_cfg())
        g = {k: loop.out[k].index_select(0, di).cpu().numpy() for k in ("system_kw", "npv", "payback_period",
                                                                         "nfev", "status")}
        for k_, rr in enumerate(ref):
            assert g["status"][k_] == 0 and g["nfev"][k_] == rr["nfev"], (y, k_)
            assert abs(g["system_kw"][k_] - rr["system_kw"]) <= 1e-9 * rr["system_kw"], (y, k_)
            assert np.isclose(g["npv"][k_], rr["npv"], rtol=1e-6, atol=1e-6), (y, k_)
            assert g["payback_period"][k_] == rr["payback_period"], (y, k_)
        # the sample's Bass step from its own carry and max market share
        pa = {k: v.index_select(0, di).cpu().numpy() for k, v in r.per_agent.items()
              if hasattr(v, "index_select") and v.dim() == 1 and v.shape[0] == n}
        _, _, mms = od.max_market_share(g["payback_period"], sec, m["sector_abbr"].tolist(),
                                        m["payback_period"].to_numpy(), m["max_market_share"].to_numpy(),
                                        m["payback_period"].to_numpy())
        assert np.array_equal(pa["max_market_share"], mms, equal_nan=True), y
        cust = loop.cust.index_select(0, di).cpu().numpy()
        d = od.diffusion(mms, pa["market_share_last_year_in"], p, q, t1, cust, g["system_kw"],
                         cols["capex"], pa["adopters_cum_last_year_in"], pa["market_value_last_year_in"],
                         pa["system_kw_cum_last_year_in"], y == 2026)
        for k in ("market_share", "new_adopters", "number_of_adopters", "system_kw_cum"):
            assert np.allclose(pa[k], d[k], rtol=1e-12, atol=1e-12), (y, k)


def test_rank_shards_balanced_on_measured_device_time(engine):
    """The 8 rank shards of a 2.5M-agent census national population (the C5
    per-GPU scale: 20M over 8 GPUs would be 8x each shard), cut by the
    partition's per-path cost model with states split where balance needs it,
    sized one after the other on this GPU: measured device time (HIP events
    of the sizing kernels) max / mean <= 1.15."""
    from dgen_amd import partition as P
    from dgen_amd.synth import STATES, national_tables, shard_population
    T = national_tables()
    engine.load_profiles(T.shapes, T.cfs, T.wholesale)
    engine.set_tariffs(T.tt.array())
    engine.set_switches(T.switches)
    naep_row = T.cfs.astype(np.float64).sum(axis=1) / 1e6
    sizes = P.census_sizes(2_500_000)
    cost = np.zeros(len(STATES))
    for s in range(len(STATES)):
        smp = make_population("national_mixed", 2000, tables=T, agent_seed=20268000 + s, state_pool=[s])
        cost[s] = P.cost_per_agent(smp.cols, naep_row[smp.cols["cf_row"]]).mean()
    plan = P.plan_partition(sizes, cost, 8)
    times, counts = [], []
    for r in range(8):
        pop, _ = shard_population(T, plan, r)
        batch = engine.upload_agents(pop.cols, pop.n_scratch, order=profile_order(pop.cols))
        out = engine.alloc_outputs(batch.n, hourly=True)
        co = engine.c_outputs(out)
        engine.size(batch, out, co)
        torch.cuda.synchronize()
        engine.kernel_times()
        for _ in range(3):
            engine.size(batch, out, co)
        torch.cuda.synchronize()
        ks, kh, kf, cnt = engine.kernel_times()
        times.append(ks + kh + kf)
        counts.append(batch.n)
        del batch, out, co
        torch.cuda.empty_cache()
    t = np.asarray(times)
    print(f"\nrank shards: agents {counts}, device ms {np.round(t, 2).tolist()}, "
          f"predicted max/mean {plan.imbalance():.3f}, measured max/mean {t.max() / t.mean():.3f}, "
          f"split states {[STATES[s] for s in plan.split_states()]}")
    assert t.max() / t.mean() <= 1.15
