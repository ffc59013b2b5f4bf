"""Device model-year loop (dgen_amd.year_loop, BASELINE C5) vs the numpy
oracle chain, three model years on a small national population.

Sizing parity is covered by test_gpu_synthetic / test_gpu_parity; here the
device sizing outputs of each year are the inputs of the oracle chain
(max market share -> Bass step -> largest-remainder attachment -> export
weights -> per-state hourly sums -> per-state totals -> carry), so the test
checks every step the loop adds and the year-to-year carry."""
import numpy as np
import pytest
import torch

from dgen_amd.engine import hourly_agent_major
from dgen_amd.synth import STATES, make_population
from dgen_amd.year_loop import SECTORS, LoopTables, YearLoop, loop_agents
from dgen_amd.market import YearTables
from oracle import attach as oa
from oracle import diffusion as od
from oracle import market as om

pytestmark = pytest.mark.gpu

N = 2500
YEARS = [2026, 2027, 2028]


def _setup(engine, hourly_chunk=None, seed=20269001, config="national_mixed", first_year=YEARS[0], export="auto"):
    pool = [STATES.index("DE")] if config == "de_res" else None
    pop = make_population(config, N, seed=seed, n_res_shapes=64, n_com_shapes=32,
                          n_cf=32, n_counties=16, n_tariffs=48, state_pool=pool)
    engine.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
    engine.set_tariffs(pop.tariffs)
    engine.set_switches(pop.switches)
    ag = loop_agents(pop, agent_id0=1000)
    tabs = LoopTables.synthetic()
    return pop, ag, tabs, YearLoop(engine, pop, ag, tabs, first_year=first_year,
                                   hourly_export=True, hourly_chunk=hourly_chunk, export=export)


@pytest.mark.parametrize("config,years", [("national_mixed", YEARS),
                                          # C1: Delaware residential, 2-year steps from 2022
                                          ("de_res", [2022, 2024, 2026])])
def test_year_loop_matches_oracle_chain(engine, config, years):
    YEARS = years
    pop, ag, tabs, loop = _setup(engine, config=config, first_year=years[0], export="planes")
    perm = loop.perm
    inv = np.empty(N, np.int64)
    inv[perm] = np.arange(N)
    h = lambda t: t.cpu().numpy()[inv]                    # device order -> caller order
    st, sec = ag["state"], ag["sector"]
    sec_s = [SECTORS[c] for c in sec]
    bass = tabs.bass.set_index(["state_abbr", "sector_abbr"])
    p = np.array([bass.loc[(STATES[s], SECTORS[c]), "bass_param_p"] for s, c in zip(st, sec)])
    q = np.array([bass.loc[(STATES[s], SECTORS[c]), "bass_param_q"] for s, c in zip(st, sec)])
    t1 = np.array([bass.loc[(STATES[s], SECTORS[c]), "teq_yr1"] for s, c in zip(st, sec)])
    m = tabs.mms_df
    # the per-year inputs restated on the host (caller order): elec.apply_*
    # merges, pinned to the reference by tests/test_market.py
    import pandas as pd
    frame = pd.DataFrame({"state_abbr": [STATES[s] for s in st], "sector_abbr": sec_s,
                          "county_id": ag["county"]})
    yt = YearTables(frame, tabs.inputs, tabs.inflation_rate)
    load0, cust0 = pop.cols["load_kwh"], ag["customers_in_bin"]
    carry = {k: np.zeros(N) for k in ("ms", "adopt", "mv", "skc", "bkw", "bkwh")}
    for y in YEARS:
        r = loop.run_year(y, keep_per_agent=True)
        o = {k: h(loop.out[k]) for k in ("payback_period", "system_kw", "batt_kw", "batt_kwh")}
        assert (h(loop.out["status"]) == 0).all()
        yin = yt.gather_host(y, load0, cust0, load0 * cust0)
        for k in ("load_kwh", "capex", "escalator", "price_mult", "pv_deg", "itc_frac"):
            assert np.array_equal(h(loop.batch.cols[k]), yin[k]), (y, k)
        capex, cust = yin["capex"], yin["customers_in_bin"]
        if y == YEARS[0]:      # elec.estimate_initial_market_shares from the state starting capacities
            ini = om.initial_market_shares([STATES[s] for s in st], sec_s, ["solar"] * N, cust, capex,
                                           tabs.caps.to_dict(orient="list"))
            for k_c, k_i in (("ms", "market_share_last_year"), ("adopt", "adopters_cum_last_year"),
                             ("mv", "market_value_last_year"), ("skc", "system_kw_cum_last_year"),
                             ("bkw", "batt_kw_cum_last_year"), ("bkwh", "batt_kwh_cum_last_year")):
                carry[k_c] = ini[k_i]
                assert np.array_equal(h(r.per_agent[k_i + "_in"]), ini[k_i]), k_i
        _, _, mms = od.max_market_share(o["payback_period"], sec_s, m["sector_abbr"].tolist(),
                                        m["payback_period"].to_numpy(), m["max_market_share"].to_numpy(),
                                        m["payback_period"].to_numpy())
        got_mms = h(r.per_agent["max_market_share"])
        assert np.array_equal(got_mms, mms, equal_nan=True), y
        d = od.diffusion(mms, carry["ms"], p, q, t1, cust, o["system_kw"],
                         capex, carry["adopt"], carry["mv"], carry["skc"], y == YEARS[0])
        for k in ("market_share", "new_adopters", "number_of_adopters", "market_value", "system_kw_cum"):
            assert np.allclose(h(r.per_agent[k]), d[k], rtol=1e-12, atol=1e-12), (y, k)
        att = oa.allocate([STATES[s] for s in st], sec_s, ag["agent_id"], h(r.per_agent["new_adopters"]),
                          tabs.attach_rate[st], o["batt_kw"], o["batt_kwh"], carry["bkw"], carry["bkwh"])
        assert np.array_equal(h(r.per_agent["added"]), att["batt_adopters_added_this_year"]), y
        assert np.allclose(h(r.per_agent["batt_kw_cum"]), att["batt_kw_cum"], rtol=1e-12, atol=1e-12)
        # per-state hourly export from the loop's own planes (caller order)
        w = oa.weights(cust, h(r.per_agent["number_of_adopters"]), carry["bkw"],
                       o["batt_kw"], att["batt_adopters_added_this_year"])
        planes = [hourly_agent_major(loop.out[k]).cpu().numpy()[inv].astype(np.float64)
                  for k in ("baseline", "net_pvonly", "net_with_batt")]
        ex = oa.export([STATES[s] for s in st], planes[0], planes[1], planes[2], w)
        hr = r.hourly.cpu().numpy()
        for s_name, ref in zip(ex["state_abbr"], ex["net_sum"]):
            assert np.allclose(hr[STATES.index(s_name)], ref, rtol=1e-10, atol=1e-9), (y, s_name)
        # per-state totals (dgen_model.py:437-440) + adopters and agent count
        tot = r.totals.cpu().numpy()
        for s in np.unique(st):
            mk = st == s
            ref = [d["system_kw_cum"][mk].sum(), att["batt_kw_cum"][mk].sum(),
                   att["batt_kwh_cum"][mk].sum(), d["number_of_adopters"][mk].sum(), mk.sum()]
            assert np.allclose(tot[s], ref, rtol=1e-11, atol=1e-9), (y, STATES[s])
        absent = np.setdiff1d(np.arange(len(STATES)), np.unique(st))
        assert not tot[absent].any()
        carry = {"ms": d["market_share"], "adopt": d["number_of_adopters"], "mv": d["market_value"],
                 "skc": d["system_kw_cum"], "bkw": att["batt_kw_cum"], "bkwh": att["batt_kwh_cum"]}
    assert carry["adopt"].sum() > 0 and carry["bkw"].sum() > 0     # the market actually moved


def test_chunked_hourly_export_matches_in_place(engine):
    """hourly_chunk re-sizes the shard in chunks (short last chunk included) for
    the export; it must agree with the export from the in-place planes."""
    *_, whole = _setup(engine, export="planes")
    *_, chunked = _setup(engine, hourly_chunk=1000, export="chunked")
    for y in YEARS[:2]:
        a, b = whole.run_year(y), chunked.run_year(y)
        assert torch.equal(a.totals, b.totals), y
        assert torch.allclose(a.hourly, b.hourly, rtol=1e-12, atol=1e-9), y


def test_with_batt_plane_export_is_bit_identical(engine):
    """export="with_batt" (the default where it fits): the sizing scan writes
    the with-battery plane alone and dgen_state_hourly_rows recomputes the load
    and PV-only net load from the rows -- the per-state rows equal the
    three-plane export's bit for bit (and the chunked re-run's), every year."""
    *_, planes = _setup(engine, export="planes")
    *_, wo = _setup(engine, export="with_batt")
    *_, chunked = _setup(engine, hourly_chunk=1700, export="chunked")
    assert wo.export_mode == "with_batt" and wo.out["baseline"] is None
    for y in YEARS:
        a, b, c = planes.run_year(y), wo.run_year(y), chunked.run_year(y)
        assert torch.equal(a.totals, b.totals), y
        assert torch.equal(a.hourly, b.hourly), y
        assert torch.allclose(c.hourly, b.hourly, rtol=1e-12, atol=1e-9), y
        assert b.hourly.abs().sum() > 0


@pytest.mark.parametrize("world,balanced", [(2, False), (3, True)])
def test_state_shards_reproduce_one_pool(engine, world, balanced):
    """Multi-GPU by construction: the ranks' state shards (rank_states(r, world),
    round robin or balanced by predicted work) run one after the other on this
    GPU reproduce the single-pool loop -- per-agent results bit for bit,
    per-state totals and hourly rows as the all-reduce would merge them
    (states are disjoint across ranks)."""
    from dgen_amd.synth import subset
    from dgen_amd.year_loop import population_work, rank_states
    pop, ag, tabs, whole = _setup(engine)
    sw = (np.bincount(ag["state"], weights=population_work(pop), minlength=len(STATES))
          if balanced else None)
    years = [2026, 2027]
    full = [whole.run_year(y, keep_per_agent=True) for y in years]
    full_out = {k: whole.out[k].cpu().numpy()[np.argsort(whole.perm)] for k in ("system_kw", "npv", "batt_kw")}
    tot = [np.zeros_like(r.totals.cpu().numpy()) for r in full]
    hrs = [np.zeros_like(r.hourly.cpu().numpy()) for r in full]
    seen = np.zeros(N, bool)
    for rank in range(world):
        mine = np.isin(ag["state"], rank_states(rank, world, state_work=sw))
        idx = np.nonzero(mine)[0]
        seen |= mine
        sp = subset(pop, idx)
        sa = {k: np.asarray(v)[idx] for k, v in ag.items()}
        loop = YearLoop(engine, sp, sa, tabs, first_year=years[0], hourly_export=True)
        for j, y in enumerate(years):
            r = loop.run_year(y, keep_per_agent=True)
            tot[j] += r.totals.cpu().numpy()
            hrs[j] += r.hourly.cpu().numpy()
            inv = np.argsort(loop.perm)
            fk = lambda t: t.cpu().numpy()[np.argsort(whole.perm)][idx]
            for k in ("market_share", "number_of_adopters", "system_kw_cum"):
                assert np.array_equal(r.per_agent[k].cpu().numpy()[inv], fk(full[j].per_agent[k])), (rank, y, k)
        for k, v in full_out.items():
            assert np.array_equal(loop.out[k].cpu().numpy()[np.argsort(loop.perm)], v[idx]), (rank, k)
    assert seen.all()
    for j in range(len(years)):
        assert np.array_equal(tot[j], full[j].totals.cpu().numpy()), years[j]
        assert np.allclose(hrs[j], full[j].hourly.cpu().numpy(), rtol=0, atol=0), years[j]


def test_lifetime_raised_by_year_table_reaches_the_kernels(engine):
    """A financing table that raises the economic lifetime from 25 to 40 in a
    later model year: the loop refreshes the batch's max_years from the year's
    gather, so the sizing kernels switch to one agent per wave and every agent
    sizes over 40 years -- bit for bit what a fresh upload of the same
    gathered columns gives (max_years was computed once)."""
    import copy
    pop = make_population("national_mixed", N, seed=20269002, n_res_shapes=64, n_com_shapes=32,
                          n_cf=32, n_counties=16, n_tariffs=48)
    engine.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
    engine.set_tariffs(pop.tariffs)
    engine.set_switches(pop.switches)
    ag = loop_agents(pop, agent_id0=7)
    tabs = copy.deepcopy(LoopTables.synthetic())
    fin = tabs.inputs["financing"]
    fin.loc[fin["year"] == 2027, "economic_lifetime_yrs"] = 40
    loop = YearLoop(engine, pop, ag, tabs, first_year=2026, hourly_export=False)
    loop.run_year(2026)
    assert loop.batch.c_agents.max_years == 25
    loop.run_year(2027)
    assert loop.batch.c_agents.max_years == 40
    assert (loop.out["status"].cpu().numpy() == 0).all()
    assert (loop.batch.cols["econ_life"].cpu().numpy() == 40).all()
    # the same gathered columns uploaded fresh (device order, no permutation)
    cols = {k: v.cpu().numpy() for k, v in loop.batch.cols.items()}
    fresh = engine.upload_agents(cols, n_scratch=loop.batch.n_scratch)
    assert fresh.c_agents.max_years == 40
    out = engine.alloc_outputs(N, hourly=False)
    engine.size(fresh, out)
    torch.cuda.synchronize()
    for k in ("system_kw", "npv", "payback_period", "npv_pv_batt"):
        assert np.array_equal(loop.out[k].cpu().numpy(), out[k].cpu().numpy(), equal_nan=True), k
    # year 40's cash flow is live, year 41's is not
    cf = loop.out["cash_flow"].cpu().numpy()
    assert np.abs(cf[:, 40]).max() > 0 and not cf[:, 41:].any()


@pytest.mark.parametrize("world", [2, 3])
def test_split_state_shards_reproduce_one_pool(engine, world):
    """States cut across ranks (partition.plan_partition with cuts inside
    states): the shards run in lockstep on this GPU, their exchanges summed as
    the all-reduce would (year_loop.run_lockstep), and reproduce the one-pool
    loop bit for bit -- per-agent diffusion and battery allocation (split
    (state, sector) groups allocated whole from the gather), the first year's
    initial market, per-state totals and 8760-h rows (chunk partials summed in
    chunk order)."""
    from dgen_amd import partition as P
    from dgen_amd.synth import national_tables, shard_population, split_state_members
    from dgen_amd.year_loop import run_lockstep
    T = national_tables(n_res_shapes=64, n_com_shapes=32, n_cf=32, n_counties=16, n_tariffs=48)
    engine.load_profiles(T.shapes, T.cfs, T.wholesale)
    engine.set_tariffs(T.tt.array())
    engine.set_switches(T.switches)
    tabs = LoopTables.synthetic()
    sizes = P.census_sizes(3000)
    chunk = 64
    cost = np.ones(sizes.size)
    cost[STATES.index("CA")] = 40.0                      # cuts inside CA (and others)
    plan = P.plan_partition(sizes, cost, world, chunk=chunk, tol=0.0)
    assert plan.split_states()
    whole = P.whole_plan(sizes, chunk=chunk)
    pop1, ag1 = shard_population(T, whole, 0)
    one = YearLoop(engine, pop1, ag1, tabs, first_year=2026, hourly_export=True, plan=whole)
    secs, ids = split_state_members("national_mixed", plan)
    shards = []
    for r in range(world):
        pop, ag = shard_population(T, plan, r)
        sg = P.split_groups(plan, r, secs, ids)
        shards.append((ag, YearLoop(engine, pop, ag, tabs, first_year=2026, hourly_export=True, plan=plan,
                                    split=sg)))
    keys = ("market_share", "number_of_adopters", "system_kw_cum", "added", "batt_kw_cum", "batt_kwh_cum",
            "market_share_last_year_in", "adopters_cum_last_year_in", "system_kw_cum_last_year_in")
    ref_id = ag1["agent_id"][one.perm]
    for y in (2026, 2027, 2028):
        ref = one.run_year(y, keep_per_agent=True)
        res = run_lockstep([lp for _, lp in shards], y, keep_per_agent=True)
        pos = {int(a): i for i, a in enumerate(ref_id)}
        for (ag, lp), r in zip(shards, res):
            assert torch.equal(r.totals, ref.totals), (y, "totals")
            assert torch.equal(r.hourly, ref.hourly), (y, "hourly")
            ix = np.array([pos[int(a)] for a in ag["agent_id"][lp.perm]])
            for k in keys:
                a = r.per_agent[k].cpu().numpy()
                b = ref.per_agent[k].cpu().numpy()[ix]
                assert np.array_equal(a, b), (y, k)
        assert ref.per_agent["added"].sum() > 0
