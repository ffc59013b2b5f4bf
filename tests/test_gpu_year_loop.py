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
from oracle import attach as oa
from oracle import diffusion as od

pytestmark = pytest.mark.gpu

N = 2500
YEARS = [2026, 2027, 2028]


def _setup(engine, hourly_chunk=None, seed=20269001):
    pop = make_population("national_mixed", N, seed=seed, n_res_shapes=64, n_com_shapes=32,
                          n_cf=32, n_counties=16, n_tariffs=48)
    engine.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
    engine.set_tariffs(pop.tariffs)
    engine.set_switches(pop.switches)
    ag = loop_agents(pop, agent_id0=1000)
    tabs = LoopTables.synthetic()
    return pop, ag, tabs, YearLoop(engine, pop, ag, tabs, first_year=YEARS[0],
                                   hourly_export=True, hourly_chunk=hourly_chunk)


def test_year_loop_matches_oracle_chain(engine):
    pop, ag, tabs, loop = _setup(engine)
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
    carry = {k: np.zeros(N) for k in ("ms", "adopt", "mv", "skc", "bkw", "bkwh")}
    for y in YEARS:
        r = loop.run_year(y, keep_per_agent=True)
        o = {k: h(loop.out[k]) for k in ("payback_period", "system_kw", "batt_kw", "batt_kwh")}
        assert (h(loop.out["status"]) == 0).all()
        capex = pop.cols["capex"] * (1.0 - 0.02) ** (y - YEARS[0])
        _, _, mms = od.max_market_share(o["payback_period"], sec_s, m["sector_abbr"].tolist(),
                                        m["payback_period"].to_numpy(), m["max_market_share"].to_numpy(),
                                        m["payback_period"].to_numpy())
        got_mms = h(r.per_agent["max_market_share"])
        assert np.array_equal(got_mms, mms, equal_nan=True), y
        d = od.diffusion(mms, carry["ms"], p, q, t1, ag["developable_agent_weight"], o["system_kw"],
                         capex, carry["adopt"], carry["mv"], carry["skc"], y == YEARS[0])
        for k in ("market_share", "new_adopters", "number_of_adopters", "market_value", "system_kw_cum"):
            assert np.allclose(h(r.per_agent[k]), d[k], rtol=1e-12, atol=1e-12), (y, k)
        att = oa.allocate([STATES[s] for s in st], sec_s, ag["agent_id"], h(r.per_agent["new_adopters"]),
                          tabs.attach_rate[st], o["batt_kw"], o["batt_kwh"], carry["bkw"], carry["bkwh"])
        assert np.array_equal(h(r.per_agent["added"]), att["batt_adopters_added_this_year"]), y
        assert np.allclose(h(r.per_agent["batt_kw_cum"]), att["batt_kw_cum"], rtol=1e-12, atol=1e-12)
        # per-state hourly export from the loop's own planes (caller order)
        w = oa.weights(ag["customers_in_bin"], h(r.per_agent["number_of_adopters"]), carry["bkw"],
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
    *_, whole = _setup(engine)
    *_, chunked = _setup(engine, hourly_chunk=1000)
    for y in YEARS[:2]:
        a, b = whole.run_year(y), chunked.run_year(y)
        assert torch.equal(a.totals, b.totals), y
        assert torch.allclose(a.hourly, b.hourly, rtol=1e-12, atol=1e-9), y
