"""Per-year attribute merges (elec.apply_*) and first-year market seeding
(elec.estimate_initial_market_shares): the host table compile + gather
restatement and the CPU oracle against the reference's own outputs
(tests/golden/market.json, make_golden_market.py).  Bit-exact."""
import numpy as np
import pandas as pd
import pytest

from dgen_amd.market import YearTables
from oracle import market as om
from tests import helpers


def _same(a, b):
    return np.array_equal(np.asarray(a, np.float64), np.asarray(b, np.float64), equal_nan=True)


def test_year_gather_matches_reference_merges():
    m = helpers.golden_market()
    ag = m["agents"]
    yt = YearTables(ag, m["tables"], m["inflation_rate"])
    for rec in m["years"]:
        y = rec["year"]
        got = yt.gather_host(y, ag["load_kwh_per_customer_in_bin_initial"].to_numpy(),
                             ag["customers_in_bin_initial"].to_numpy(), ag["load_kwh_in_bin_initial"].to_numpy())
        for ref_name, ours in helpers.MARKET_COLS.items():
            ref = rec["columns"][ref_name]
            g = got[ours]
            if g.dtype.kind == "i":               # merge miss: NaN there, -1 here
                g = np.where(g < 0, np.nan, g)
            assert _same(g, ref), (y, ref_name)
        assert _same(got["customers_in_bin"], rec["columns"]["developable_agent_weight"]), y


def test_escalator_year_cap_and_clip():
    """After 2040 the escalator is frozen at the 2040 CAGR (year_cap) and every
    value is clipped to [-0.01, 0.01] (elec.py:64-73)."""
    m = helpers.golden_market()
    by_year = {r["year"]: r["columns"]["elec_price_escalator"] for r in m["years"]}
    assert _same(by_year[2042], by_year[2050]) and _same(by_year[2044], by_year[2046])
    assert all(np.nanmax(np.abs(v)) <= 0.01 for v in by_year.values())


def test_duplicate_table_keys_are_refused():
    m = helpers.golden_market()
    t = dict(m["tables"])
    t["pv_tech"] = pd.concat([t["pv_tech"], t["pv_tech"].iloc[:1]])
    yt = YearTables(m["agents"], t, 0.025)
    with pytest.raises(ValueError, match="more than once"):
        yt.compile(2026)


def test_initial_market_shares_oracle_matches_reference():
    m = helpers.golden_market()
    ag = m["agents"]
    rec = m["years"][0]
    ini = rec["initial"]
    w = rec["columns"]["developable_agent_weight"]
    capex = rec["columns"]["system_capex_per_kw"]
    got = om.initial_market_shares(ag["state_abbr"].tolist(), ag["sector_abbr"].tolist(), ag["tech"].tolist(),
                                   w, capex, ini["caps"])
    for k, ref in ini["columns"].items():
        assert _same(got[k], ref), k
    # the fixture covers the branches: a zero-developable group, zero-weight
    # agents, a state with no starting-capacity row
    assert (w == 0).any() and (ini["columns"]["market_share_last_year"] == 0).any()


def test_kahan_group_sum_is_pandas():
    rng = np.random.default_rng(3)
    v = rng.lognormal(0, 3, 5000)
    v[::97] = np.nan
    df = pd.DataFrame({"g": rng.integers(0, 7, v.size), "v": v})
    ref = df.groupby("g")["v"].sum()
    for g, s in ref.items():
        got, _ = om.group_sum_kahan(df.loc[df.g == g, "v"].tolist())
        assert got == s, g


def test_financing_max_years_follows_the_year_and_rejects_misses():
    """The per-year lifetimes pick the sizing kernels' lanes-per-agent form, so
    the loop refreshes the batch maximum every year and refuses a merge miss
    (NaN) or a lifetime outside [1, MAXY]."""
    from dgen_amd.market import financing_max_years
    from dgen_amd.year_loop import LoopTables
    tabs = LoopTables.synthetic()
    fin = tabs.inputs["financing"].copy()
    fin.loc[(fin["year"] == 2027) & (fin["sector_abbr"] == "com"), "economic_lifetime_yrs"] = 40
    t = dict(tabs.inputs, financing=fin)
    frame = pd.DataFrame({"state_abbr": ["DE", "DE", "CA"], "sector_abbr": ["res", "com", "com"],
                          "county_id": [0, 1, 2]})
    yt = YearTables(frame, t, 0.025)
    assert financing_max_years(yt.compile(2026)["by_sector"], yt.k_sector, 2026) == 25
    assert financing_max_years(yt.compile(2027)["by_sector"], yt.k_sector, 2027) == 40
    res_only = [k for k, s in zip(yt.k_sector, frame["sector_abbr"]) if s == "res"]
    assert financing_max_years(yt.compile(2027)["by_sector"], res_only, 2027) == 25
    bs = yt.compile(2027)["by_sector"].copy()
    bs[:, 5] = np.nan
    with pytest.raises(ValueError, match="merge miss"):
        financing_max_years(bs, yt.k_sector, 2027)
    bs = yt.compile(2027)["by_sector"].copy()
    bs[:, 5] = 51
    with pytest.raises(ValueError, match="outside"):
        financing_max_years(bs, yt.k_sector, 2027)
