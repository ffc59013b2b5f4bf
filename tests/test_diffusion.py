"""Diffusion step: numpy oracle and host table builder vs the
reference's calc_max_market_share / calc_diffusion_solar (tests/golden/diffusion.json)."""
import json
import os

import numpy as np
import pandas as pd
import pytest

from dgen_amd.diffusion import mms_table
from oracle import diffusion as od
from tests.helpers import GOLDEN


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(GOLDEN, "diffusion.json")) as f:
        return json.load(f)


def _mms(gold):
    inp = pd.DataFrame(gold["inputs"])
    mdf = pd.DataFrame(gold["mms_df"])
    sel = (mdf.metric == "payback_period") & (mdf.business_model == "host_owned")
    allpb = mdf.loc[mdf.metric == "payback_period", "payback_period"].to_numpy(float)
    return inp, mdf, od.max_market_share(inp.payback_period.to_numpy(float), inp.sector_abbr,
                                         mdf.sector_abbr[sel], mdf.payback_period[sel],
                                         mdf.max_market_share[sel], allpb)


def test_oracle_max_market_share(gold):
    inp, mdf, (bounded, factor, mms) = _mms(gold)
    ref = np.array(gold["mms_out"]["max_market_share"], dtype=float)
    assert np.array_equal(mms, ref, equal_nan=True)


def test_host_mms_table_matches_merge(gold):
    inp, mdf, (bounded, factor, mms) = _mms(gold)
    tab, rows, fmin, min_pb, max_pb = mms_table(mdf)
    got = []
    for s, f in zip(inp.sector_abbr, factor):
        r = rows.get(s, -1)
        k = int(f) - fmin
        got.append(tab[r, k] if r >= 0 and 0 <= k < tab.shape[1] else np.nan)
    assert np.array_equal(np.array(got), np.array(gold["mms_out"]["max_market_share"], float),
                          equal_nan=True)


@pytest.mark.parametrize("phase", ["first", "later"])
def test_oracle_diffusion(gold, phase):
    g = gold["diffusion"][phase]
    d = pd.DataFrame(g["df"])
    o = od.diffusion(d.max_market_share.to_numpy(float), d.market_share_last_year.to_numpy(float),
                     d.bass_param_p.to_numpy(float), d.bass_param_q.to_numpy(float),
                     d.teq_yr1.to_numpy(float), d.developable_agent_weight.to_numpy(float),
                     d.system_kw.to_numpy(float), d.system_capex_per_kw.to_numpy(float),
                     d.adopters_cum_last_year.to_numpy(float), d.market_value_last_year.to_numpy(float),
                     d.system_kw_cum_last_year.to_numpy(float), phase == "first")
    for k, v in o.items():
        assert np.array_equal(v, d[k].to_numpy(float), equal_nan=True), k
    assert g["columns"][-3:] == ["system_kw_cum", "batt_kw_cum", "batt_kwh_cum"]


@pytest.fixture(scope="module")
def anchor_gold():
    with open(os.path.join(GOLDEN, "anchor.json")) as f:
        return json.load(f)


def _observed_map(g):
    o = g["observed"]
    return {(s, c, int(y)): float(mw) for s, c, y, mw in
            zip(o["state_abbr"], o["sector_abbr"], o["year"], o["observed_solar_mw"])}


@pytest.mark.parametrize("year", ["2014", "2016", "2018"])
def test_oracle_anchor_years(anchor_gold, year):
    """Anchor-year rescale (diffusion_functions_elec.py:99-133) against the
    reference's own output: pre-anchor cumulative = last year + new capacity,
    Kahan group totals, observed MW -> bit-exact."""
    r = pd.DataFrame(anchor_gold["years"][year]["df"])
    pre = r["system_kw_cum_last_year"].to_numpy(float) + r["new_system_kw"].to_numpy(float)
    cum, ad, ms = od.anchor(r["state_abbr"].tolist(), r["sector_abbr"].tolist(), r["year"].tolist(),
                            r["developable_agent_weight"].to_numpy(float), pre,
                            _observed_map(anchor_gold))
    assert np.array_equal(cum, r["system_kw_cum"].to_numpy(float), equal_nan=True)
    assert np.array_equal(ad, r["number_of_adopters"].to_numpy(float), equal_nan=True)
    assert np.array_equal(ms, r["market_share"].to_numpy(float), equal_nan=True)
    # the fixture covers the NaN (state without observed rows) and all-zero-group branches
    assert np.isnan(cum).any() and np.isfinite(cum).any()
    zero = (r["state_abbr"] == "DE") & (r["sector_abbr"] == "ind")
    assert zero.any() and np.all(pre[zero.to_numpy()] == 0.0)
