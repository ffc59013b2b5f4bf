"""Device diffusion step via the drop-in functions vs the reference's own
outputs (tests/golden/diffusion.json).  Lookup / index work bit-exact; the
log / pow arithmetic within 1e-12 relative (device libm vs glibc)."""
import json
import os

import numpy as np
import pandas as pd
import pytest

from dgen_amd import diffusion as gd
from tests.helpers import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(GOLDEN, "diffusion.json")) as f:
        return json.load(f)


def test_max_market_share_device(gold, engine):
    inp = pd.DataFrame(gold["inputs"]).set_index("agent_id")
    mdf = pd.DataFrame(gold["mms_df"])
    out = gd.calc_max_market_share(inp, mdf, engine=engine)
    assert list(out.columns) == gold["mms_out"]["columns"]
    assert np.array_equal(out["max_market_share"].to_numpy(float),
                          np.array(gold["mms_out"]["max_market_share"], float), equal_nan=True)


@pytest.mark.parametrize("phase", ["first", "later"])
def test_diffusion_device(gold, engine, phase):
    inp = pd.DataFrame(gold["inputs"]).set_index("agent_id")
    inp["max_market_share"] = gold["mms_out"]["max_market_share"]
    inp["metric"] = "payback_period"
    bass = pd.DataFrame(gold["bass"])
    df, mly = gd.calc_diffusion_solar(inp, phase == "first", bass, 2026 if phase == "first" else 2027,
                                      engine=engine)
    g = gold["diffusion"][phase]
    assert list(df.columns) == g["columns"]
    assert list(mly.columns) == g["mly_columns"]
    ref = pd.DataFrame(g["df"])
    for k in gd.DIFF_OUT + ["new_batt_kw", "batt_kw_cum"]:
        a, b = df[k].to_numpy(float), ref[k].to_numpy(float)
        assert np.allclose(a, b, rtol=1e-12, atol=1e-300, equal_nan=True), k


@pytest.mark.parametrize("year", [2014, 2016, 2018])
def test_anchor_years_device(engine, year):
    """Anchor years through the drop-in (device diffusion + device group sums)
    vs the reference's calc_diffusion_solar output (tests/golden/anchor.json):
    same columns and order, values within 1e-12 (device fixed-order sums vs
    pandas' Kahan group sums)."""
    with open(os.path.join(GOLDEN, "anchor.json")) as f:
        g = json.load(f)
    y = g["years"][str(year)]
    inp = pd.DataFrame(g["inputs"]).set_index("agent_id")
    mdf = pd.DataFrame(g["mms_df"])
    d2 = gd.calc_max_market_share(inp, mdf, engine=engine)
    d2.index = inp.index
    d2["year"] = year
    obs = pd.DataFrame(g["observed"])[g["observed_columns"]]
    df, mly = gd.calc_diffusion_solar(d2, y["first"], pd.DataFrame(g["bass"]), year, engine=engine,
                                      observed_deployment=obs)
    assert list(df.columns) == y["columns"]
    assert list(mly.columns) == y["mly_columns"]
    ref = pd.DataFrame(y["df"])
    for k in ("system_kw_cum", "number_of_adopters", "market_share", "observed_storage_mw",
              "new_system_kw", "market_value"):
        a, b = df[k].to_numpy(float), ref[k].to_numpy(float)
        assert np.allclose(a, b, rtol=1e-12, atol=1e-300, equal_nan=True), k
    rm = pd.DataFrame(y["market_last_year"])
    assert np.allclose(mly["system_kw_cum_last_year"].to_numpy(float),
                       rm["system_kw_cum_last_year"].to_numpy(float), rtol=1e-12, equal_nan=True)
    with pytest.raises(FileNotFoundError):
        gd.calc_diffusion_solar(d2, y["first"], pd.DataFrame(g["bass"]), year, engine=engine)
