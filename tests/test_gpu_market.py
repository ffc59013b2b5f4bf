"""Device per-year attribute gathers (dgen_year_inputs) and first-year market
seeding (dgen_initial_market_shares) against the reference's own outputs
(tests/golden/market.json): bit-exact."""
import numpy as np
import pytest
import torch

from dgen_amd.market import YEAR_OUT_F64, YearInputs, YearTables, initial_market_shares
from tests import helpers

pytestmark = pytest.mark.gpu


def _same(a, b):
    return np.array_equal(np.asarray(a, np.float64), np.asarray(b, np.float64), equal_nan=True)


def test_year_inputs_gather_matches_reference(engine):
    m = helpers.golden_market()
    ag = m["agents"]
    n = len(ag)
    yt = YearTables(ag, m["tables"], m["inflation_rate"])
    yi = YearInputs(engine, yt, ag["load_kwh_per_customer_in_bin_initial"].to_numpy(),
                    ag["customers_in_bin_initial"].to_numpy(), ag["load_kwh_in_bin_initial"].to_numpy())
    dev = engine.dev
    cols = {k: torch.full((n,), -7.0, dtype=torch.float64, device=dev) for k in YEAR_OUT_F64}
    cols.update({k: torch.full((n,), -7, dtype=torch.int32, device=dev)
                 for k in ("econ_life", "loan_term", "wholesale_row")})
    loop = {k: torch.empty(n, dtype=torch.float64, device=dev) for k in ("customers_in_bin", "load_kwh_in_bin")}
    for rec in m["years"]:
        yi.apply(rec["year"], cols, loop)
        torch.cuda.synchronize()
        got = {k: v.cpu().numpy() for k, v in {**cols, **loop}.items()}
        for ref_name, ours in helpers.MARKET_COLS.items():
            g = got[ours]
            if g.dtype.kind == "i":
                g = np.where(g < 0, np.nan, g)
            assert _same(g, rec["columns"][ref_name]), (rec["year"], ref_name)


def test_initial_market_shares_device_matches_reference(engine):
    m = helpers.golden_market()
    ag = m["agents"]
    rec = m["years"][0]
    ini = rec["initial"]
    dev = engine.dev
    w = torch.as_tensor(rec["columns"]["developable_agent_weight"], device=dev)
    capex = torch.as_tensor(rec["columns"]["system_capex_per_kw"], device=dev)
    import pandas as pd
    out = initial_market_shares(engine, ag["state_abbr"].tolist(), ag["sector_abbr"].tolist(),
                                ag["tech"].tolist(), w, capex, pd.DataFrame(ini["caps"]))
    for k, ref in ini["columns"].items():
        assert _same(out[k].cpu().numpy(), ref), k
    # per-group developable customers: pandas' group sum exactly
    df = pd.DataFrame({"s": ag["state_abbr"], "c": ag["sector_abbr"], "t": ag["tech"],
                       "w": rec["columns"]["developable_agent_weight"]})
    ref = df.groupby(["s", "c", "t"])["w"].sum()
    dc = out["developable_customers_in_state"].cpu().numpy()
    for g, key in enumerate(out["groups"]):
        assert dc[g] == ref.loc[key], key
