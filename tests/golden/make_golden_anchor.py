"""Generate tests/golden/anchor.json: the reference's calc_diffusion_solar in
its historical anchor years (diffusion_functions_elec.py:99-133), where the PV
cumulative capacity of each (state, sector, year) is rescaled to the observed
deployment table (config.OBSERVED_DEPLOYMENT_BY_STATE).

Run IN THE BUILD CONTAINER ONLY (reads /root/reference):
    python tests/golden/make_golden_anchor.py

Inputs: make_golden.diffusion_inputs (states DE/CA/NY/TX and ZZ, which the
observed table lacks -> NaN rows) with a 'year' column, plus one (state,
sector) group whose cumulative capacity is all zero (the 1 / agent_count
branch).  The observed table rows the frame can hit are stored beside the
outputs, so the test needs nothing from /root/reference.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402

OBSERVED = "/root/reference/dgen_os/input_data/observed_deployment_by_state_sector_2020.csv"


def main():
    ff, _ = mg.install_stubs()
    import config
    import diffusion_functions_elec as dfe
    # config.py builds the path from the working directory's parent; point it
    # at the reference's own file
    config.OBSERVED_DEPLOYMENT_BY_STATE = OBSERVED
    rng = np.random.default_rng(20260014)
    df, mms_df, bass = mg.diffusion_inputs(rng, n=300)
    zero = (df["state_abbr"] == "DE") & (df["sector_abbr"] == "ind")
    df.loc[zero, "system_kw_cum_last_year"] = 0.0
    df.loc[zero, "system_kw"] = 0.0
    out_mms = ff.calc_max_market_share(df, mms_df)
    d2 = out_mms.copy()
    d2.index = df.index
    obs = pd.read_csv(OBSERVED)
    res = {}
    for year, first in ((2014, True), (2016, False), (2018, False)):
        d3 = d2.copy()
        d3["year"] = year
        out, mly = dfe.calc_diffusion_solar(d3, first, bass, year)
        res[str(year)] = {"first": first, "columns": list(out.columns),
                          "df": out.to_dict(orient="list"),
                          "mly_columns": list(mly.columns),
                          "market_last_year": mly.to_dict(orient="list")}
    keep = obs[obs["state_abbr"].isin(df["state_abbr"].unique())]
    fix = {"inputs": df.reset_index().to_dict(orient="list"),
           "mms_df": mms_df.to_dict(orient="list"), "bass": bass.to_dict(orient="list"),
           "observed": keep.to_dict(orient="list"), "observed_columns": list(obs.columns),
           "years": res}
    with open(os.path.join(HERE, "anchor.json"), "w") as f:
        json.dump(mg._jsonable(fix), f)
    for y, r in res.items():
        kw = np.asarray(r["df"]["system_kw_cum"], dtype=float)
        print(y, "rows", len(kw), "nan", int(np.isnan(kw).sum()), "sum", np.nansum(kw))


if __name__ == "__main__":
    main()
