"""Generate tests/golden/market.json: the reference's own per-year attribute
merges and first-year market seeding on synthetic agent frames.

Run IN THE BUILD CONTAINER ONLY (reads /root/reference):
    python tests/golden/make_golden_market.py

Functions exercised (reference code, run unmodified through the stub import of
make_golden.install_stubs):
  agent_mutation/elec.py
    apply_load_growth                         :398-411   (year, sector, county)
    apply_elec_price_multiplier_and_escalator :29-82     (sector, county; CAGR to the final year)
    apply_pv_tech_performance                 :135-158   (sector, year)
    apply_pv_prices                           :177-198   (sector, year)
    apply_pv_plus_batt_prices                 :239-280   (year, sector)
    apply_batt_prices                         :204-236   (sector, year)
    apply_value_of_resiliency                 :284-314   (state, sector)
    apply_financial_params                    :347-394   (year, sector) + ITC (year, tech, sector)
    apply_wholesale_elec_prices               :608-616   (county, year)
    calculate_developable_customers_and_load  :414-423
    estimate_initial_market_shares            :701-765   (state, sector, tech) Kahan group sums
The fixture holds every input table and frame and the columns the reference
produced; tests/test_market.py and tests/test_gpu_market.py replay them.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import install_stubs  # noqa: E402

STATES = ["DE", "CA", "NY", "TX", "AZ", "WY"]
SECTORS = ["res", "com", "ind"]
COUNTIES = list(range(101, 113))
YEARS = list(range(2026, 2051, 2))        # 2-year steps, start 2026 (config.py:18)
FIN_COLS = ["economic_lifetime_yrs", "loan_term_yrs", "loan_interest_rate", "down_payment_fraction",
            "real_discount_rate", "tax_rate"]


def tables(rng):
    yrs = list(range(2026, 2051))
    rows = []
    for y in yrs:
        for s in SECTORS:
            for c in COUNTIES:
                rows.append({"year": y, "sector_abbr": s, "county_id": c,
                             "load_multiplier": float(1.0 + 0.01 * (y - 2026) * rng.uniform(0.5, 1.5))})
    load_growth = pd.DataFrame(rows)
    rows = []
    for y in yrs:
        for s in SECTORS:
            for c in COUNTIES:
                rows.append({"year": y, "sector_abbr": s, "county_id": c,
                             "elec_price_multiplier": float(rng.uniform(0.8, 1.4) * (1 + 0.004 * (y - 2026)))})
    elec = pd.DataFrame(rows)
    pv_tech = pd.DataFrame([{"year": y, "sector_abbr": s, "pv_degradation_factor": float(rng.uniform(0.004, 0.007)),
                             "pv_power_density_w_per_sqft": 15.0 + 0.1 * (y - 2026)}
                            for y in yrs for s in SECTORS])
    pv_price = pd.DataFrame([{"year": y, "sector_abbr": s,
                              "system_capex_per_kw": float(rng.uniform(1500, 4700) * 0.98 ** (y - 2026)),
                              "system_om_per_kw": float(rng.uniform(10, 30))} for y in yrs for s in SECTORS])
    pvb_price = pd.DataFrame([{"year": y, "sector_abbr": s,
                               "system_capex_per_kw": float(rng.uniform(1400, 4500)),
                               "batt_capex_per_kwh": float(rng.uniform(190, 440) * 0.97 ** (y - 2026)),
                               "batt_capex_per_kw": float(rng.uniform(100, 300)),
                               "linear_constant": 0.0, "batt_om_per_kw": float(rng.uniform(1, 5)),
                               "batt_om_per_kwh": float(rng.uniform(0.5, 2))} for y in yrs for s in SECTORS])
    batt_price = pd.DataFrame([{"year": y, "sector_abbr": s, "batt_capex_per_kwh": float(rng.uniform(200, 500)),
                                "batt_capex_per_kw": float(rng.uniform(100, 300)), "linear_constant": 0.0,
                                "batt_om_per_kwh": 1.0, "batt_om_per_kw": 2.0} for y in yrs for s in SECTORS])
    vor = pd.DataFrame([{"state_abbr": st, "sector_abbr": s, "value_of_resiliency_usd": float(rng.uniform(0, 400))}
                        for st in STATES[:-1] for s in SECTORS])          # WY missing -> NaN
    fin = []
    for y in yrs:
        for s in SECTORS:
            fin.append({"year": y, "sector_abbr": s, "economic_lifetime_yrs": 25,
                        "loan_term_yrs": 20 if s == "res" else 30, "loan_interest_rate": float(rng.uniform(0.04, 0.08)),
                        "down_payment_fraction": 0.3 if s == "res" else 1.0,
                        "real_discount_rate": 0.05 if s == "res" else 0.0378, "tax_rate": 0.2574})
    fin = pd.DataFrame(fin)
    itc = pd.DataFrame([{"year": y, "tech": "solar", "sector_abbr": s,
                         "itc_fraction_of_capex": 0.3 if y < 2033 else (0.26 if y < 2035 else 0.1)}
                        for y in yrs for s in SECTORS])
    whl = pd.DataFrame([{"county_id": c, "year": y, "wholesale_elec_usd_per_kwh": float(rng.uniform(0.02, 0.08))}
                        for c in COUNTIES[:-1] for y in yrs])                # last county missing -> NaN
    return dict(load_growth=load_growth, elec=elec, pv_tech=pv_tech, pv_price=pv_price, pvb_price=pvb_price,
                batt_price=batt_price, vor=vor, fin=fin, itc=itc, whl=whl)


def agents(rng, n):
    st = rng.choice(STATES, n)
    sec = rng.choice(SECTORS, n, p=[0.7, 0.2, 0.1])
    cnty = rng.choice(COUNTIES, n)
    cust = np.where(sec == "res", rng.lognormal(np.log(300), 0.6, n), rng.lognormal(np.log(30), 0.8, n))
    cust[::37] = 0.0                              # agents with no developable customers
    kwh = np.where(sec == "res", rng.lognormal(np.log(9000), 0.3, n), rng.lognormal(np.log(2e5), 1.0, n))
    df = pd.DataFrame({
        "agent_id": np.arange(n) * 3 + 11, "state_abbr": st, "sector_abbr": sec, "county_id": cnty,
        "tech": "solar", "customers_in_bin_initial": cust,
        "load_kwh_per_customer_in_bin_initial": kwh, "load_kwh_in_bin_initial": kwh * cust,
    })
    # one (state, sector) group with zero developable customers (1 / agent_count branch)
    g = (df.state_abbr == "AZ") & (df.sector_abbr == "ind")
    df.loc[g, "customers_in_bin_initial"] = 0.0
    return df.set_index("agent_id")


def starting_caps(rng):
    rows = []
    for st in STATES:
        for s in SECTORS:
            if st == "WY" and s == "com":
                continue                           # merge miss -> NaN -> fillna(0)
            rows.append({"state_abbr": st, "sector_abbr": s, "system_mw": float(rng.uniform(0, 900)),
                         "batt_mw": float(rng.uniform(0, 50)), "batt_mwh": float(rng.uniform(0, 200)),
                         "pv_systems_count": float(rng.integers(0, 200000)),
                         "batt_systems_count": float(rng.integers(0, 20000))})
    return pd.DataFrame(rows)


def enc(v):
    v = np.asarray(v)
    if v.dtype.kind == "f":
        return [None if np.isnan(x) else float(x) for x in v]
    if v.dtype.kind in "iu":
        return [int(x) for x in v]
    return [str(x) for x in v]


def main():
    ff, elec = install_stubs()
    rng = np.random.default_rng(20260707)
    T = tables(rng)
    base = agents(rng, 420)
    out_years = []
    for y in YEARS:
        df = base.copy()
        df["year"] = y
        df = elec.apply_load_growth(df, T["load_growth"])
        df = elec.apply_elec_price_multiplier_and_escalator(df, y, T["elec"])
        df = elec.apply_pv_tech_performance(df, T["pv_tech"])
        df = elec.apply_pv_prices(df, T["pv_price"])
        df = elec.apply_batt_prices(df, T["batt_price"], None, y)
        df = elec.apply_pv_plus_batt_prices(df, T["pvb_price"].copy(), None, y)
        df = elec.apply_value_of_resiliency(df, T["vor"])
        df = elec.apply_wholesale_elec_prices(df, T["whl"])
        df = elec.apply_financial_params(df, T["fin"], T["itc"], 0.025)
        df = elec.calculate_developable_customers_and_load(df)
        cols = ["load_kwh_per_customer_in_bin", "customers_in_bin", "load_kwh_in_bin", "elec_price_multiplier",
                "elec_price_escalator", "pv_degradation_factor", "system_capex_per_kw",
                "system_capex_per_kw_combined", "batt_capex_per_kwh_combined", "value_of_resiliency_usd",
                "wholesale_elec_usd_per_kwh", "itc_fraction_of_capex", "inflation_rate",
                "developable_agent_weight", "developable_load_kwh_in_bin"] + FIN_COLS
        rec = {"year": y, "agent_id": enc(df.index.to_numpy()),
               "columns": {c: enc(df[c].to_numpy(dtype=np.float64)) for c in cols}}
        if y == YEARS[0]:
            caps = starting_caps(rng)
            init = elec.estimate_initial_market_shares(df.copy(), caps)
            icols = ["initial_number_of_adopters", "initial_pv_kw", "initial_batt_kw", "initial_batt_kwh",
                     "initial_market_share", "initial_market_value", "adopters_cum_last_year",
                     "system_kw_cum_last_year", "batt_kw_cum_last_year", "batt_kwh_cum_last_year",
                     "market_share_last_year", "market_value_last_year"]
            rec["initial"] = {"caps": caps.to_dict(orient="list"),
                              "agent_id": enc(init["agent_id"].to_numpy() if "agent_id" in init
                                              else init.index.to_numpy()),
                              "columns": {c: enc(init[c].to_numpy(dtype=np.float64)) for c in icols}}
        out_years.append(rec)
    meta = {
        "generator": "tests/golden/make_golden_market.py",
        "reference": "tsgsteele/dgen @ 2025-09-19, agent_mutation/elec.py",
        "agents": {c: enc(base.reset_index()[c].to_numpy()) for c in base.reset_index().columns},
        "tables": {k: v.to_dict(orient="list") for k, v in T.items()},
        "inflation_rate": 0.025,
        "years": out_years,
    }
    with open(os.path.join(HERE, "market.json"), "w") as f:
        json.dump(meta, f, separators=(",", ":"))
    print("wrote market.json:", len(out_years), "years,", len(base), "agents")


if __name__ == "__main__":
    main()
