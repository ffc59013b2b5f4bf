"""CPU oracle for the first-year market seeding (TEST INFRASTRUCTURE ONLY:
imported by tests/ as the checker; the product never imports it).

Restates agent_mutation/elec.py:701-765 estimate_initial_market_shares in
plain Python/numpy: pandas' group_sum (pandas/_libs/groupby.pyx: Kahan
compensation in row order, NaN skipped and not counted, a NaN compensation
reset to 0) per (state_abbr, sector_abbr, tech) group, the merge of the state
starting capacities on (state_abbr, sector_abbr), the per-agent portions and
fillna(0).  Pinned by tests/golden/market.json (the reference run itself).
"""
from __future__ import annotations

import math
from typing import Dict, Sequence

import numpy as np

CAP_COLS = ["system_mw", "batt_mw", "batt_mwh", "pv_systems_count", "batt_systems_count"]


def group_sum_kahan(values: Sequence[float]):
    s = c = 0.0
    n = 0
    for v in values:
        if v != v:
            continue
        n += 1
        y = v - c
        t = s + y
        c = (t - s) - y
        if c != c:
            c = 0.0
        s = t
    return s, n


def initial_market_shares(state, sector, tech, weight, capex, caps: Dict) -> Dict[str, np.ndarray]:
    n = len(state)
    groups: Dict = {}
    for i in range(n):
        groups.setdefault((state[i], sector[i], tech[i]), []).append(i)
    capmap = {}
    for r in range(len(caps["state_abbr"])):
        capmap[(caps["state_abbr"][r], caps["sector_abbr"][r])] = [float(caps[c][r]) for c in CAP_COLS]
    out = {k: np.zeros(n) for k in ("adopters_cum_last_year", "system_kw_cum_last_year", "batt_kw_cum_last_year",
                                     "batt_kwh_cum_last_year", "market_share_last_year",
                                     "market_value_last_year")}
    z = lambda v: 0.0 if v != v else v
    for key, rows in groups.items():
        dev, cnt = group_sum_kahan([weight[i] for i in rows])
        sys_mw, batt_mw, batt_mwh, pv_n, _ = capmap.get((key[0], key[1]), [math.nan] * 5)
        for i in rows:
            w = weight[i]
            with np.errstate(all="ignore"):
                portion = w / dev if dev > 0 else 1.0 / cnt
                adopt = portion * pv_n
                skc = (portion * sys_mw) * 1000.
                bkw = (portion * batt_mw) * 1000.0
                bkwh = (portion * batt_mwh) * 1000.0
                ms = 0.0 if w == 0 else adopt / w
                mv = capex[i] * skc
            out["adopters_cum_last_year"][i] = z(adopt)
            out["system_kw_cum_last_year"][i] = z(skc)
            out["batt_kw_cum_last_year"][i] = z(bkw)
            out["batt_kwh_cum_last_year"][i] = z(bkwh)
            out["market_share_last_year"][i] = z(ms)
            out["market_value_last_year"][i] = z(mv)
    out["initial_number_of_adopters"] = out["adopters_cum_last_year"].copy()
    out["initial_pv_kw"] = out["system_kw_cum_last_year"].copy()
    out["initial_batt_kw"] = out["batt_kw_cum_last_year"].copy()
    out["initial_batt_kwh"] = out["batt_kwh_cum_last_year"].copy()
    out["initial_market_share"] = out["market_share_last_year"].copy()
    out["initial_market_value"] = np.zeros(n)
    return out
