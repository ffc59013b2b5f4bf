"""CPU restatement of the reference's battery-attachment allocation and per-state
hourly export.

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker for the device
kernels k_batt_attach / k_state_hourly.  The product package never imports it.
Pinned by tests/golden/attach.json (the reference's own functions run on
synthetic frames, tests/golden/make_golden_attach.py).

  allocate()  attachment_rate_functions.py:58-138  _allocate_battery_adopters_integer
  export()    attachment_rate_functions.py:141-206 export_state_hourly_with_storage_mix
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np


def _groups(keys: Sequence) -> Dict:
    """First-appearance order of keys -> row indices (pandas groupby sort=False)."""
    out: Dict = {}
    for i, k in enumerate(keys):
        out.setdefault(k, []).append(i)
    return out


def allocate(state, sector, agent_id, new_adopters, rate, batt_kw, batt_kwh,
             batt_kw_cum_last_year, batt_kwh_cum_last_year) -> Dict[str, np.ndarray]:
    """Largest-remainder integer battery adopters per state x sector
    (attachment_rate_functions.py:105-129), then capacities (:133-136)."""
    n_all = len(state)
    new = np.asarray(new_adopters, dtype=np.float64)
    alloc = np.zeros(n_all, dtype=np.int64)
    for (_, _), idx in _groups(list(zip(state, sector))).items():
        idx = np.asarray(idx)
        r = float(rate[idx[0]])                          # :108
        r = max(0.0, min(1.0, r))                        # :109
        n = new[idx]
        if n.sum() <= 0 or r <= 0:                       # :112
            continue
        target = int(round(r * n.sum()))                 # :116 (round half to even)
        f = r * n                                        # :119
        base = np.floor(f).astype(np.int64)
        rem = target - base.sum()                        # :121
        if rem > 0:
            frac = f - base
            aid = [str(agent_id[i]) for i in idx]
            # sort by frac desc, then agent_id string asc (:125-128); take rem
            order = sorted(range(len(idx)), key=lambda k: (-frac[k], aid[k]))
            base = base.copy()
            base[np.asarray(order[:rem], dtype=np.int64)] += 1
        alloc[idx] = base
    bkw = np.asarray(batt_kw, dtype=np.float64)
    bkwh = np.asarray(batt_kwh, dtype=np.float64)
    new_kw = alloc * bkw
    new_kwh = alloc * bkwh
    return {"batt_adopters_added_this_year": alloc, "new_batt_kw": new_kw, "new_batt_kwh": new_kwh,
            "batt_kw_cum": np.asarray(batt_kw_cum_last_year, dtype=np.float64) + new_kw,
            "batt_kwh_cum": np.asarray(batt_kwh_cum_last_year, dtype=np.float64) + new_kwh}


def weights(customers_in_bin, number_of_adopters, batt_kw_cum_last_year, batt_kw, added):
    """Per-agent (pvo_cum, batt_cum, n_non) multipliers of the export
    (attachment_rate_functions.py:181-190)."""
    eps = 1e-9
    n = len(customers_in_bin)
    w = np.zeros((3, n), dtype=np.float64)
    for i in range(n):
        n_cust = float(customers_in_bin[i])
        n_adopt = float(number_of_adopters[i])
        n_non = max(n_cust - n_adopt, 0.0)
        prev = float(batt_kw_cum_last_year[i]) / max(float(batt_kw[i]) or eps, eps)
        prev = int(round(max(prev, 0.0)))
        batt_cum = max(prev + int(added[i]), 0)
        pvo_cum = max(int(round(n_adopt)) - batt_cum, 0)
        w[0, i], w[1, i], w[2, i] = pvo_cum, batt_cum, n_non
    return w


def export(state, baseline, pvonly, with_batt, w) -> Dict[str, List]:
    """Per-state hourly net sums in MW, states in first-appearance order
    (attachment_rate_functions.py:156-198).  baseline / pvonly / with_batt:
    [n_agents, n_hours]; w from weights()."""
    states, sums = [], []
    for s, idx in _groups(list(state)).items():
        acc = np.zeros(baseline.shape[1], dtype=np.float64)
        for i in idx:                                    # :179 iterrows order
            acc += (pvonly[i] * w[0, i]) + (with_batt[i] * w[1, i]) + (baseline[i] * w[2, i])
        states.append(s)
        sums.append(acc / 1000.0)
    return {"state_abbr": states, "net_sum": sums}
