"""Generate tests/golden/attach.json: the reference's own battery-attachment
allocation and per-state hourly export on synthetic post-diffusion frames.

Run IN THE BUILD CONTAINER ONLY (reads /root/reference):
    python tests/golden/make_golden_attach.py
Outputs: attach.json (inputs, allocation, export records) and attach.npz
(the f32 hourly planes fed to the export).

Functions exercised (reference code, run unmodified):
  attachment_rate_functions._allocate_battery_adopters_integer   :58-138
  attachment_rate_functions.export_state_hourly_with_storage_mix :141-206
The module's only import that needs a database, input_data_functions, is
replaced by a stub whose df_to_psql records the frame it is handed (the
records the reference would write to state_hourly_agg).  Hourly arrays are
96 h long here (the export is length-agnostic); full 8760-h sizes are tested
against the oracle restatement (oracle/attach.py).
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/dgen_os/python"
NHX = 96
HOURLY = {}


def load_ref():
    captured = []
    fake = types.ModuleType("input_data_functions")

    def df_to_psql(df, engine, schema, owner, name, if_exists="replace", append_transformations=False):
        captured.append({"name": name, "records": df.to_dict(orient="list")})

    fake.df_to_psql = df_to_psql
    sys.modules["input_data_functions"] = fake
    sys.path.insert(0, REF)
    import attachment_rate_functions as arf  # noqa
    return arf, captured


def frame(rng, n, states, sectors, *, ties=False, ids=None):
    st = rng.choice(states, n)
    sec = rng.choice(sectors, n)
    new = rng.uniform(0, 4, n) * (rng.random(n) < 0.85)
    if ties:
        new[: n // 3] = 1.25               # identical fractional parts -> agent_id tie-break
    n_adopt = new + rng.uniform(0, 30, n)
    batt_kw = np.where(rng.random(n) < 0.1, 0.0, rng.uniform(2, 40, n))
    batt_kwh = batt_kw * 2.0
    prev = np.round(rng.uniform(0, 6, n)) * batt_kw + rng.uniform(-0.3, 0.3, n) * (batt_kw > 0)
    prev = np.maximum(prev, 0.0)
    ids = np.arange(n) * 7 + 3 if ids is None else ids
    rate = {s: float(v) for s, v in zip(states, rng.uniform(0, 0.6, len(states)))}
    rate[states[0]] = 0.0                  # a state with no storage attachment
    df = pd.DataFrame({
        "agent_id": ids, "state_abbr": st, "sector_abbr": sec,
        "new_adopters": new, "number_of_adopters": n_adopt,
        "batt_kw": batt_kw, "batt_kwh": batt_kwh,
        "batt_kw_cum_last_year": prev, "batt_kwh_cum_last_year": prev * 2.0,
        "storage_attachment_rate": [rate[s] for s in st],
        "customers_in_bin": n_adopt + rng.uniform(-5, 200, n),
    })
    # one group whose new adopters are all zero (n.sum() <= 0 branch)
    g0 = (df.state_abbr == states[1]) & (df.sector_abbr == sectors[0])
    df.loc[g0, "new_adopters"] = 0.0
    return df.set_index("agent_id", drop=False)


def hourly(rng, n):
    f32 = lambda a: a.astype(np.float32).astype(np.float64)  # the device planes are f32
    base = f32(rng.uniform(0.2, 3.0, (n, NHX)))
    pvo = f32(np.maximum(base - rng.uniform(0, 3.0, (n, NHX)), 0.0))
    wbt = f32(np.maximum(pvo - rng.uniform(0, 1.0, (n, NHX)), 0.0))
    return base, pvo, wbt


def case(arf, captured, rng, name, n, states, sectors, **kw):
    df = frame(rng, n, states, sectors, **kw)
    out = arf._allocate_battery_adopters_integer(df, 2027)
    base, pvo, wbt = hourly(rng, n)
    out = out.copy()
    out["baseline_net_hourly"] = list(base)
    out["adopter_net_hourly_pvonly"] = list(pvo)
    out["adopter_net_hourly_with_batt"] = list(wbt)
    captured.clear()
    arf.export_state_hourly_with_storage_mix(None, "s", "o", 2027, out)
    rec = captured[0]["records"] if captured else {"state_abbr": [], "net_sum": []}
    cols = ["agent_id", "state_abbr", "sector_abbr", "new_adopters", "number_of_adopters", "batt_kw",
            "batt_kwh", "batt_kw_cum_last_year", "batt_kwh_cum_last_year", "storage_attachment_rate",
            "customers_in_bin"]
    HOURLY[name] = (base, pvo, wbt)
    return {
        "name": name,
        "inputs": {c: df[c].tolist() for c in cols},
        "alloc": {c: out[c].tolist() for c in ["batt_adopters_added_this_year", "new_batt_kw",
                                                "new_batt_kwh", "batt_kw_cum", "batt_kwh_cum"]},
        "export": {"state_abbr": list(rec["state_abbr"]), "net_sum": [list(map(float, v)) for v in rec["net_sum"]],
                   "n_hours": [int(v) for v in rec.get("n_hours", [])]},
    }


def main():
    arf, captured = load_ref()
    rng = np.random.default_rng(20260005)
    cases = [
        case(arf, captured, rng, "mixed", 400, ["DE", "CA", "NY", "TX", "WA"], ["res", "com", "ind"]),
        case(arf, captured, rng, "ties", 240, ["MA", "AZ", "FL"], ["res", "com"], ties=True),
        # agent ids whose string order differs from numeric order (9 > 10 > 100 as strings)
        case(arf, captured, rng, "str_ids", 150, ["ZZ", "YY", "NJ", "CO"], ["res"],
             ids=np.concatenate([np.arange(1, 76), np.arange(90, 165) * 11])),
    ]
    np.savez_compressed(os.path.join(HERE, "attach.npz"),
                        **{f"{k}__{p}": v.astype(np.float32) for k, (b, q, w) in HOURLY.items()
                           for p, v in (("baseline", b), ("pvonly", q), ("with_batt", w))})
    with open(os.path.join(HERE, "attach.json"), "w") as f:
        json.dump({"n_hours": NHX, "cases": cases}, f)
    for c in cases:
        print(c["name"], "added", int(np.sum(c["alloc"]["batt_adopters_added_this_year"])),
              "states", len(c["export"]["state_abbr"]))


if __name__ == "__main__":
    main()
