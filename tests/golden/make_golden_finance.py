"""Generate tests/golden/finance_series.json: the reference's own
finance_series_export.export_agent_finance_series on synthetic agent frames.

Run IN THE BUILD CONTAINER ONLY (reads /root/reference):
    python tests/golden/make_golden_finance.py

Functions exercised (reference code, run unmodified):
  finance_series_export._norm25                       :9-20
  finance_series_export.export_agent_finance_series   :22-81
input_data_functions (DB) is replaced by a stub whose df_to_psql records the
frame it is handed; sqlalchemy (not installed) by a stub module exposing
Engine (a type annotation only).  Inputs are stored as JSON with non-finite
floats spelled as strings ("nan", "inf", "-inf").
"""
from __future__ import annotations

import json
import math
import os
import sys
import types

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/dgen_os/python"


def load_ref():
    captured = []
    idf = types.ModuleType("input_data_functions")

    def df_to_psql(df, engine, schema, owner, name, if_exists="replace", append_transformations=False):
        captured.append({"name": name, "if_exists": if_exists, "records": df.to_dict(orient="records")})

    idf.df_to_psql = df_to_psql
    sys.modules["input_data_functions"] = idf
    sa = types.ModuleType("sqlalchemy")
    sae = types.ModuleType("sqlalchemy.engine")
    sae.Engine = object
    sa.engine = sae
    sys.modules.setdefault("sqlalchemy", sa)
    sys.modules.setdefault("sqlalchemy.engine", sae)
    sys.path.insert(0, REF)
    import finance_series_export as fse  # noqa
    return fse, captured


def enc(v):
    """JSON-safe cell: lists/arrays -> {"list"/"array": [...]} with non-finite as strings."""
    f = lambda x: x if (isinstance(x, float) and math.isfinite(x)) or isinstance(x, int) else str(x)
    if isinstance(v, np.ndarray):
        return {"array": [f(float(x)) for x in v.tolist()]}
    if isinstance(v, (list, tuple)):
        return {"list": [f(float(x)) if isinstance(x, (int, float, np.floating)) else x for x in v]}
    if isinstance(v, float):
        return {"scalar": f(v)}
    return {"scalar": v}


def frame(rng):
    rows = []
    cols = ["cf_energy_value_pv_only", "utility_bill_w_sys_pv_only", "utility_bill_wo_sys_pv_only",
            "cf_energy_value_pv_batt", "utility_bill_w_sys_pv_batt", "utility_bill_wo_sys_pv_batt"]
    for k in range(40):
        n1 = [26, 26, 26, 21, 31, 10, 51, 26][k % 8]
        r = {"agent_id": int(1000 + 7 * k)}
        for c in cols:
            v = list(rng.normal(500, 300, n1))
            if k % 5 == 1:
                v[3] = float("nan")
            if k % 7 == 2:
                v[min(24, n1 - 1)] = float("inf")
                v[0] = float("-inf")
            r[c] = v
        if k % 9 == 4:                       # pv_batt lists absent: scalars -> no pv_batt row
            for c in cols[3:]:
                r[c] = float("nan")
        if k % 11 == 5:                      # numpy arrays do not count as lists (isinstance)
            for c in cols[:3]:
                r[c] = np.asarray(r[c])
        if k % 13 == 6:                      # one list column is enough; others zero-filled
            r[cols[1]] = float("nan")
            r[cols[2]] = "n/a"
        rows.append(r)
    return pd.DataFrame(rows)


def main():
    fse, captured = load_ref()
    rng = np.random.default_rng(20260008)
    df = frame(rng)
    cases = []
    for name, d in (("columns", df), ("index_agent_id", df.set_index("agent_id"))):
        captured.clear()
        fse.export_agent_finance_series(None, "s", "o", 2027, d)
        cases.append({"name": name, "index_agent_id": name == "index_agent_id",
                      "rows": [{k: enc(v) for k, v in r.items()} for r in df.to_dict(orient="records")],
                      "table": captured[0]["name"], "if_exists": captured[0]["if_exists"],
                      "records": captured[0]["records"]})
    # no finance columns at all -> nothing written
    captured.clear()
    fse.export_agent_finance_series(None, "s", "o", 2027, df[["agent_id"]])
    cases.append({"name": "no_columns", "rows": [{"agent_id": {"scalar": int(a)}} for a in df.agent_id],
                  "index_agent_id": False, "records": None if not captured else captured[0]["records"]})
    with open(os.path.join(HERE, "finance_series.json"), "w") as f:
        json.dump({"year": 2027, "cases": cases}, f)
    for c in cases:
        print(c["name"], 0 if c["records"] is None else len(c["records"]), "records")


if __name__ == "__main__":
    main()
