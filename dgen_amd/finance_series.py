"""Finance-series export on the device: drop-in for

    finance_series_export.export_agent_finance_series(engine, schema, owner, year, df_agents)
                                                        finance_series_export.py:22-81
    (its helper _norm25, :9-20, is the k_finance_series kernel)

Every agent contributes a "pv_only" and a "pv_batt" record with three 25-long
series (cf_energy_value, utility_bill_w_sys, utility_bill_wo_sys): the first 25
entries of the agent's 26-long yearly list (the reference truncates), zero past
the list, non-finite entries 0.  series_from_outputs() takes them straight
from dgen_size_agents' yearly outputs on the device; the DataFrame drop-in
stages the frame's lists and runs the same kernel.  The DB append itself
(iFuncs.df_to_psql into agent_finance_series) is plumbing outside the path: it
is handed to `writer` when one is given.
"""
from __future__ import annotations

import ctypes
from typing import Callable, Dict, Optional

import numpy as np
import pandas as pd

from . import _lib
from .hourly_column import RowColumn

TABLE = "agent_finance_series"
NORM = 25
STRIDE = _lib.MAXY + 1
CASES = (("pv_only", ("cf_energy_value_pv_only", "utility_bill_w_sys_pv_only",
                      "utility_bill_wo_sys_pv_only")),
         ("pv_batt", ("cf_energy_value_pv_batt", "utility_bill_w_sys_pv_batt",
                      "utility_bill_wo_sys_pv_batt")))
SERIES = ("cf_energy_value", "utility_bill_w_sys", "utility_bill_wo_sys")
# dgen_outputs fields in the kernel's series order (include/dgen_hip.h)
OUT_FIELDS = ("cfev_pv", "bill_w_pv", "bill_wo_pv", "cfev_batt", "bill_w_batt", "bill_wo_batt")


def _engine(engine):
    if engine is not None:
        return engine
    from .financial_functions import get_engine
    return get_engine()


def _run(eng, c_out: _lib.Outputs, list_len, n: int):
    """k_finance_series -> [6, n, 25] float64 device tensor."""
    import torch
    out = torch.empty((6, n, NORM), dtype=torch.float64, device=eng.dev)
    if n == 0:
        return out
    ln = eng._to_dev(np.asarray(list_len, dtype=np.int32), torch.int32)
    _lib.check(eng.lib.dgen_finance_series(eng.ctx, ctypes.byref(c_out), ln.data_ptr(), n,
                                           out.data_ptr(), eng.stream_handle()),
               "dgen_finance_series")
    torch.cuda.current_stream(eng.dev).synchronize()
    return out


def series_from_outputs(engine, out: Dict[str, object], econ_life, perm=None) -> Dict[str, np.ndarray]:
    """The six normalised series of every sized agent, [n, 25] each, in caller
    order.  out: Engine.alloc_outputs() buffers after Engine.size(); econ_life:
    economic_lifetime_yrs in caller order; perm: AgentBatch.perm (device order)."""
    eng = _engine(engine)
    ln = np.asarray(econ_life, dtype=np.int64) + 1                       # list length N + 1
    if perm is not None:
        ln = ln[np.asarray(perm)]
    c_out = eng.c_outputs(out)
    res = _run(eng, c_out, ln, len(ln)).cpu().numpy()
    if perm is not None:
        u = np.empty_like(res)
        u[:, np.asarray(perm)] = res
        res = u
    return {f"{s}_{case}": res[3 * ci + si] for ci, (case, _) in enumerate(CASES)
            for si, s in enumerate(SERIES)}


def _as_float_list(x):
    """The values _norm25 would see (list(x) as float64), or None where the
    reference's try block falls back to zeros."""
    try:
        return np.asarray(list(x), dtype=float).ravel()
    except Exception:
        return None


def _stage_rows(col: RowColumn, dst: np.ndarray) -> None:
    """A RowColumn's cells into dst [n][STRIDE], zero past each cell's length."""
    a = col.to_2d()
    k = min(a.shape[1], STRIDE)
    dst[:, :k] = a[:, :k]
    ln = col.cell_lens()
    if (ln < k).any():
        dst[np.arange(STRIDE)[None, :] >= ln[:, None]] = 0.0


def export_agent_finance_series(engine, schema, owner, year: int, df_agents: pd.DataFrame,
                                writer: Optional[Callable] = None, dev_engine=None):
    """finance_series_export.py:22 -- one record per agent and case, returned
    as the frame the reference appends to agent_finance_series (None when the
    reference writes nothing); handed to `writer(rec, engine, schema, owner,
    "agent_finance_series", if_exists="append", append_transformations=False)`
    when given."""
    import torch
    need_any = [c for _, cols in CASES for c in cols]
    if not any(c in df_agents.columns for c in need_any):                 # :38-43
        return None
    df = df_agents
    if df.index.name == "agent_id" and "agent_id" not in df.columns:     # :45-47
        df = df.reset_index()
    n = len(df)
    eng = _engine(dev_engine)
    # stage the lists zero-padded to [6][n][51] (the first 25 entries are kept;
    # shorter lists are already zero past their end, so the kernel's list
    # length is the full stride).  A series column of the drop-in's frames
    # (hourly_column.RowColumn) is staged whole from its [n][w] rows; any other
    # column cell by cell as the reference reads it.
    host = np.zeros((6, n, STRIDE), dtype=np.float64)
    present = np.zeros((2, n), dtype=bool)
    for ci, (case, cols) in enumerate(CASES):
        for si, c in enumerate(cols):
            if c in df.columns and isinstance(df[c].array, RowColumn):
                _stage_rows(df[c].array, host[3 * ci + si])
                present[ci] |= df[c].array.cells_are_lists()              # :54-56, 66-68
                continue
            col = df[c].tolist() if c in df.columns else [None] * n   # r.get(c) is None
            for r, v in enumerate(col):
                present[ci, r] |= isinstance(v, (list, tuple))            # :54-56, 66-68
                a = _as_float_list(v)
                if a is None:
                    continue
                k = min(a.size, STRIDE)
                host[3 * ci + si, r, :k] = a[:k]
    dev = torch.from_numpy(host).to(eng.dev)
    c_out = _lib.Outputs(**{f: dev[j].data_ptr() for j, f in enumerate(OUT_FIELDS)})
    res = _run(eng, c_out, np.full(n, STRIDE, dtype=np.int32), n).cpu().numpy()
    aid = (df["agent_id"].to_numpy() if "agent_id" in df.columns else np.full(n, -1)).astype(np.int64)
    # records in iterrows order (:50-73): per row its pv_only, then its pv_batt
    r_idx, c_idx = np.nonzero(present.T)
    if r_idx.size == 0:
        return None
    rec = {"agent_id": aid[r_idx].tolist(), "year": [int(year)] * r_idx.size,
           "scenario_case": [CASES[c][0] for c in c_idx.tolist()]}
    for si, s in enumerate(SERIES):
        rec[s] = res[3 * c_idx + si, r_idx].tolist()
    out = pd.DataFrame(rec)
    if writer is not None:
        writer(out, engine, schema, owner, TABLE, if_exists="append", append_transformations=False)
    return out
