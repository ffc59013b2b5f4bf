"""Drop-in replacement for the hot-path API of dGen's financial_functions
module (tsgsteele/dgen dgen_os/python/financial_functions.py):

    calc_system_size_and_performance(con, agent, sectors, rate_switch_table=None)  ff:291
    size_chunk(static_agents_df, sectors, rate_switch_table, mode="simple")         ff:1136
    _init_worker(dsn, role)                                                         ff:1129
    normalize_tariff / process_tariff                                               ff:962 / ff:575

Same signatures, same output columns and the same error behaviour (a sizing
failure raises and aborts the caller, like r.get() at dgen_model.py:382).  The
difference is where the work runs: a chunk is columnarised once and sized in
one batched launch of the gfx950 kernels; PySAM is not used.

``con`` is either a ProfileStore (dgen_amd.profiles) or a DB-API connection,
on which the reference's two profile queries run once per distinct key.
"""
from __future__ import annotations

import os
import threading
from typing import Dict, Optional, Tuple

import numpy as np
import pandas as pd

from . import _lib
from .columnar import PopulationBuilder
from .profiles import ProfileStore, SqlProfileSource, as_source
from .tariff import (FORCE_NET_BILLING, SKIP_DEMAND_CHARGES, normalize_tariff,  # noqa: F401
                     process_tariff)

NH = _lib.NH

_worker_conn = None
_engine = None
_engine_lock = threading.Lock()
_sql_sources: Dict[int, SqlProfileSource] = {}


def get_engine():
    """Process-wide Engine on this rank's GPU (LOCAL_RANK, else 0)."""
    global _engine
    with _engine_lock:
        if _engine is None:
            from .engine import Engine
            _engine = Engine(int(os.environ.get("LOCAL_RANK", "0")))
        return _engine


def _init_worker(dsn, role):
    """Pool initializer (ff:1129-1134): open this worker's DB connection.  The
    sizing itself no longer needs a pool; the connection only feeds profiles."""
    global _worker_conn
    try:
        import psycopg2  # noqa: F401
    except Exception as e:  # pragma: no cover - no DB driver offline
        raise RuntimeError("_init_worker needs a DB driver (psycopg2) for the profile queries") from e
    import psycopg2 as pg
    _worker_conn = pg.connect(dsn)
    if role:
        cur = _worker_conn.cursor()
        cur.execute(f"SET ROLE {role};")
        cur.close()


def _source(con) -> ProfileStore:
    if isinstance(con, ProfileStore):
        return con
    src = _sql_sources.get(id(con))
    if src is None or src.con is not con:
        src = as_source(con)
        _sql_sources[id(con)] = src
    return src


# ----------------------------------------------------------------------------
# batch core
# ----------------------------------------------------------------------------
def _finite_float(x, default=np.nan) -> float:
    try:
        return float(x)
    except Exception:
        return default


def _columnarize(rows, src: ProfileStore, rate_switch_table):
    b = PopulationBuilder(rate_switch_table)
    for agent in rows:
        b.add(load_row=src.load_row(agent), cf_row=src.solar_row(agent),
              sector_abbr=agent["sector_abbr"], state_abbr=agent.get("state_abbr", ""),
              eia_id=agent["eia_id"], tariff_dict=agent["tariff_dict"],
              wholesale=agent.get("wholesale_prices", None),
              load_kwh=_finite_float(agent["load_kwh_per_customer_in_bin"]),
              price_mult=_finite_float(agent["elec_price_multiplier"]),
              econ_life=int(agent["economic_lifetime_yrs"]), loan_term=int(agent["loan_term_yrs"]),
              inflation=_finite_float(agent["inflation_rate"]),
              pv_deg=_finite_float(agent["pv_degradation_factor"]),
              escalator=_finite_float(agent["elec_price_escalator"]),
              down_payment=_finite_float(agent["down_payment_fraction"]),
              tax_rate=_finite_float(agent["tax_rate"]),
              real_discount=_finite_float(agent["real_discount_rate"]),
              itc_frac=_finite_float(agent["itc_fraction_of_capex"]),
              capex=_finite_float(agent["system_capex_per_kw"]),
              capex_combined=_finite_float(agent["system_capex_per_kw_combined"]),
              batt_capex_kwh=_finite_float(agent["batt_capex_per_kwh_combined"]),
              ccm=_finite_float(agent["cap_cost_multiplier"]),
              vor=_finite_float(agent["value_of_resiliency_usd"]))
    return b


def _raise_for_status(status: np.ndarray, agent_ids) -> None:
    bad = np.nonzero(status & (_lib.ST_FATAL | _lib.ST_ZERO_LOAD | _lib.ST_EMPTY_EC))[0]
    if bad.size == 0:
        return
    k = int(bad[0])
    s = int(status[k])
    who = agent_ids[k]
    if s & _lib.ST_BOUNDS:
        raise ValueError(f"agent {who}: Optimization bounds must be finite scalars.")
    if s & _lib.ST_ZERO_LOAD:
        # ff:549 first_without / load_kwh_per_customer_in_bin with a zero load
        raise ZeroDivisionError(f"agent {who}: float division by zero (load_kwh_per_customer_in_bin == 0)")
    if s & _lib.ST_EMPTY_EC:
        raise _lib.DgenError(f"agent {who}: tariff has no energy-charge matrix "
                             "(the reference would price it with stale PySAM state)")
    if s & _lib.ST_UNIT:
        raise _lib.DgenError(f"agent {who}: tariff usage unit kWh/kW is not supported")
    if s & _lib.ST_DEMAND:
        raise _lib.DgenError(f"agent {who}: demand-charge matrix outside SSC's limits "
                             "(0-based month, 1-based period <= 8, contiguous tiers <= 4)")
    raise _lib.DgenError(f"agent {who}: sizing failed with status 0x{s:x}")


def size_rows(rows, con, rate_switch_table, hourly: str = "list"):
    """Size a list of agent rows (pd.Series) in one batched device call.
    Returns (list of output Series, host outputs dict)."""
    if rate_switch_table is None:
        # elec.py:840 filters the table unconditionally for kw > 0
        raise AttributeError("'NoneType' object has no attribute 'loc' (rate_switch_table is required)")
    src = _source(con)
    src.ensure(rows)
    b = _columnarize(rows, src, rate_switch_table)
    cols = b.columns()
    eng = get_engine()
    from .engine import outputs_to_host, profile_order
    import torch
    eng.load_profiles(src.shapes, src.cfs, b.wholesale.array())
    eng.set_tariffs(b.tariffs.array())
    eng.set_switches(b.switches.array())
    batch = eng.upload_agents(cols, order=profile_order(cols))
    out = eng.alloc_outputs(batch.n, hourly=True)
    eng.size(batch, out)
    torch.cuda.synchronize(eng.dev)
    o = outputs_to_host(out, batch.perm)
    ids = [r.get("agent_id", r.name) for r in rows]
    _raise_for_status(o["status"], ids)
    cfs = src.cfs
    result = []
    for i, agent in enumerate(rows):
        result.append(_output_row(agent, i, o, b, cfs[cols["cf_row"][i]], hourly))
    return result, o


def _hourly(a: np.ndarray, fmt: str):
    if fmt == "list":
        return a.astype(np.float64).tolist()
    if fmt == "array":
        return a.astype(np.float64)
    return None


def _output_row(agent: pd.Series, i: int, o, b: PopulationBuilder, cf_row, fmt: str) -> pd.Series:
    """Fields in the order ff:449-565 writes them."""
    a = agent.copy()
    if "agent_id" not in a.index:
        a.loc["agent_id"] = a.name
    n1 = int(agent["economic_lifetime_yrs"]) + 1
    yl = lambda k: [float(v) for v in o[k][i, :n1]]
    a.loc["naep"] = float(o["naep"][i])
    a.loc["cf_energy_value_pv_only"] = yl("cfev_pv")
    a.loc["utility_bill_w_sys_pv_only"] = yl("bill_w_pv")
    a.loc["utility_bill_wo_sys_pv_only"] = yl("bill_wo_pv")
    if int(o["switched"][i]):
        # elec.py:852-855: the sticky switch rewrites the agent in place
        r = b.switches.row_of_tariff.get(int(o["tariff_final"][i]))
        a["nem_system_kw_limit"] = 1e6
        if r is not None:
            a["tariff_id"] = r["rate_id_alias"]
            a["tariff_dict"] = r["json"]
    a.loc["cf_energy_value_pv_batt"] = yl("cfev_batt")
    a.loc["utility_bill_w_sys_pv_batt"] = yl("bill_w_batt")
    a.loc["utility_bill_wo_sys_pv_batt"] = yl("bill_wo_batt")
    if fmt != "none":
        a.loc["baseline_net_hourly"] = _hourly(o["baseline"][i], fmt)
        a.loc["adopter_net_hourly_pvonly"] = _hourly(o["net_pvonly"][i], fmt)
        a.loc["adopter_net_hourly_with_batt"] = _hourly(o["net_with_batt"][i], fmt)
        a.loc["adopter_net_hourly"] = _hourly(o["net_pvonly"][i], fmt)
    a.loc["system_kw"] = float(o["system_kw"][i])
    a.loc["annual_energy_production_kwh"] = float(o["annual_kwh"][i])
    a.loc["naep"] = float(o["naep"][i])
    a.loc["capacity_factor"] = float(o["capacity_factor"][i])
    a.loc["price_per_kwh"] = float(o["price_per_kwh"][i])
    a.loc["npv"] = float(o["npv"][i])
    a.loc["payback_period"] = float(o["payback_period"][i])
    a.loc["cash_flow"] = yl("cash_flow")
    a.loc["batt_kw"] = float(o["batt_kw"][i])
    a.loc["batt_kwh"] = float(o["batt_kwh"][i])
    if fmt != "none":
        gpk = np.asarray(cf_row, dtype=float) / 1e6
        a.loc["pv_per_kw_hourly"] = gpk.tolist() if fmt == "list" else gpk
    return a


# ----------------------------------------------------------------------------
# reference API
# ----------------------------------------------------------------------------
def calc_system_size_and_performance(con, agent: pd.Series, sectors, rate_switch_table=None):
    """ff:291 -- size one agent (PV kW via bounded Brent, then one PV+battery
    run) and return the agent row with the output fields populated."""
    rows, _ = size_rows([agent], con, rate_switch_table)
    return rows[0]


_DROP = ("adopter_load_hourly", "adopter_pv_hourly", "adopter_batt_to_load_hourly",
         "adopter_grid_to_batt_hourly", "pv_per_kw_hourly", "consumption_hourly",
         "generation_hourly", "batt_dispatch_profile", "net_hourly")


def size_chunk(static_agents_df: pd.DataFrame, sectors, rate_switch_table, mode="simple"):
    """ff:1136 -- size a chunk; returns (df_out, agg) with
    agg["net_sum_kw"][h] = sum_agents adopter[h] * n_adopt + baseline[h] * (n_cust - n_adopt)."""
    global _worker_conn
    rows = []
    for aid, row in static_agents_df.iterrows():
        r = row.copy()
        r.name = aid
        rows.append(r)
    if not rows:
        return pd.DataFrame([]), {"mode": "simple", "n_hours": 0, "net_sum_kw": []}
    sized, o = size_rows(rows, _worker_conn, rate_switch_table)
    n_cust = np.array([_finite_float(s.get("customers_in_bin", 0.0), 0.0) for s in sized])
    n_adopt = np.array([_finite_float(s.get("number_of_adopters", 0.0), 0.0) for s in sized])
    n_non = np.maximum(n_cust - n_adopt, 0.0)
    adop = o["net_pvonly"].astype(np.float64)
    base = o["baseline"].astype(np.float64)
    net_sum = np.zeros(NH)
    for k in range(len(sized)):        # agent order, like the reference's running sum
        net_sum += adop[k] * n_adopt[k] + base[k] * n_non[k]
    out_rows = []
    for s in sized:
        for c in _DROP:
            if c in s.index:
                s = s.drop(labels=[c])
        out_rows.append(s)
    df_out = pd.DataFrame(out_rows)
    agg = {"mode": "simple", "n_hours": NH, "net_sum_kw": net_sum.tolist()}
    return df_out, agg
