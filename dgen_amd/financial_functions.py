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
from .columnar import PopulationBuilder, columnize_frame
from .profiles import ProfileStore, SqlProfileSource, as_source
from .tariff import (FORCE_NET_BILLING, SKIP_DEMAND_CHARGES, normalize_tariff,  # noqa: F401
                     process_tariff)

NH = _lib.NH

_worker_conn = None
_engine = None
_engine_lock = threading.Lock()
_sql_sources: Dict[int, SqlProfileSource] = {}


def worker_device() -> int:
    """The GPU this process sizes on, chosen before anything touches the GPU.

    * ``LOCAL_RANK`` (a torchrun rank): that device;
    * otherwise this process's index among its parent's children -- the
      reference's caller spawns ``LOCAL_CORES`` pool workers per model year
      (``dgen_model.py:309-317``, 8-32 per node), numbered consecutively by
      multiprocessing (``current_process()._identity``), so worker k takes
      device (k - 1) mod the device count and the pool spreads evenly over the
      node's GPUs with ``dgen_model.py`` unchanged;
    * ``DGEN_DEVICES`` (e.g. ``"0,2,4,6"``) restricts that rotation to a list;
    * the main process (the reference's ``cores=None`` path): device 0 (or the
      list's first).
    ``torch.cuda.device_count()`` does not initialise HIP on this image, so
    the spawned worker may ask it before its Engine opens the device."""
    lr = os.environ.get("LOCAL_RANK")
    if lr is not None and lr.strip() != "":
        return int(lr)
    import multiprocessing as mp
    ident = getattr(mp.current_process(), "_identity", ()) or ()
    k = int(ident[-1]) - 1 if ident else 0
    devs = os.environ.get("DGEN_DEVICES", "").strip()
    if devs:
        lst = [int(x) for x in devs.split(",") if x.strip()]
        if not lst:
            raise ValueError(f"DGEN_DEVICES={devs!r} names no device")
        return lst[k % len(lst)]
    import torch
    n = int(torch.cuda.device_count())
    return k % n if n > 0 else 0


def get_engine():
    """Process-wide Engine on this process's GPU (worker_device())."""
    global _engine
    with _engine_lock:
        if _engine is None:
            from .engine import Engine
            _engine = Engine(worker_device())
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
    """Raise like the reference for a chunk-fatal agent status.  Agents whose
    tariff bills kWh/kW tiers whose month peaks the batch cannot supply
    (ST_UNIT: no demand record behind the tariff) are not fatal: they come
    back unsized (NaN outputs, no-system hourly planes) with a warning, and
    the rest of the chunk is sized."""
    unit = np.nonzero(status & _lib.ST_UNIT)[0]
    if unit.size:
        import warnings
        ids = [agent_ids[int(k)] for k in unit[:5]]
        warnings.warn(f"{unit.size} agent(s) left unsized: kWh/kW tiers without month peaks (no demand "
                      f"record behind the tariff); NaN outputs (first: {ids})", RuntimeWarning,
                      stacklevel=3)
    bad = np.nonzero(status & ((_lib.ST_FATAL & ~_lib.ST_UNIT) | _lib.ST_ZERO_LOAD | _lib.ST_EMPTY_EC))[0]
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
    if s & _lib.ST_DEMAND:
        raise _lib.DgenError(f"agent {who}: demand-charge matrix outside SSC's limits "
                             "(0-based month, 1-based period <= 8, contiguous tiers <= 4)")
    raise _lib.DgenError(f"agent {who}: sizing failed with status 0x{s:x}")


_loaded = {}


def _device_tables(eng, src: ProfileStore, b: PopulationBuilder):
    """Upload the profile tables (and their row / slot sums) only when the
    store has grown or the wholesale table changed since the last call: a
    chunk loop re-sizes against the same tables."""
    wh = b.wholesale.array()
    wkey = None if wh is None else (wh.shape, hash(wh.tobytes()))
    key = (id(eng), id(src), src.n_load, src.n_solar, wkey)
    if _loaded.get("key") != key:
        eng.load_profiles(src.shapes, src.cfs, wh)
        _loaded["key"] = key
    eng.set_tariffs(b.tariffs.array())
    eng.set_switches(b.switches.array())


def agent_device_bytes(eng) -> int:
    """HBM one agent of a drop-in call holds while it is sized: the three fp64
    hourly planes (3 x 8760 x 8 B), its share of the workspace (bins, scratch
    plane, split records: dgen_workspace_bytes at a scratch slot per agent),
    the yearly and scalar outputs twice (the caller-order gather before the
    download) and the agent columns."""
    k = 4096
    ws = int(eng.lib.dgen_workspace_bytes(k, k)) // k
    yearly = len(_lib.OUTPUT_YEARLY) * (_lib.MAXY + 1) * 8
    return 3 * NH * 8 + ws + 2 * (yearly + 8 * len(_lib.OUTPUT_SCALARS)) + 8 * len(_lib.AGENT_COLUMNS)


def device_rows_budget(eng, frac: float = 0.3) -> int:
    """Largest agent count one sizing call puts on the device at a time:
    ``DGEN_MAX_ROWS`` if set, else frac x (free HBM + this process's cached,
    unused blocks) / agent_device_bytes.  frac 0.3: two sub-batches are
    resident at once (one sizing while the previous one's planes download),
    and other workers sharing the GPU (a spawn pool larger than the node's GPU
    count) see the rest.  Workers that share a device may read the free
    memory at the same moment, so frac is divided by ``DGEN_WORKERS_PER_DEVICE``
    (pool size / GPUs; default 1); _run_device also halves its sub-batch and
    retries when a device allocation fails.  At least 1024."""
    env = os.environ.get("DGEN_MAX_ROWS", "").strip()
    if env:
        return max(1, int(env))
    import torch
    share = max(1, int(os.environ.get("DGEN_WORKERS_PER_DEVICE", "1").strip() or 1))
    free, _total = torch.cuda.mem_get_info(eng.dev)
    spare = torch.cuda.memory_reserved(eng.dev) - torch.cuda.memory_allocated(eng.dev)
    return max(1024, int(frac / share * (free + max(spare, 0)) / agent_device_bytes(eng)))


def _run_device(b: PopulationBuilder, cols, src: ProfileStore, timing: Optional[dict] = None,
                net_weights: Optional[Tuple[np.ndarray, np.ndarray]] = None, hourly_async: bool = False,
                hourly_device: bool = False, max_rows: Optional[int] = None):
    """Size the batch in sub-batches of at most max_rows agents (default
    device_rows_budget()): a frame larger than the device budget is cut into
    consecutive caller-order row ranges, each sized in its own device call
    with its own outputs; the host outputs are concatenated (an agent's
    outputs do not depend on the other agents of its batch, so they are the
    bits a single call gives), net_sum_kw is the sum of the sub-batches'
    (to rounding: 1e-12 relative), and the hourly planes are one segmented
    plane over the sub-batches' (hourly_column._Segments).  At most two
    sub-batches are on the device at once: sub-batch k sizes while k - 1's
    planes download, and k waits for k - 2's.  hourly_device with more than
    one sub-batch: the planes come to the host instead (keeping every
    sub-batch's planes in HBM would undo the bound)."""
    n = len(cols["load_kwh"])
    if max_rows is None:
        max_rows = device_rows_budget(get_engine())
    max_rows = max(1, int(max_rows))
    import torch
    try:
        return _run_device_rows(b, cols, src, timing, net_weights, hourly_async, hourly_device, max_rows)
    except torch.cuda.OutOfMemoryError:
        # another worker on this device took the memory the budget counted on:
        # free this process's cached blocks and size in halves (down to 1024)
        smaller = min(n, max_rows) // 2
        if smaller < 1024:
            raise
        torch.cuda.empty_cache()
        return _run_device(b, cols, src, timing, net_weights, hourly_async, hourly_device, max_rows=smaller)


def _run_device_rows(b, cols, src, timing, net_weights, hourly_async, hourly_device, max_rows: int):
    n = len(cols["load_kwh"])
    if n <= max_rows:
        return _run_device_once(b, cols, src, timing, net_weights, hourly_async, hourly_device)
    from .hourly_column import _Segments
    parts = []
    tm_sum: dict = {}
    for lo in range(0, n, max_rows):
        hi = min(n, lo + max_rows)
        if len(parts) >= 2:            # bound: k - 2's planes have left the device
            for name in _lib.OUTPUT_HOURLY:
                p = parts[-2].get(name)
                if p is not None and hasattr(p, "result"):
                    p.result()
        sub = {k: v[lo:hi] for k, v in cols.items()}
        nw = None if net_weights is None else tuple(np.asarray(w)[lo:hi] for w in net_weights)
        tm: dict = {}
        parts.append(_run_device_once(b, sub, src, tm, nw, hourly_async=True, hourly_device=False))
        for k, v in tm.items():
            tm_sum[k] = tm_sum.get(k, 0.0) + v
    o = {}
    for name, _ in _lib.OUTPUT_SCALARS:
        o[name] = np.concatenate([p[name] for p in parts])
    for name in _lib.OUTPUT_YEARLY:
        o[name] = np.concatenate([p[name] for p in parts])
    for name in _lib.OUTPUT_HOURLY:
        segs = _Segments([(p[name], np.arange(p[name].n, dtype=np.int64), None, False) for p in parts])
        if hourly_async or hourly_device:
            o[name] = segs
        else:
            o[name] = segs.result()
    if net_weights is not None:
        net = parts[0]["net_sum_kw"].copy()
        for p in parts[1:]:
            net += p["net_sum_kw"]
        o["net_sum_kw"] = net
    if timing is not None:
        timing.update(tm_sum, sub_batches=len(parts))
    return o


def _run_device_once(b: PopulationBuilder, cols, src: ProfileStore, timing: Optional[dict] = None,
                     net_weights: Optional[Tuple[np.ndarray, np.ndarray]] = None, hourly_async: bool = False,
                     hourly_device: bool = False):
    """Size the batch in one device call; net_weights = (number_of_adopters, non-adopters) per
    caller row also returns o["net_sum_kw"], size_chunk's hourly aggregate
    summed on the device from the planes in place (k_state_hourly, one
    segment, fixed order) instead of a host loop over the agents.
    hourly_async: the three hourly planes come back as engine.HostPlane
    (downloading on a background thread), everything else at once."""
    import time
    import torch
    from .attachment import state_hourly
    from .engine import outputs_to_host, profile_order
    eng = get_engine()
    t0 = time.perf_counter()
    _device_tables(eng, src, b)
    batch = eng.upload_agents(cols, order=profile_order(cols))
    # fp64 hourly planes: the reference's hourly lists are fp64 (ff:523,536-539)
    out = eng.alloc_outputs(batch.n, hourly=True, hourly_f64=True)
    torch.cuda.synchronize(eng.dev)
    t1 = time.perf_counter()
    eng.size(batch, out)
    net = None
    if net_weights is not None:
        perm = batch.perm if batch.perm is not None else np.arange(batch.n)
        na = eng._to_dev(np.asarray(net_weights[0], np.float64)[perm], torch.float64)
        nn = eng._to_dev(np.asarray(net_weights[1], np.float64)[perm], torch.float64)
        pv = out["net_pvonly"]
        net = state_hourly(eng, (out["baseline"], pv, pv), (na, torch.zeros_like(na), nn), None,
                           [0, batch.n])[0] * 1000.0
    torch.cuda.synchronize(eng.dev)
    t2 = time.perf_counter()
    o = outputs_to_host(out, batch.perm, hourly_async=hourly_async, hourly_device=hourly_device)
    del out
    unsized = (o["status"] & _lib.ST_UNIT) != 0
    if unsized.any():          # kWh/kW tiers without month peaks: every sizing output NaN
        for k, v in o.items():
            if v is not None and k not in _lib.OUTPUT_HOURLY and v.dtype.kind == "f":
                v[unsized] = np.nan
    if net is not None:
        o["net_sum_kw"] = net.cpu().numpy()
    if timing is not None:
        timing.update(upload_s=t1 - t0, device_s=t2 - t1, download_s=time.perf_counter() - t2)
    return o


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
    o = _run_device(b, cols, src)
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


def _yearly_lists(a: np.ndarray, n1: np.ndarray, fmt: str = "list"):
    """Row i's first n1[i] values as a Python list, one tolist() per distinct
    analysis length (the frame usually has one or two); fmt "array": each
    row as a float64 ndarray view of one [rows, n] block instead (no per-value
    Python float)."""
    uniq = np.unique(n1)
    if fmt == "array" and uniq.size == 1:
        return list(a[:, :int(uniq[0])])
    out = np.empty(a.shape[0], dtype=object)
    for n in uniq:
        ix = np.nonzero(n1 == n)[0]
        if fmt == "array":
            for j, r in zip(ix.tolist(), a[ix, :n]):
                out[j] = r
        else:
            out[ix] = a[ix, :n].tolist() if ix.size > 1 else [a[ix[0], :n].tolist()]
    return list(out)


def size_frame(df: pd.DataFrame, con, rate_switch_table, hourly: str = "lazy",
               timing: Optional[dict] = None, net_weights=None, max_rows: Optional[int] = None):
    """The batched form of calc_system_size_and_performance over a whole agent
    frame (what size_chunk needs), built by column: the frame is columnised
    at once (columnar.columnize_frame), sized in one device call, and the
    output columns are assigned whole.  Same values and columns as mapping
    calc_system_size_and_performance over the rows (ff:449-565 write order);
    hourly: "lazy" (the default: every series column is an
    hourly_column.RowColumn, a pandas extension array built in O(1) -- an
    hourly cell is the agent's float64 row of a plane that is still crossing
    PCIe on a background thread when the frame is returned (reading a cell
    waits for it), a yearly cell the agent's Python list, made when read; the
    reference's consumers read hourly cells with len() and np.asarray,
    attachment_rate_functions.py:166-182, and yearly cells as lists,
    finance_series_export.py:51-64), "device" (as lazy, but the hourly planes
    stay in HBM: attachment.export_state_hourly_with_storage_mix reduces them
    there and they never cross PCIe unless a cell is read), "array" (the planes on the host before
    returning: hourly and yearly cells float64 row views -- the reference's
    own finance export skips non-list cells), "list" (the reference's fp64
    lists throughout) or "none" (no hourly columns, yearly lists).  The device
    computes the hourly planes in fp64 for this path (the PCIe-bound phase:
    3 x 8760 x 8 B per agent), downloaded while the frame is assembled.
    timing: filled with the host / device phases (seconds).  max_rows: the
    most agents on the device at once (default device_rows_budget(): a frame
    larger than free HBM allows is sized in consecutive sub-batches with the
    same outputs, _run_device)."""
    import time
    if rate_switch_table is None:
        raise AttributeError("'NoneType' object has no attribute 'loc' (rate_switch_table is required)")
    t0 = time.perf_counter()
    src = _source(con)
    src.ensure_frame(df)
    b = columnize_frame(df, src, rate_switch_table)
    cols = b.frame_columns
    t1 = time.perf_counter()
    dev_t: dict = {}
    o = _run_device(b, cols, src, dev_t, net_weights, hourly_async=hourly in ("lazy", "array", "list"),
                    hourly_device=hourly == "device", max_rows=max_rows)
    t2 = time.perf_counter()
    ids = df["agent_id"].tolist() if "agent_id" in df else list(df.index)
    _raise_for_status(o["status"], ids)
    out = df.copy(deep=False)
    if "agent_id" not in out.columns:
        out.insert(len(out.columns), "agent_id", list(df.index))
    n1 = df["economic_lifetime_yrs"].astype(np.int64).to_numpy() + 1
    from .hourly_column import hourly_column, yearly_column
    if hourly in ("lazy", "device"):
        def ycol(a):     # O(1): lists made when a cell is read
            return pd.Series(yearly_column(a, n1), index=out.index, copy=False)
    else:
        def ycol(a):
            return _yearly_lists(a, n1, "array" if hourly == "array" else "list")
    out["naep"] = o["naep"]
    out["cf_energy_value_pv_only"] = ycol(o["cfev_pv"])
    out["utility_bill_w_sys_pv_only"] = ycol(o["bill_w_pv"])
    out["utility_bill_wo_sys_pv_only"] = ycol(o["bill_wo_pv"])
    sw = np.nonzero(o["switched"] != 0)[0]
    if sw.size:
        # elec.py:852-855: the sticky switch rewrites the agent in place
        lim = (np.asarray(out["nem_system_kw_limit"].tolist(), dtype=object) if "nem_system_kw_limit" in out
               else np.full(len(out), np.nan, dtype=object))
        tid = np.asarray(out["tariff_id"].tolist(), dtype=object) if "tariff_id" in out else None
        tdi = np.empty(len(out), dtype=object)
        tdi[:] = out["tariff_dict"].tolist()
        for i in sw:
            lim[i] = 1e6
            r = b.switches.row_of_tariff.get(int(o["tariff_final"][i]))
            if r is not None:
                if tid is not None:
                    tid[i] = r["rate_id_alias"]
                tdi[i] = r["json"]
        out["nem_system_kw_limit"] = pd.Series(lim, index=out.index).infer_objects()
        if tid is not None:
            out["tariff_id"] = pd.Series(tid, index=out.index).infer_objects()
        out["tariff_dict"] = pd.Series(tdi, index=out.index)
    out["cf_energy_value_pv_batt"] = ycol(o["cfev_batt"])
    out["utility_bill_w_sys_pv_batt"] = ycol(o["bill_w_batt"])
    out["utility_bill_wo_sys_pv_batt"] = ycol(o["bill_wo_batt"])
    t_wait = 0.0
    if hourly != "none":
        def conv(plane):
            nonlocal t_wait
            if hourly in ("lazy", "device"):
                # O(1): the column is the plane and its row index
                return pd.Series(hourly_column(plane), index=out.index, copy=False)
            tw = time.perf_counter()
            a = plane.result()
            t_wait += time.perf_counter() - tw
            return a.tolist() if hourly == "list" else list(a)
        out["baseline_net_hourly"] = conv(o["baseline"])
        out["adopter_net_hourly_pvonly"] = conv(o["net_pvonly"])
        out["adopter_net_hourly_with_batt"] = conv(o["net_with_batt"])
        out["adopter_net_hourly"] = out["adopter_net_hourly_pvonly"]
    out["system_kw"] = o["system_kw"]
    out["annual_energy_production_kwh"] = o["annual_kwh"]
    out["capacity_factor"] = o["capacity_factor"]
    out["price_per_kwh"] = o["price_per_kwh"]
    out["npv"] = o["npv"]
    out["payback_period"] = o["payback_period"]
    out["cash_flow"] = ycol(o["cash_flow"])
    out["batt_kw"] = o["batt_kw"]
    out["batt_kwh"] = o["batt_kwh"]
    t3 = time.perf_counter()
    if timing is not None:
        # download_wait_s: time the frame assembly waited for the hourly planes
        timing.update(columnize_s=t1 - t0, device_call_s=t2 - t1, output_frame_s=t3 - t2,
                      download_wait_s=t_wait, **dev_t)
    return out, o


def size_chunk(static_agents_df: pd.DataFrame, sectors, rate_switch_table, mode="simple",
               hourly: str = "lazy", timing: Optional[dict] = None, max_rows: Optional[int] = None):
    """ff:1136 -- size a chunk; returns (df_out, agg) with
    agg["net_sum_kw"][h] = sum_agents adopter[h] * n_adopt + baseline[h] * (n_cust - n_adopt)."""
    global _worker_conn
    if len(static_agents_df) == 0:
        return pd.DataFrame([]), {"mode": "simple", "n_hours": 0, "net_sum_kw": []}
    df = static_agents_df
    num = lambda c: (np.array([_finite_float(v, 0.0) for v in df[c].tolist()], np.float64)
                     if c in df else np.zeros(len(df)))
    n_cust, n_adopt = num("customers_in_bin"), num("number_of_adopters")
    n_non = np.maximum(n_cust - n_adopt, 0.0)
    # net_sum_kw[h] = sum_agents adopter[h] * n_adopt + baseline[h] * n_non (ff:1186),
    # on the device; the reference's running sum in agent order and the
    # kernel's fixed-order tree agree to rounding (parity test: 1e-12 relative)
    df_out, o = size_frame(df, _worker_conn, rate_switch_table, hourly=hourly, timing=timing,
                           net_weights=(n_adopt, n_non), max_rows=max_rows)
    df_out = df_out.drop(columns=[c for c in _DROP if c in df_out.columns])
    agg = {"mode": "simple", "n_hours": NH, "net_sum_kw": o["net_sum_kw"].tolist()}
    return df_out, agg
