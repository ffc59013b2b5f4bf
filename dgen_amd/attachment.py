"""Battery attachment and the per-state hourly export on the device:
drop-ins for

    attachment_rate_functions._allocate_battery_adopters_integer(df, year)          :58-148
    attachment_rate_functions.export_state_hourly_with_storage_mix(engine, schema,
        owner, year, solar_agents_df)                                               :151-206

Grouping keys, string ranks of agent_id and the records frame stay on the host;
the per-group largest-remainder allocation (k_batt_attach: numpy-order group
sum, floor, radix-select of the winners by (fraction desc, str(agent_id) asc)),
the export multipliers (k_export_weights) and the per-state hourly sums
(k_state_hourly) run through the C-ABI.  state_hourly_from_outputs() feeds the
sizing kernels' hourly planes to the export in place, so a national run never
materialises the 3 x 8760 hourly lists per agent ("output volume").
"""
from __future__ import annotations

import ctypes
from typing import Callable, Dict, Optional, Sequence

import numpy as np
import pandas as pd

from . import _lib

ATTACH_IN = ["new_adopters", "aid_rank", "batt_kw", "batt_kwh", "batt_kw_cum_last_year",
             "batt_kwh_cum_last_year"]
ATTACH_OUT = ["added", "new_batt_kw", "new_batt_kwh", "batt_kw_cum", "batt_kwh_cum"]
_NEED = ['state_abbr', 'sector_abbr', 'agent_id', 'new_adopters', 'number_of_adopters', 'batt_kw',
         'batt_kwh', 'batt_kw_cum_last_year', 'batt_kwh_cum_last_year', 'storage_attachment_rate']
HOURLY_COLS = ("baseline_net_hourly", "adopter_net_hourly_pvonly", "adopter_net_hourly_with_batt")


class AttachIn(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in ATTACH_IN]


class AttachOut(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in ATTACH_OUT]


def _bind(L):
    if getattr(L, "_dgen_attach_bound", False):
        return L
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    L.dgen_batt_attach.restype = i32
    L.dgen_batt_attach.argtypes = [vp, ctypes.POINTER(AttachIn), ctypes.POINTER(AttachOut), vp, vp,
                                   i64, vp]
    L.dgen_export_weights.restype = i32
    L.dgen_export_weights.argtypes = [vp, vp, vp, vp, vp, vp, i64, vp, vp, vp, vp]
    L.dgen_state_hourly.restype = i32
    L.dgen_state_hourly.argtypes = [vp, vp, vp, vp, i32, vp, vp, vp, vp, i64, i32, vp, i64, vp, vp]
    L._dgen_attach_bound = True
    return L


def _engine(engine):
    if engine is not None:
        return engine
    from .financial_functions import get_engine
    return get_engine()


def _isnan(k) -> bool:
    return isinstance(k, float) and k != k


def group_segments(keys: Sequence):
    """pandas groupby(sort=False) on the host: groups in first-appearance order,
    rows in row order inside a group, rows with a NaN key in no group
    (dropna=True).  Returns (idx[m] row numbers grouped, seg_off[S+1], keys)."""
    uniq: Dict = {}
    gid = np.full(len(keys), -1, dtype=np.int64)
    for i, k in enumerate(keys):
        if _isnan(k) or (isinstance(k, tuple) and any(_isnan(x) for x in k)):
            continue
        gid[i] = uniq.setdefault(k, len(uniq))
    sel = np.flatnonzero(gid >= 0)
    idx = sel[np.argsort(gid[sel], kind="stable")]
    counts = np.bincount(gid[sel], minlength=len(uniq))
    seg_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    return idx.astype(np.int64), seg_off, list(uniq.keys())


def string_ranks(agent_id) -> np.ndarray:
    """Rank of str(agent_id) in ascending string order (the reference's
    tie-break, :125-128); equal strings keep row order (stable sort)."""
    s = np.asarray([str(a) for a in agent_id], dtype=np.str_)
    order = np.argsort(s, kind="stable")
    rank = np.empty(len(s), dtype=np.int64)
    rank[order] = np.arange(len(s), dtype=np.int64)
    return rank


def allocate_arrays(engine, state, sector, agent_id, new_adopters, rate, batt_kw, batt_kwh,
                    batt_kw_cum_last_year, batt_kwh_cum_last_year) -> Dict[str, np.ndarray]:
    """k_batt_attach on host columns (row order).  Returns the five allocation
    columns in row order (rows outside every group get 0 added)."""
    import torch
    eng = _engine(engine)
    L = _bind(eng.lib)
    n = len(state)
    idx, seg_off, _ = group_segments(list(zip(state, sector)))
    f64 = lambda a: np.asarray(a, dtype=np.float64)[idx]
    cols = {"new_adopters": f64(new_adopters), "aid_rank": string_ranks(agent_id)[idx],
            "batt_kw": f64(batt_kw), "batt_kwh": f64(batt_kwh),
            "batt_kw_cum_last_year": f64(batt_kw_cum_last_year),
            "batt_kwh_cum_last_year": f64(batt_kwh_cum_last_year)}
    m = len(idx)
    bkw, bkwh = np.asarray(batt_kw, np.float64), np.asarray(batt_kwh, np.float64)
    # rows in no group: added 0, capacities from last year's cumulatives (:140-146)
    base = {"added": np.zeros(n, np.int64), "new_batt_kw": 0 * bkw, "new_batt_kwh": 0 * bkwh,
            "batt_kw_cum": np.asarray(batt_kw_cum_last_year, np.float64) + 0 * bkw,
            "batt_kwh_cum": np.asarray(batt_kwh_cum_last_year, np.float64) + 0 * bkwh}
    if m == 0:
        return base
    g_rate = np.asarray(rate, dtype=np.float64)[idx[seg_off[:-1]]]            # :111
    dev ={k: eng._to_dev(v, torch.int64 if k == "aid_rank" else torch.float64) for k, v in cols.items()}
    outs = {k: torch.empty(m, dtype=torch.int64 if k == "added" else torch.float64, device=eng.dev)
            for k in ATTACH_OUT}
    t_off = eng._to_dev(seg_off, torch.int64)
    t_rate = eng._to_dev(g_rate, torch.float64)
    ci = AttachIn(**{k: dev[k].data_ptr() for k in ATTACH_IN})
    co = AttachOut(**{k: outs[k].data_ptr() for k in ATTACH_OUT})
    _lib.check(L.dgen_batt_attach(eng.ctx, ctypes.byref(ci), ctypes.byref(co), t_off.data_ptr(),
                                  t_rate.data_ptr(), len(seg_off) - 1, eng.stream_handle()),
               "dgen_batt_attach")
    torch.cuda.synchronize(eng.dev)
    res = {}
    for k in ATTACH_OUT:
        v = base[k].copy()
        v[idx] = outs[k].cpu().numpy()
        res[k] = v
    return res


def _allocate_battery_adopters_integer(df: pd.DataFrame, year: int, engine=None) -> pd.DataFrame:
    """attachment_rate_functions.py:58 -- integer battery adopters per state x
    sector by largest remainders; adds batt_adopters_added_this_year,
    new_batt_kw(h), batt_kw(h)_cum.  `year` is unused, as in the reference."""
    df = df.copy()
    for c in _NEED:                                                     # :97-104
        if c not in df.columns:
            df[c] = df.index.astype(str) if c == 'agent_id' else 0.0
    o = allocate_arrays(engine, df['state_abbr'].tolist(), df['sector_abbr'].tolist(),
                        df['agent_id'].tolist(), df['new_adopters'], df['storage_attachment_rate'],
                        df['batt_kw'], df['batt_kwh'], df['batt_kw_cum_last_year'],
                        df['batt_kwh_cum_last_year'])
    df['batt_adopters_added_this_year'] = o["added"].astype(int)
    df['new_batt_kw'] = o["new_batt_kw"]
    df['new_batt_kwh'] = o["new_batt_kwh"]
    df['batt_kw_cum'] = o["batt_kw_cum"]
    df['batt_kwh_cum'] = o["batt_kwh_cum"]
    return df


def export_weights(engine, customers_in_bin, number_of_adopters, batt_kw_cum_last_year, batt_kw,
                   added):
    """k_export_weights: device tensors (w_pvo, w_batt, w_non) [n] float64."""
    import torch
    eng = _engine(engine)
    L = _bind(eng.lib)
    f = lambda a: eng._to_dev(a, torch.float64)
    c, a, p, b = f(customers_in_bin), f(number_of_adopters), f(batt_kw_cum_last_year), f(batt_kw)
    ad = eng._to_dev(added, torch.int64)
    n = c.numel()
    w = [torch.empty(n, dtype=torch.float64, device=eng.dev) for _ in range(3)]
    if n == 0:
        return tuple(w)
    _lib.check(L.dgen_export_weights(eng.ctx, c.data_ptr(), a.data_ptr(), p.data_ptr(), b.data_ptr(),
                                     ad.data_ptr(), n, w[0].data_ptr(), w[1].data_ptr(),
                                     w[2].data_ptr(), eng.stream_handle()), "dgen_export_weights")
    torch.cuda.current_stream(eng.dev).synchronize()
    return tuple(w)


def state_hourly(engine, planes, weights, idx, seg_off):
    """k_state_hourly: planes = (baseline, pvonly, with_batt) device tensors,
    float32 or float64 in dgen_size_agents' hour-quad tiles [n_hours / 4, n, 4]
    (the sizing outputs in place; engine.tile_hourly makes them from
    [n_hours, n]) or float64 [n_hours, n]; weights from export_weights(), idx: plane column of
    each group member (None: identity), seg_off [S+1].  Returns a [S, n_hours]
    float64 device tensor in MW."""
    import torch
    eng = _engine(engine)
    L = _bind(eng.lib)
    base, pvo, wbt = planes
    if any(p.shape != base.shape or p.dtype != base.dtype for p in (pvo, wbt)):
        raise ValueError("state_hourly: the three planes must share shape and dtype")
    if base.dtype not in (torch.float32, torch.float64):
        raise TypeError("state_hourly: planes must be float32 or float64")
    if base.dim() == 3:
        if base.shape[2] != 4:
            raise ValueError("state_hourly: tiled planes must be hour-quad tiles [n_hours/4, n, 4]")
        nh, n = base.shape[0] * 4, base.shape[1]
        layout = 1 if base.dtype == torch.float32 else 2
    elif base.dtype == torch.float64 and base.dim() == 2:
        nh, n = base.shape
        layout = 0
    else:
        raise ValueError("state_hourly: float32 planes must be hour-quad tiles [n_hours/4, n, 4]; "
                         "float64 planes tiles or [n_hours, n]")
    if any(w.numel() != n for w in weights):
        raise ValueError("state_hourly: one weight per plane column")
    so = np.asarray(seg_off, dtype=np.int64)
    m = int(so[-1]) if len(so) else 0
    if len(so) < 1 or so[0] != 0 or np.any(np.diff(so) < 0):
        raise ValueError("segment offsets must start at 0 and be non-decreasing")
    ti = None
    if idx is not None:
        ix = np.asarray(idx, dtype=np.int64)
        if len(ix) != m or (m and (ix.min() < 0 or ix.max() >= n)):
            raise ValueError("state_hourly: idx out of range")
        ti = eng._to_dev(ix, torch.int64)
    elif m > n:
        raise ValueError("state_hourly: segments exceed the plane width")
    S = len(so) - 1
    out = torch.empty((S, nh), dtype=torch.float64, device=eng.dev)
    keep = [p.contiguous() for p in planes] + [w.contiguous() for w in weights]
    t_off = eng._to_dev(so, torch.int64)
    _lib.check(L.dgen_state_hourly(eng.ctx, keep[0].data_ptr(), keep[1].data_ptr(),
                                   keep[2].data_ptr(), layout,
                                   keep[3].data_ptr(), keep[4].data_ptr(), keep[5].data_ptr(),
                                   None if ti is None else ti.data_ptr(), n, nh, t_off.data_ptr(),
                                   S, out.data_ptr(), eng.stream_handle()), "dgen_state_hourly")
    torch.cuda.current_stream(eng.dev).synchronize()
    del keep
    return out


def state_hourly_combined(engine, plane, idx, seg_off):
    """k_state_hourly over Engine.export_plane's combined plane (float64
    hour-quad tiles [n_hours / 4, n, 4]): the rows state_hourly gives from the
    three planes and their weights, bit for bit (dgen_state_hourly
    planes_f32 = 3).  idx / seg_off as in state_hourly."""
    import torch
    eng = _engine(engine)
    L = _bind(eng.lib)
    if plane.dtype != torch.float64 or plane.dim() != 3 or plane.shape[2] != 4:
        raise ValueError("state_hourly_combined: the plane is float64 hour-quad tiles [n_hours/4, n, 4]")
    nh, n = plane.shape[0] * 4, plane.shape[1]
    so = np.asarray(seg_off, dtype=np.int64)
    m = int(so[-1]) if len(so) else 0
    if len(so) < 1 or so[0] != 0 or np.any(np.diff(so) < 0):
        raise ValueError("segment offsets must start at 0 and be non-decreasing")
    ti = None
    if idx is not None:
        ix = np.asarray(idx, dtype=np.int64)
        if len(ix) != m or (m and (ix.min() < 0 or ix.max() >= n)):
            raise ValueError("state_hourly_combined: idx out of range")
        ti = eng._to_dev(ix, torch.int64)
    elif m > n:
        raise ValueError("state_hourly_combined: segments exceed the plane width")
    S = len(so) - 1
    out = torch.empty((S, nh), dtype=torch.float64, device=eng.dev)
    pl = plane.contiguous()
    t_off = eng._to_dev(so, torch.int64)
    _lib.check(L.dgen_state_hourly(eng.ctx, pl.data_ptr(), None, None, 3, None, None, None,
                                   None if ti is None else ti.data_ptr(), n, nh, t_off.data_ptr(),
                                   S, out.data_ptr(), eng.stream_handle()), "dgen_state_hourly")
    torch.cuda.current_stream(eng.dev).synchronize()
    return out


def state_hourly_rows(engine, batch, c_out, with_batt, weights, idx, seg_off):
    """The per-state rows of a batch sized with the with-battery plane alone
    (Engine.alloc_outputs(..., hourly="with_batt"), float32 hour-quad tiles):
    dgen_state_hourly_rows recomputes each agent-hour's load and PV-only net
    load from the profile rows as the scan forms them, so the rows are
    state_hourly's over the three planes, bit for bit.  idx / seg_off as in
    state_hourly; returns a [S, 8760] float64 device tensor in MW."""
    import torch
    eng = _engine(engine)
    if with_batt.dtype != torch.float32 or with_batt.dim() != 3 or with_batt.shape[2] != 4:
        raise ValueError("state_hourly_rows: the with-battery plane is float32 hour-quad tiles [8760/4, n, 4]")
    nh, n = with_batt.shape[0] * 4, with_batt.shape[1]
    if nh != NH_FULL or n != batch.n:
        raise ValueError("state_hourly_rows: one 8760-h plane column per batch agent")
    w = [x.contiguous() for x in weights]
    if any(x.numel() != n for x in w):
        raise ValueError("state_hourly_rows: one weight per agent")
    so = np.asarray(seg_off, dtype=np.int64)
    m = int(so[-1]) if len(so) else 0
    if len(so) < 1 or so[0] != 0 or np.any(np.diff(so) < 0):
        raise ValueError("segment offsets must start at 0 and be non-decreasing")
    ti = None
    if isinstance(idx, torch.Tensor):            # a device index kept by the caller (checked once there)
        if idx.dtype != torch.int64 or idx.device != eng.dev or idx.numel() != m:
            raise ValueError("state_hourly_rows: a device idx is int64, one entry per segment member")
        ti = idx.contiguous()
    elif idx is not None:
        ix = np.asarray(idx, dtype=np.int64)
        if len(ix) != m or (m and (ix.min() < 0 or ix.max() >= n)):
            raise ValueError("state_hourly_rows: idx out of range")
        ti = eng._to_dev(ix, torch.int64)
    elif m > n:
        raise ValueError("state_hourly_rows: segments exceed the batch")
    S = len(so) - 1
    out = torch.empty((S, nh), dtype=torch.float64, device=eng.dev)
    t_off = eng._to_dev(so, torch.int64)
    _lib.check(eng.lib.dgen_state_hourly_rows(eng.ctx, ctypes.byref(eng.tables), ctypes.byref(batch.c_agents),
                                              ctypes.byref(c_out), with_batt.data_ptr(), w[0].data_ptr(),
                                              w[1].data_ptr(), w[2].data_ptr(),
                                              None if ti is None else ti.data_ptr(), n, t_off.data_ptr(), S,
                                              out.data_ptr(), eng.stream_handle()), "dgen_state_hourly_rows")
    torch.cuda.current_stream(eng.dev).synchronize()
    return out


def _len_safe(x) -> int:
    try:
        return len(x)
    except Exception:
        return 0


NH_FULL = 8760


def _device_planes(df):
    """((baseline, pvonly, with_batt) tiled device planes, device column of
    each frame row) when the frame's three hourly columns are full-width rows
    of DevicePlanes of one sizing call (size_frame(hourly="device")), else None."""
    from .engine import DevicePlane
    from .hourly_column import RowColumn
    arrs = [df[c].array for c in HOURLY_COLS]
    if not all(isinstance(a, RowColumn) and isinstance(a._plane, DevicePlane) and a._lens is None
               for a in arrs):
        return None
    p0 = arrs[0]._plane
    if any(a._plane.t.shape != p0.t.shape or a._plane.t.device != p0.t.device or
           not np.array_equal(a._idx, arrs[0]._idx) for a in arrs):
        return None
    if any((a._plane.inv is None) != (p0.inv is None) or
           (a._plane.inv is not None and not bool((a._plane.inv == p0.inv).all())) for a in arrs):
        return None
    cols = p0.device_columns()[arrs[0]._idx]
    if np.unique(cols).size != cols.size:
        # two frame rows on one plane column (pd.concat([df, df]), a take with
        # repeats): each row carries its own weights, which a scatter into
        # device columns cannot hold -- the host path sums them row by row
        return None
    return tuple(a._plane.t for a in arrs), cols


def export_state_hourly_with_storage_mix(engine, schema, owner, year: int,
                                         solar_agents_df: pd.DataFrame,
                                         writer: Optional[Callable] = None, dev_engine=None):
    """attachment_rate_functions.py:151 -- per-state hourly net load (MW) with
    the PV-only / PV+battery / non-adopter mix.  The records frame the reference
    appends to `state_hourly_agg` is returned; it is handed to
    `writer(rec, engine, schema, owner, "state_hourly_agg", if_exists="append",
    append_transformations=False)` (the reference's iFuncs.df_to_psql, DB
    plumbing out of scope here) when one is given."""
    import torch
    if not set(HOURLY_COLS).issubset(solar_agents_df.columns):          # :153-155
        return None
    eng = _engine(dev_engine)
    df = solar_agents_df
    n = len(df)
    idx, seg_off, states = group_segments(df['state_abbr'].tolist())
    from .hourly_column import RowColumn

    def cell_lens(c):          # series columns know their cells' lengths without reading them
        a = df[c].array
        return a.cell_lens() if isinstance(a, RowColumn) else df[c].map(_len_safe).to_numpy(np.int64)
    lens = np.stack([cell_lens(c) for c in HOURLY_COLS]) if n else np.zeros((3, 0), np.int64)
    if not states:
        return None
    nh_state = []
    for s in range(len(states)):                                        # :165-171
        rows = idx[seg_off[s]:seg_off[s + 1]]
        ls = lens[:, rows].astype(np.float64)
        ls[ls == 0] = np.nan
        # Series.min() skips NaN (all-NaN -> NaN); Python's min() then keeps
        # its first argument whenever a comparison with NaN is false
        mins = [float(np.nanmin(r)) if np.isfinite(r).any() else float("nan") for r in ls]
        m = min(mins[0], mins[1], mins[2])
        if m != m:
            raise ValueError("cannot convert float NaN to integer")     # int(nan), :165
        nh_state.append(int(m))

    def col(c, default=0.0):
        return (df[c].to_numpy(np.float64) if c in df.columns else np.full(n, default))

    added = (df['batt_adopters_added_this_year'].to_numpy(np.int64)
             if 'batt_adopters_added_this_year' in df.columns else np.zeros(n, np.int64))
    w = export_weights(eng, col('customers_in_bin'), col('number_of_adopters'),
                       col('batt_kw_cum_last_year'), col('batt_kw'), added)
    out_rows = [None] * len(states)
    dev = _device_planes(df)
    if dev is not None and all(nh == NH_FULL for nh in nh_state):
        # size_frame(hourly="device"): the three planes are still in HBM, full
        # rows -- the same sums in the same member order straight from the
        # tiles (the cells' values are these planes' entries), no PCIe
        planes, dcol = dev
        ncol = planes[0].shape[1]
        wd = []
        cols_t = torch.as_tensor(dcol, device=eng.dev)
        for x in w:
            z = torch.zeros(ncol, dtype=torch.float64, device=eng.dev)
            z.index_copy_(0, cols_t, x)
            wd.append(z)
        res = state_hourly(eng, planes, tuple(wd), dcol[idx], seg_off).cpu().numpy()
        for s_ in range(len(states)):
            out_rows[s_] = res[s_]
        nh_state = [NH_FULL] * len(states)
    for nh in (sorted(set(nh_state)) if dev is None or out_rows[0] is None else []):
        sids = [s for s in range(len(states)) if nh_state[s] == nh]
        members = np.concatenate([idx[seg_off[s]:seg_off[s + 1]] for s in sids])
        so = np.concatenate([[0], np.cumsum([seg_off[s + 1] - seg_off[s] for s in sids])])
        cols = sorted(set(members.tolist()))
        pos = {r: j for j, r in enumerate(cols)}
        planes = []
        for c in HOURLY_COLS:
            a = np.zeros((nh, len(cols)), dtype=np.float64)
            for j, r in enumerate(cols):                                # _arr(), :173-175
                v = np.asarray(df[c].iat[r], dtype=float).ravel()
                k = min(v.size, nh)
                a[:k, j] = v[:k]
            planes.append(torch.from_numpy(a).to(eng.dev))
        wsub = tuple(t[torch.as_tensor(cols, dtype=torch.int64, device=eng.dev)] for t in w)
        res = state_hourly(eng, planes, wsub, [pos[r] for r in members], so).cpu().numpy()
        for j, s in enumerate(sids):
            out_rows[s] = res[j]
    records = [{"state_abbr": states[s], "year": int(year), "n_hours": int(nh_state[s]),
                "net_sum": out_rows[s].tolist()} for s in range(len(states))]
    if not records:
        return None
    rec = pd.DataFrame.from_records(records)
    if writer is not None:
        writer(rec, engine, schema, owner, "state_hourly_agg", if_exists="append",
               append_transformations=False)
    return rec


def state_hourly_from_outputs(engine, out, perm, state_abbr, customers_in_bin, number_of_adopters,
                              batt_kw_cum_last_year, batt_kw, added):
    """Per-state hourly sums straight from dgen_size_agents' device hourly
    planes (out["baseline"/"net_pvonly"/"net_with_batt"], tiled [2190, n, 4], device
    order `perm` = AgentBatch.perm or None).  Host columns are in caller order.
    Returns ([S, 8760] float64 device tensor in MW, state keys)."""
    import torch
    eng = _engine(engine)
    n = len(state_abbr)
    idx, seg_off, states = group_segments(list(state_abbr))
    inv = np.arange(n, dtype=np.int64)
    if perm is not None:
        inv = np.empty(n, dtype=np.int64)
        inv[np.asarray(perm, dtype=np.int64)] = np.arange(n, dtype=np.int64)
    # weights per device column
    g = (lambda a: np.asarray(a)[np.asarray(perm)]) if perm is not None else (lambda a: np.asarray(a))
    w = export_weights(eng, g(customers_in_bin), g(number_of_adopters), g(batt_kw_cum_last_year),
                       g(batt_kw), g(np.asarray(added, np.int64)))
    planes = (out["baseline"], out["net_pvonly"], out["net_with_batt"])
    if any(p is None for p in planes):
        raise ValueError("state_hourly_from_outputs: the sizing ran without hourly outputs")
    return state_hourly(eng, planes, w, inv[idx], seg_off), states
