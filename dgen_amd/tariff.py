"""Host-side tariff compiler.

Restates, field for field, what the reference does to a URDB-style tariff
before PySAM sees it (tsgsteele/dgen @ 2025-09-19):

* ``normalize_tariff``  -- financial_functions.py:962-1007 and its helpers
  (_parse_tariff_dict :655, _num :674, _coerce_bool :685, _plus1_sched :699,
  _sched_12x24 :719, _mat2d :738, _list1d_8760 :751, _build_ur_ec_from_e_parts
  :763, _build_ur_dc_from_d_parts :793, _reconcile_periods_and_equalize_tiers
  :830, _harmonize_tier_caps_and_units :919);
* ``process_tariff``    -- financial_functions.py:575-648 (the
  Utilityrate5.ElectricityRates fields it writes);
* the California NEM3 override (ff:180-191, 244-255, 371-381).

The reference re-runs this on every objective evaluation (ff:248); here it runs
once per distinct (tariff, CA?) pair and the result is packed into the
``dgen_tariff`` record the kernels read.  The quirks are kept on purpose and are
pinned by tests/golden/tariffs.json (bit-exact, float32 rounding included):
period ids remapped in the matrix but not in the schedules (ids > P clamp to 1),
one cap per tier (the smallest finite one), unit code = the mode, BIG = 1e38.

Demand charges (extension mode).  The reference compiles the ``ur_dc_*`` mats
but never passes them (SKIP_DEMAND_CHARGES = True, ff:35,601-603).  With
``skip_demand_charges=False`` the compiler takes process_tariff's other branch
(ff:604-615; its field output is pinned by tests/golden/tariffs_dc.json,
captured from the reference with the switch flipped) and packs the mats into a
``dgen_demand`` record (include/dgen_hip.h) that the kernels bill.  The SSC
demand arithmetic itself is parity unpinned.
"""
from __future__ import annotations

import ast
import json
from collections import OrderedDict
import re
from dataclasses import dataclass
from typing import Any, Dict, Iterable, List, Optional, Tuple

import numpy as np

BIG = 1e38
BIG_THRESH = 1e37
MAXP = 12
MAXT = 6

# financial_functions.py:35,38 module switches (reference values)
SKIP_DEMAND_CHARGES = True
FORCE_NET_BILLING = False

_UNIT_CODES = {"kWh": 0, "kWh/kW": 1, "kWh daily": 2, "kWh/kW daily": 3}
_NULLISH = re.compile(r"\b(nan|none|null)\b", flags=re.IGNORECASE)


# ----------------------------------------------------------------------------
# scalar / shape coercions
# ----------------------------------------------------------------------------
def parse_tariff(raw) -> Dict[str, Any]:
    """dict passes through; a string is read as JSON after quote / null
    normalisation, else as a Python literal; anything else is {} (ff:655)."""
    if isinstance(raw, dict):
        return raw
    if not isinstance(raw, str):
        return {}
    text = _NULLISH.sub("null", raw.replace("'", '"'))
    try:
        return json.loads(text)
    except json.JSONDecodeError:
        pass
    try:
        return ast.literal_eval(raw)
    except Exception:
        return {}


def as_number(x, default: float = 0.0) -> float:
    """float(x) with None / '' / 'nan' / 'none' / 'null' / failures -> default."""
    if x is None:
        return default
    if isinstance(x, str) and x.strip().lower() in ("", "nan", "none", "null"):
        return default
    try:
        return float(x)
    except Exception:
        return default


def as_flag(x, default=False) -> bool:
    if isinstance(x, bool):
        return x
    if isinstance(x, (int, float)):
        return bool(int(x))
    if isinstance(x, str):
        return x.strip().lower() in ("1", "true", "t", "yes", "y")
    return bool(default)


def _ones_12x24() -> List[List[int]]:
    return [[1] * 24 for _ in range(12)]


def legacy_schedule(mat) -> List[List[int]]:
    """0-based legacy 12x24 -> 1-based, ragged rows padded with 0 (-> 1)."""
    if not mat:
        return _ones_12x24()
    out = []
    for r in range(12):
        row = mat[r] if r < len(mat) else []
        fixed = []
        for col in range(24):
            v = row[col] if col < len(row) else 0
            try:
                fixed.append(int(v) + 1)
            except Exception:
                fixed.append(1)
        out.append(fixed)
    return out


def fit_12x24(x) -> List[List[int]]:
    """Strict 12x24 int schedule: exact, trimmed, zero-padded, else zeros."""
    zeros = [[0] * 24 for _ in range(12)]
    if x is None:
        return zeros
    a = np.asarray(x)
    if a.ndim != 2:
        return zeros
    r, c = a.shape
    if (r, c) == (12, 24):
        return a.astype(np.int32, copy=False).tolist()
    if r >= 12 and c >= 24:
        return a[:12, :24].astype(np.int32, copy=False).tolist()
    if r <= 12 and c <= 24:
        z = np.zeros((12, 24), dtype=np.int32)
        z[:r, :c] = np.asarray(a, dtype=np.int32)
        return z.tolist()
    return zeros


def small_f32_matrix(x, size_limit: int = 4096) -> List[List[float]]:
    """2-D, non-empty, <= size_limit, all finite -> float32-rounded rows; else []."""
    if x is None or x == []:
        return []
    a = np.asarray(x)
    if a.ndim != 2 or a.size == 0 or a.size > size_limit:
        return []
    if not np.isfinite(a.astype(np.float64, copy=False)).all():
        return []
    return a.astype(np.float32, copy=False).tolist()


def series_8760(x: Optional[Iterable[float]]) -> Optional[List[float]]:
    """float32-rounded 8760 series if finite and exactly 8760 long, else None."""
    if x is None:
        return None
    try:
        a = np.asarray(x, dtype=np.float32).ravel()
    except Exception:
        return None
    if a.size != 8760 or not np.isfinite(a).all():
        return None
    return a.tolist()


# ----------------------------------------------------------------------------
# legacy (e_* / d_*) structures
# ----------------------------------------------------------------------------
def legacy_energy_rows(td: Dict[str, Any], sell: float = 0.0) -> List[List[float]]:
    """e_prices[tier][period] (+ e_levels) -> [period, tier, cap, unit, buy, sell]."""
    prices = td.get("e_prices") or []
    if not prices:
        return []
    levels = td.get("e_levels") or []
    n_tier = len(prices)
    n_per = len(prices[0]) if n_tier else 0
    if (not levels) or len(levels) != n_tier or any(len(lv) != n_per for lv in levels):
        levels = [[BIG] * n_per for _ in range(n_tier)]
    unit = _UNIT_CODES.get(str(td.get("energy_rate_unit", "kWh")), 0)
    return [[float(p + 1), float(t + 1), float(levels[t][p]), float(unit), float(prices[t][p]),
             float(sell)]
            for p in range(n_per) for t in range(n_tier)]


def _legacy_dc_block(levels, prices) -> List[List[float]]:
    n_tier = len(levels)
    n_per = len(levels[0]) if n_tier else 0
    return [[p + 1, t + 1, float(levels[t][p]), float(prices[t][p])]
            for p in range(n_per) for t in range(n_tier)]


def legacy_demand(td: Dict[str, Any]) -> Tuple[Dict[str, Any], int]:
    out: Dict[str, Any] = {"ur_dc_flat_mat": [], "ur_dc_tou_mat": []}
    fl, fp = td.get("d_flat_levels") or [], td.get("d_flat_prices") or []
    if fl and fp:
        out["ur_dc_flat_mat"] = _legacy_dc_block(fl, fp)
    tl, tp = td.get("d_tou_levels") or [], td.get("d_tou_prices") or []
    if tl and tp:
        out["ur_dc_tou_mat"] = _legacy_dc_block(tl, tp)
    out["ur_dc_sched_weekday"] = legacy_schedule(td.get("ur_dc_sched_weekday") or td.get("d_wkday_12by24"))
    out["ur_dc_sched_weekend"] = legacy_schedule(td.get("ur_dc_sched_weekend") or td.get("d_wkend_12by24"))
    enable = 1 if (out["ur_dc_flat_mat"] or out["ur_dc_tou_mat"] or as_flag(td.get("d_flat_exists"))
                   or as_flag(td.get("d_tou_exists"))) else 0
    return out, enable


# ----------------------------------------------------------------------------
# matrix reconciliation
# ----------------------------------------------------------------------------
def _clamp_schedule(s: np.ndarray, P: Optional[int]) -> List[List[int]]:
    s = np.asarray(fit_12x24(s.tolist()), dtype=int)
    s[s < 1] = 1
    if P is not None:
        s[s > P] = 1
    return s.tolist()


def reconcile_periods(ec_rows, wk, we):
    """Periods -> contiguous 1..P in the matrix; every period padded to the max
    tier count with BIG-cap clones of its last tier; schedules fitted to 12x24
    and ids outside 1..P set to 1 (NOT remapped, ff:906-913)."""
    tou = np.asarray(ec_rows or [], dtype=float)
    wk_a = np.asarray(wk or [], dtype=int)
    we_a = np.asarray(we or [], dtype=int)
    if tou.size == 0:
        return [], _clamp_schedule(wk_a, None), _clamp_schedule(we_a, None)

    old_ids = np.unique(tou[:, 0].astype(int))
    if old_ids.size == 0:
        tou[:, 0] = 1
        old_ids = np.array([1], dtype=int)
    lookup = {int(o): k + 1 for k, o in enumerate(old_ids.tolist())}
    tou[:, 0] = np.vectorize(lambda v: lookup.get(int(v), 1))(tou[:, 0])

    groups: Dict[int, np.ndarray] = {}
    max_tiers = 0
    for p in np.unique(tou[:, 0].astype(int)):
        rows = tou[tou[:, 0] == p]
        rows = rows[np.argsort(rows[:, 1])]
        groups[int(p)] = rows
        max_tiers = max(max_tiers, np.unique(rows[:, 1].astype(int)).size)

    blocks = []
    for p in sorted(groups):
        rows = groups[p]
        n_have = np.unique(rows[:, 1].astype(int)).size
        if n_have == max_tiers:
            for k in range(rows.shape[0]):
                rows[k, 1] = float(k + 1)
            blocks.append(rows)
            continue
        last = rows[-1]
        unit = last[3] if rows.shape[1] >= 4 else 0.0
        price = last[4] if rows.shape[1] >= 5 else 0.0
        sell = last[5] if rows.shape[1] >= 6 else 0.0
        padded = [r.copy() for r in rows]
        for t in range(n_have + 1, max_tiers + 1):
            padded.append(np.array([float(p), float(t), BIG, float(unit), float(price), float(sell)]))
        padded = np.vstack(padded)
        padded = padded[np.argsort(padded[:, 1])]
        for k in range(padded.shape[0]):
            padded[k, 1] = float(k + 1)
        blocks.append(padded)

    fixed = np.vstack(blocks)
    P = int(np.max(fixed[:, 0]).astype(int))
    wk_out = _clamp_schedule(wk_a, P)
    we_out = _clamp_schedule(we_a, P)
    fixed = fixed[np.lexsort((fixed[:, 1], fixed[:, 0]))]
    return fixed.astype(np.float32).tolist(), wk_out, we_out


def harmonize_caps(ec_rows) -> List[List[float]]:
    """One cap per tier (smallest finite positive cap across periods, else BIG),
    one unit code (the mode, ties -> smallest), rows sorted, float32-rounded."""
    if not ec_rows:
        return []
    tou = np.asarray(ec_rows, dtype=float)
    if tou.ndim != 2 or tou.shape[1] < 6:
        return []
    units = tou[:, 3].astype(int)
    shift = max(0, -int(units.min()))
    mode = int(np.argmax(np.bincount(units + shift)) - shift)
    for t in np.unique(tou[:, 1].astype(int)):
        sel = tou[:, 1].astype(int) == t
        caps = tou[sel, 2]
        finite = caps[(caps > 0) & (caps < BIG_THRESH)]
        tou[sel, 2] = float(np.min(finite)) if finite.size else float(BIG)
    tou[:, 3] = float(mode)
    tou = tou[np.lexsort((tou[:, 1], tou[:, 0]))]
    return tou.astype(np.float32).tolist()


# ----------------------------------------------------------------------------
# public: normalize / process
# ----------------------------------------------------------------------------
def normalize_tariff(raw, net_sell_rate_scalar=0.0, debug=False) -> Dict[str, Any]:
    """financial_functions.normalize_tariff (ff:962-1007)."""
    td = parse_tariff(raw)
    out: Dict[str, Any] = {}
    out["en_electricity_rates"] = int(td.get("en_electricity_rates", 1))
    mo_in = int(td.get("ur_metering_option", 0))
    out["ur_metering_option"] = 2 if FORCE_NET_BILLING else mo_in
    out["ur_monthly_fixed_charge"] = as_number(td.get("ur_monthly_fixed_charge",
                                                      td.get("fixed_charge", 0.0)), 0.0)
    ec = td.get("ur_ec_tou_mat") or legacy_energy_rows(td, net_sell_rate_scalar)
    wk = td.get("ur_ec_sched_weekday") or legacy_schedule(td.get("e_wkday_12by24")) or _ones_12x24()
    we = td.get("ur_ec_sched_weekend") or legacy_schedule(td.get("e_wkend_12by24")) or _ones_12x24()
    ec, wk, we = reconcile_periods(ec, wk, we)
    ec = harmonize_caps(ec)
    out["ur_ec_tou_mat"] = ec
    out["ur_ec_sched_weekday"] = wk
    out["ur_ec_sched_weekend"] = we
    dc, dc_guess = legacy_demand(td)
    out["ur_dc_flat_mat"] = td.get("ur_dc_flat_mat") or dc["ur_dc_flat_mat"] or []
    out["ur_dc_tou_mat"] = td.get("ur_dc_tou_mat") or dc["ur_dc_tou_mat"] or []
    out["ur_dc_sched_weekday"] = (td.get("ur_dc_sched_weekday") or dc["ur_dc_sched_weekday"]
                                  or _ones_12x24())
    out["ur_dc_sched_weekend"] = (td.get("ur_dc_sched_weekend") or dc["ur_dc_sched_weekend"]
                                  or _ones_12x24())
    out["ur_dc_enable"] = int(td.get("ur_dc_enable", dc_guess))
    out["ur_enable_billing_demand"] = bool(td.get("ur_enable_billing_demand", False))
    return out


def rate_fields(td: Dict[str, Any], net_billing_sell_rate=0.0, ts_sell_rate=None,
                ts_buy_rate=None, skip_demand_charges: Optional[bool] = None) -> Dict[str, Any]:
    """The ElectricityRates fields process_tariff (ff:575-648) writes, as a dict
    in write order.  ``skip_demand_charges`` None = the reference's module
    switch (ff:35)."""
    skip_dc = SKIP_DEMAND_CHARGES if skip_demand_charges is None else bool(skip_demand_charges)
    f: Dict[str, Any] = {}
    mo_in = int(td.get("ur_metering_option", 0))
    mo = 2 if FORCE_NET_BILLING else mo_in
    f["ur_metering_option"] = mo
    f["ur_monthly_fixed_charge"] = float(td.get("ur_monthly_fixed_charge", 0.0))
    f["ur_annual_min_charge"] = 0.0
    f["ur_monthly_min_charge"] = 0.0
    flat_raw, tou_raw = td.get("ur_dc_flat_mat"), td.get("ur_dc_tou_mat")
    dc_on = bool(td.get("ur_dc_enable", 0)) or bool(flat_raw) or bool(tou_raw)
    if skip_dc or not dc_on:
        f["ur_dc_enable"] = 0
        f["ur_enable_billing_demand"] = 0
    else:   # ff:604-615 (extension mode)
        flat, tou = small_f32_matrix(flat_raw), small_f32_matrix(tou_raw)
        enable = bool(flat) or bool(tou)
        f["ur_dc_sched_weekday"] = fit_12x24(td.get("ur_dc_sched_weekday"))
        f["ur_dc_sched_weekend"] = fit_12x24(td.get("ur_dc_sched_weekend"))
        f["ur_dc_flat_mat"] = flat if enable else []
        f["ur_dc_tou_mat"] = tou if enable else []
        f["ur_enable_billing_demand"] = 0
        f["ur_dc_enable"] = int(enable)
    ec = td.get("ur_ec_tou_mat")
    if ec:
        f["ur_ec_tou_mat"] = small_f32_matrix(ec)
        f["ur_ec_sched_weekday"] = fit_12x24(td.get("ur_ec_sched_weekday"))
        f["ur_ec_sched_weekend"] = fit_12x24(td.get("ur_ec_sched_weekend"))
    if mo == 2:
        sell = series_8760(ts_sell_rate)
        if sell is not None:
            f["ur_en_ts_sell_rate"] = 1
            f["ur_ts_sell_rate"] = sell
        else:
            f["ur_en_ts_sell_rate"] = 0
            f["ur_ts_sell_rate"] = [0.0]
        buy = series_8760(ts_buy_rate)
        if buy is not None:
            f["ur_en_ts_buy_rate"] = 1
            f["ur_ts_buy_rate"] = buy
        else:
            f["ur_en_ts_buy_rate"] = 0
    else:
        f["ur_en_ts_sell_rate"] = 0
        f["ur_ts_sell_rate"] = [0.0]
        f["ur_en_ts_buy_rate"] = 0
    return f


def process_tariff(utilityrate, tariff_dict, net_billing_sell_rate, ts_sell_rate=None,
                   ts_buy_rate=None, skip_demand_charges: Optional[bool] = None):
    """Drop-in for financial_functions.process_tariff: writes the fields onto
    ``utilityrate.ElectricityRates`` (any attribute bag) and returns it."""
    er = utilityrate.ElectricityRates
    for k, v in rate_fields(tariff_dict, net_billing_sell_rate, ts_sell_rate, ts_buy_rate,
                            skip_demand_charges).items():
        setattr(er, k, v)
    return utilityrate


def apply_ca_nem3(td: Dict[str, Any]) -> Dict[str, Any]:
    """ff:186-191: CA sell column = 0.25 x buy, metering option 2."""
    if td.get("ur_ec_tou_mat"):
        tou = np.asarray(td["ur_ec_tou_mat"], dtype=float)
        if tou.ndim == 2 and tou.shape[1] >= 6:
            tou[:, 5] = tou[:, 4] * 0.25
            td["ur_ec_tou_mat"] = tou.tolist()
    td["ur_metering_option"] = 2
    return td


# ----------------------------------------------------------------------------
# device record
# ----------------------------------------------------------------------------
TARIFF_DTYPE = np.dtype([
    ("P", "<i4"), ("T", "<i4"), ("mo", "<i4"), ("unit", "<i4"), ("fixed", "<f8"),
    ("cap", "<f8", (MAXT,)), ("buy", "<f8", (MAXP, MAXT)), ("sell", "<f8", (MAXP, MAXT)),
    ("wkday", "u1", (12, 24)), ("wkend", "u1", (12, 24)), ("flags", "<i4"), ("dc", "<i4"),
])
assert TARIFF_DTYPE.itemsize == 1808

# dgen_demand (include/dgen_hip.h): demand-charge mats of one tariff
DCP = 8     # TOU demand periods
DCT = 4     # demand tiers
DEMAND_DTYPE = np.dtype([
    ("tou_nt", "<i4", (DCP,)), ("flat_nt", "<i4", (12,)), ("flags", "<i4"), ("pad", "<i4"),
    ("tou_cap", "<f8", (DCP, DCT)), ("tou_price", "<f8", (DCP, DCT)),
    ("flat_cap", "<f8", (12, DCT)), ("flat_price", "<f8", (12, DCT)),
    ("wkday", "u1", (12, 24)), ("wkend", "u1", (12, 24)),
])
assert DEMAND_DTYPE.itemsize == 1944

ST_EMPTY_EC = 0x04
ST_UNIT = 0x08
ST_DEMAND = 0x80


class TariffError(ValueError):
    pass


def peak_only_record() -> np.ndarray:
    """A demand record with no charges and one demand period (every hour in
    period 0): the month peaks of a tariff whose tiers are in kWh/kW (unit
    codes 1 and 3, SSC scales those caps by the month's peak import) come from
    the demand machinery's flat peak, whether or not demand charges are billed."""
    return np.zeros((), dtype=DEMAND_DTYPE)


def attach_peak_records(records: np.ndarray, demand: Optional[np.ndarray]):
    """(records, demand) with every kWh/kW-tier tariff that has no demand record
    pointing at one shared peak_only_record (appended), and whether any tariff
    bills its tiers in kWh/kW (dgen_tables.peak_units)."""
    recs = np.array(records, dtype=TARIFF_DTYPE, copy=True)
    dem = np.zeros(0, DEMAND_DTYPE) if demand is None else np.ascontiguousarray(demand, DEMAND_DTYPE)
    pk = (recs["unit"] == 1) | (recs["unit"] == 3)
    need = pk & (recs["dc"] == 0)
    if need.any():
        dem = np.concatenate([dem, peak_only_record()[None]])
        recs["dc"][need] = dem.size
    return recs, dem, bool(pk.any())


@dataclass
class CompiledTariff:
    fields: Dict[str, Any]          # ElectricityRates fields (ts variant: no TS series)
    record: np.ndarray              # one TARIFF_DTYPE element
    demand: Optional[np.ndarray] = None   # one DEMAND_DTYPE element (demand charges on)


def pack_record(fields: Dict[str, Any]) -> np.ndarray:
    """ElectricityRates energy fields -> dgen_tariff record."""
    rec = np.zeros((), dtype=TARIFF_DTYPE)
    rec["mo"] = int(fields["ur_metering_option"])
    rec["fixed"] = float(fields["ur_monthly_fixed_charge"])
    mat = fields.get("ur_ec_tou_mat") or []
    flags = 0
    if rec["mo"] not in (0, 1, 2, 3, 4):
        # SAM's ur_metering_option enumeration (the reference passes the
        # tariff's value through to Utilityrate5, ff:586-588, 970-971)
        raise TariffError(f"metering option {int(rec['mo'])} is not one of SAM's options 0-4")
    if not mat:
        flags |= ST_EMPTY_EC
        rec["P"], rec["T"] = 1, 1
        rec["cap"][0] = BIG
        wk = we = [[1] * 24] * 12
    else:
        m = np.asarray(mat, dtype=np.float64)
        P = int(m[:, 0].max())
        T = int(m[:, 1].max())
        if P > MAXP or T > MAXT:
            raise TariffError(f"tariff with {P} periods x {T} tiers exceeds {MAXP}x{MAXT}")
        if m.shape[0] != P * T:
            raise TariffError("tariff matrix is not a complete period x tier grid")
        rec["P"], rec["T"] = P, T
        unit = int(m[0, 3])
        if unit not in (0, 1, 2, 3):
            flags |= ST_UNIT
        rec["unit"] = unit
        for row in m:
            p, t = int(row[0]) - 1, int(row[1]) - 1
            rec["cap"][t] = row[2]
            rec["buy"][p, t] = row[4]
            rec["sell"][p, t] = row[5]
        wk = fields["ur_ec_sched_weekday"]
        we = fields["ur_ec_sched_weekend"]
    P = int(rec["P"])
    for name, sched in (("wkday", wk), ("wkend", we)):
        s = np.asarray(sched, dtype=np.int64).reshape(12, 24)
        s = np.where((s < 1) | (s > P), 1, s)
        rec[name] = (s - 1).astype(np.uint8)
    rec["flags"] = flags
    return rec


def _dc_tiers(rows: np.ndarray, n_groups: int, cap: np.ndarray, price: np.ndarray,
              nt: np.ndarray, group_base: int) -> int:
    """Rows [group, tier, max kW, $/kW] -> per-group tier arrays.  SSC reads the
    group column as a 0-based month (flat mat) or a 1-based period (TOU mat) and
    tiers 1..k; the last tier of a group is unbounded above.  Returns
    ST_DEMAND when a row falls outside the record's limits."""
    flags = 0
    seen: Dict[int, Dict[int, Tuple[float, float]]] = {}
    for r in rows:
        if r.shape[0] < 4:
            return ST_DEMAND
        g, t = int(r[0]) - group_base, int(r[1]) - 1
        if not (0 <= g < n_groups) or not (0 <= t < DCT):
            flags |= ST_DEMAND
            continue
        seen.setdefault(g, {})[t] = (float(r[2]), float(r[3]))
    for g, tiers in seen.items():
        k = max(tiers) + 1
        if sorted(tiers) != list(range(k)):
            flags |= ST_DEMAND          # a gap in the tier numbers
            continue
        nt[g] = k
        for t, (c, pr) in tiers.items():
            cap[g, t] = c
            price[g, t] = pr
    return flags


def pack_demand(fields: Dict[str, Any]) -> Optional[np.ndarray]:
    """ElectricityRates demand fields (ff:604-615) -> dgen_demand record, or
    None when demand charges are off for the tariff."""
    if not int(fields.get("ur_dc_enable", 0)):
        return None
    rec = np.zeros((), dtype=DEMAND_DTYPE)
    flags = 0
    flat = np.asarray(fields.get("ur_dc_flat_mat") or [], dtype=np.float64)
    tou = np.asarray(fields.get("ur_dc_tou_mat") or [], dtype=np.float64)
    if flat.size:
        flags |= _dc_tiers(flat.reshape(flat.shape[0], -1), 12, rec["flat_cap"], rec["flat_price"],
                           rec["flat_nt"], 0)
    if tou.size:
        flags |= _dc_tiers(tou.reshape(tou.shape[0], -1), DCP, rec["tou_cap"], rec["tou_price"],
                           rec["tou_nt"], 1)
    for name, key in (("wkday", "ur_dc_sched_weekday"), ("wkend", "ur_dc_sched_weekend")):
        s = np.asarray(fit_12x24(fields.get(key)), dtype=np.int64).reshape(12, 24)
        if tou.size and ((s < 1) | (s > DCP)).any():
            flags |= ST_DEMAND          # SSC rejects a schedule period outside 1..n
        rec[name] = (np.clip(s, 1, DCP) - 1).astype(np.uint8)
    rec["flags"] = flags
    return rec


def compile_tariff(raw, is_ca: bool, skip_demand_charges: Optional[bool] = None) -> CompiledTariff:
    """normalize_tariff -> CA NEM3 -> process_tariff -> device record(s)."""
    td = normalize_tariff(raw, net_sell_rate_scalar=0.0)
    if is_ca:
        td = apply_ca_nem3(td)
    fields = rate_fields(td, 0.0, ts_sell_rate=None, skip_demand_charges=skip_demand_charges)
    rec = pack_record(fields)
    dem = pack_demand(fields)
    if dem is not None:
        rec["flags"] = int(rec["flags"]) | int(dem["flags"])
    return CompiledTariff(fields=fields, record=rec, demand=dem)


def tariff_key(raw) -> str:
    if isinstance(raw, str):
        return "s:" + raw
    try:
        return "j:" + json.dumps(raw, sort_keys=True, default=repr)
    except Exception:
        return "r:" + repr(raw)


_COMPILE_CACHE: "OrderedDict[Tuple[str, bool, Any], CompiledTariff]" = OrderedDict()
_COMPILE_CACHE_MAX = 8192


def _compiled(raw, key: str, is_ca: bool, skip_demand_charges) -> CompiledTariff:
    """compile_tariff, memoised across tables by the tariff's content (a chunk
    loop meets the same tariffs call after call): a copy of the records, so a
    table may set its own `dc`."""
    ck = (key if key[:2] in ("s:", "j:", "r:") else tariff_key(raw), is_ca, skip_demand_charges)
    ct = _COMPILE_CACHE.get(ck)
    if ct is None:
        ct = compile_tariff(raw, is_ca, skip_demand_charges)
        _COMPILE_CACHE[ck] = ct
        if len(_COMPILE_CACHE) > _COMPILE_CACHE_MAX:
            _COMPILE_CACHE.popitem(last=False)
    else:
        _COMPILE_CACHE.move_to_end(ck)
    return CompiledTariff(fields=ct.fields, record=ct.record.copy(),
                          demand=None if ct.demand is None else ct.demand.copy())


class TariffTable:
    """Deduplicating table of compiled tariffs (one entry per (tariff, CA?)).
    With demand charges on, tariffs that carry them get a ``dgen_demand``
    record; the tariff record's ``dc`` field is 1 + its index (0 = none)."""

    def __init__(self, skip_demand_charges: Optional[bool] = None):
        self._index: Dict[Tuple[str, bool], int] = {}
        self.records: List[np.ndarray] = []
        self.demand: List[np.ndarray] = []
        self.raw: List[Any] = []
        self.skip_demand_charges = skip_demand_charges

    def add(self, raw, is_ca: bool, key: Optional[str] = None) -> int:
        """Index of the compiled (raw, is_ca) tariff; `key` overrides the
        content key (rate-switch rows get one entry each)."""
        key = (key if key is not None else tariff_key(raw), bool(is_ca))
        hit = self._index.get(key)
        if hit is not None:
            return hit
        ct = _compiled(raw, key[0], bool(is_ca), self.skip_demand_charges)
        if ct.demand is not None:
            self.demand.append(ct.demand)
            ct.record["dc"] = len(self.demand)
        idx = len(self.records)
        self._index[key] = idx
        self.records.append(ct.record)
        self.raw.append(raw)
        return idx

    def __len__(self):
        return len(self.records)

    def array(self) -> np.ndarray:
        if not self.records:
            return np.zeros(0, dtype=TARIFF_DTYPE)
        return np.stack(self.records).astype(TARIFF_DTYPE)

    def demand_array(self) -> np.ndarray:
        if not self.demand:
            return np.zeros(0, dtype=DEMAND_DTYPE)
        return np.stack(self.demand).astype(DEMAND_DTYPE)
