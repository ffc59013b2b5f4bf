"""Agent rows -> structure-of-arrays columns for the device.

Replaces the per-row work the reference does inside
``calc_system_size_and_performance`` before any arithmetic
(financial_functions.py:330-421): profile lookup (elec.py:508-558), tariff
normalisation (ff:374-382, re-done per evaluation in the reference), the rate
switch table filter (elec.py:840-847) and the finance-column reads.
"""
from __future__ import annotations

import hashlib
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd

from . import _lib
from .engine import SWITCH_DTYPE
from .tariff import TariffTable, series_8760


def _is_ca(state) -> bool:
    return str(state if state is not None else "").upper() == "CA"


class SwitchIndex:
    """rate_switch_lkup rows grouped by (tech, eia_id, res_com), expanded per
    agent into device candidate lists.  Every row gets its own tariff-table
    entry so that the final tariff index identifies the row (tariff_id)."""

    def __init__(self, table, tariffs: TariffTable):
        self.tariffs = tariffs
        self.groups: Dict[Tuple[Any, Any, Any], List[dict]] = {}
        self.rows: List[np.ndarray] = []
        self.row_of_tariff: Dict[int, dict] = {}
        self._cache: Dict[Tuple, Tuple[int, int]] = {}
        self._n = 0
        if table is not None and len(table):
            recs = table.to_dict(orient="records")
            for k, r in enumerate(recs):
                r = dict(r)
                r["_row"] = k
                key = (r.get("tech"), r.get("eia_id"), r.get("res_com"))
                self.groups.setdefault(key, []).append(r)

    def _lookup(self, tech, eia_id, res_com) -> List[dict]:
        try:
            return self.groups.get((tech, eia_id, res_com), [])
        except TypeError:      # unhashable eia_id
            return []

    def candidates(self, tech: str, eia_id, sector_abbr, is_ca: bool) -> Tuple[int, int]:
        res_com = str(sector_abbr).upper()[0]
        ckey = (tech, eia_id, res_com, is_ca)
        try:
            hit = self._cache.get(ckey)
        except TypeError:          # unhashable eia_id
            ckey = (tech, repr(eia_id), res_com, is_ca)
            hit = self._cache.get(ckey)
        if hit is not None:
            return hit
        rows = self._lookup(tech, eia_id, res_com)
        off = self._n
        for r in rows:
            tix = self.tariffs.add(r["json"], is_ca, key=f"switch-row:{r['_row']}")
            rec = np.zeros((), dtype=SWITCH_DTYPE)
            rec["min_kw"] = float(r["min_kw_limit"])
            rec["max_kw"] = float(r["max_kw_limit"])
            rec["one_time_charge"] = float(r["one_time_charge"])
            rec["tariff"] = tix
            self.rows.append(rec)
            self.row_of_tariff[tix] = r
            self._n += 1
        res = (off, len(rows))
        self._cache[ckey] = res
        return res

    def array(self) -> np.ndarray:
        if not self.rows:
            return np.zeros(0, dtype=SWITCH_DTYPE)
        return np.stack(self.rows).astype(SWITCH_DTYPE)


class WholesaleIndex:
    """Deduplicates the per-agent 8760 wholesale_prices arrays (per county)."""

    def __init__(self):
        self.rows: List[np.ndarray] = []
        self._index: Dict[bytes, int] = {}

    def add(self, arr, mult: float) -> int:
        if arr is None:
            return -1
        try:
            a = np.asarray(arr, dtype=np.float64).ravel()
        except Exception:
            return -1
        # ff:182 np.asarray(...).ravel() * mult, then _list1d_8760 (f32, finite, 8760)
        if series_8760(a * mult) is None:
            return -1
        key = hashlib.blake2b(a.tobytes(), digest_size=16).digest()
        k = self._index.get(key)
        if k is None:
            k = len(self.rows)
            self._index[key] = k
            self.rows.append(a)
        return k

    def add_frame(self, arrs: Sequence, mult: np.ndarray, skip: np.ndarray) -> np.ndarray:
        """add() over a whole frame column at once: conversion, finiteness scan
        and content hash once per distinct array object (rows share them), the
        per-row validity (arr * mult finite in float32 -- series_8760 -- which
        follows from the largest |x|, |x * mult| being monotone in |x|)
        vectorised, and table rows entered in the order of their first valid
        use, exactly as add() row by row.  skip: rows that take -1 (CA)."""
        n = len(arrs)
        obj: Dict[int, int] = {}          # id(array object) -> distinct-object index
        ckey: List[int] = []              # distinct object -> content index (-1: invalid)
        cmax: List[float] = []
        contents: Dict[bytes, int] = {}
        carr: List[np.ndarray] = []
        oix = np.empty(n, np.int64)
        for i, arr in enumerate(arrs):
            k = obj.get(id(arr))
            if k is None:
                k = obj[id(arr)] = len(ckey)
                c, mx = -1, 0.0
                if arr is not None:
                    try:
                        v = np.asarray(arr, dtype=np.float64).ravel()
                    except Exception:
                        v = None
                    if v is not None and v.size == 8760 and bool(np.isfinite(v).all()):
                        h = hashlib.blake2b(v.tobytes(), digest_size=16).digest()
                        c = contents.get(h)
                        if c is None:
                            c = contents[h] = len(carr)
                            carr.append(v)
                        mx = float(np.abs(v).max())
                ckey.append(c)
                cmax.append(mx)
            oix[i] = k
        ck = np.asarray(ckey, np.int64)[oix] if n else np.zeros(0, np.int64)
        mxr = np.asarray(cmax, np.float64)[oix] if n else np.zeros(0)
        with np.errstate(over="ignore", invalid="ignore"):
            ok = (ck >= 0) & ~np.asarray(skip, bool) & np.isfinite(mult) & \
                np.isfinite((mxr * np.abs(mult)).astype(np.float32))
        out = np.full(n, -1, np.int64)
        if ok.any():
            rows = np.nonzero(ok)[0]
            u, first = np.unique(ck[rows], return_index=True)
            order = np.argsort(first, kind="stable")          # first valid use
            slot = np.empty(int(u.max()) + 1, np.int64)
            key_of = {c: h for h, c in contents.items()}
            for c in u[order].tolist():
                h = key_of[c]
                k = self._index.get(h)
                if k is None:
                    k = self._index[h] = len(self.rows)
                    self.rows.append(carr[c])
                slot[c] = k
            out[rows] = slot[ck[rows]]
        return out

    def array(self) -> Optional[np.ndarray]:
        return np.stack(self.rows) if self.rows else None


def empty_columns(n: int) -> Dict[str, np.ndarray]:
    return {name: np.zeros(n, dtype=dt) for name, dt in _lib.AGENT_COLUMNS}


class PopulationBuilder:
    """Accumulates agents into SoA columns + the tables they index."""

    def __init__(self, switch_table=None, skip_demand_charges: Optional[bool] = None):
        """skip_demand_charges: None/True = the reference (ff:35); False =
        extension mode (tariffs with demand charges get dgen_demand records)."""
        self.tariffs = TariffTable(skip_demand_charges)
        self.switches = SwitchIndex(switch_table, self.tariffs)
        self.wholesale = WholesaleIndex()
        self.rows: List[Dict[str, Any]] = []

    def add(self, *, load_row: int, cf_row: int, sector_abbr, state_abbr, eia_id, tariff_dict,
            wholesale, load_kwh, price_mult, econ_life, loan_term, inflation, pv_deg, escalator,
            down_payment, tax_rate, real_discount, itc_frac, capex, capex_combined, batt_capex_kwh,
            ccm, vor) -> int:
        is_ca = _is_ca(state_abbr)
        is_res = sector_abbr == "res"
        t0 = self.tariffs.add(tariff_dict, is_ca)
        so, sc = self.switches.candidates("solar", eia_id, sector_abbr, is_ca)
        to, tc = self.switches.candidates("storage", eia_id, sector_abbr, is_ca)
        wrow = -1 if is_ca else self.wholesale.add(wholesale, float(price_mult))
        self.rows.append(dict(
            load_row=int(load_row), cf_row=int(cf_row), wholesale_row=wrow, tariff0=t0,
            sw_solar_off=so, sw_solar_cnt=sc, sw_storage_off=to, sw_storage_cnt=tc,
            scratch_slot=-1, flags=(1 if is_res else 0) | (2 if is_ca else 0),
            econ_life=int(econ_life), loan_term=int(loan_term), load_kwh=float(load_kwh),
            price_mult=float(price_mult), inflation=float(inflation), pv_deg=float(pv_deg),
            escalator=float(escalator), down_payment=float(down_payment), tax_rate=float(tax_rate),
            real_discount=float(real_discount), itc_frac=float(itc_frac), capex=float(capex),
            capex_combined=float(capex_combined), batt_capex_kwh=float(batt_capex_kwh),
            ccm=float(ccm), vor=float(vor)))
        return len(self.rows) - 1

    def columns(self) -> Dict[str, np.ndarray]:
        n = len(self.rows)
        cols = empty_columns(n)
        for i, r in enumerate(self.rows):
            for k, v in r.items():
                cols[k][i] = v
        assign_scratch(cols, self.tariffs.array(), self.switches.array())
        return cols


def assign_scratch(cols: Dict[str, np.ndarray], tariffs: np.ndarray, switches: np.ndarray) -> int:
    """Give an hourly scratch slot to every agent whose battery-case tariff can
    be net billing (mo 2), carry demand charges (both bill hourly imports) or
    bill its tiers in kWh/kW (month peaks): its initial tariff or any
    rate-switch candidate."""
    n = len(cols["load_kwh"])
    # net billing (metering options 2 and 3) bills hourly imports
    # kWh/kW tier units (codes 1, 3) need the battery case's month peaks: the plane too
    mo2 = ((tariffs["mo"] == 2) | (tariffs["mo"] == 3) | (tariffs["dc"] > 0) | (tariffs["unit"] == 1) |
           (tariffs["unit"] == 3)) if tariffs.size else np.zeros(0, bool)
    need = mo2[cols["tariff0"]] if n else np.zeros(0, bool)
    if switches.size:
        sw_mo2 = mo2[switches["tariff"]]
        csum = np.concatenate([[0], np.cumsum(sw_mo2.astype(np.int64))])
        for k in ("solar", "storage"):
            off = cols[f"sw_{k}_off"].astype(np.int64)
            cnt = cols[f"sw_{k}_cnt"].astype(np.int64)
            need |= (csum[off + cnt] - csum[off]) > 0
    slots = np.full(n, -1, dtype=np.int32)
    slots[need] = np.arange(int(need.sum()), dtype=np.int32)
    cols["scratch_slot"] = slots
    return int(need.sum())


def _factorize_rows(*cols):
    """(codes, first row of each distinct key) over the row tuples of `cols`,
    keys numbered in order of first appearance -- the order a row-by-row pass
    meets them; key equality is the dict's (identity, then ==).  None when a
    key is unhashable."""
    n = len(cols[0])
    if n == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    try:
        codes, uniq = pd.factorize(pd.Series(list(zip(*cols)), dtype=object), sort=False)
    except TypeError:
        return None
    codes = np.asarray(codes, np.int64)
    if (codes < 0).any():          # a NaN-like key pandas will not number: take the row path
        return None
    first = np.empty(len(uniq), np.int64)
    first[codes[::-1]] = np.arange(n - 1, -1, -1, dtype=np.int64)
    return codes, first


def _num(series) -> np.ndarray:
    """float(x) per cell, NaN where that raises (financial_functions._finite_float)."""
    out = pd.to_numeric(series, errors="coerce")
    return np.asarray(out, dtype=np.float64)


def columnize_frame(df, src, rate_switch_table=None, skip_demand_charges=None) -> "PopulationBuilder":
    """Vectorised PopulationBuilder over an agent DataFrame in the reference's
    schema (the columns calc_system_size_and_performance reads, ff:330-421):
    numeric columns converted whole, profile keys / tariffs / rate-switch
    candidates / wholesale series resolved once per distinct object (tariff
    dicts and wholesale arrays that rows share, as pandas merges leave them,
    are compiled / validated / hashed once).  Produces exactly the columns and
    tables add() row by row would (tests/test_boundary.py)."""
    b = PopulationBuilder(rate_switch_table, skip_demand_charges)
    n = len(df)
    cols = empty_columns(n)
    sector = df["sector_abbr"].tolist()
    state = df["state_abbr"].tolist() if "state_abbr" in df else [""] * n
    st_s = pd.Series(state, dtype=object)
    is_ca = (st_s.where(st_s.notna(), "").astype(str).str.upper() == "CA").to_numpy(bool) if n else np.zeros(0, bool)
    is_res = (pd.Series(sector, dtype=object) == "res").to_numpy(bool) if n else np.zeros(0, bool)
    # profile rows: one lookup per distinct key (the store is append-only, so
    # the key -> row maps are kept on it across calls)
    bldg, gid = df["bldg_id"].tolist(), df["solar_re_9809_gid"].tolist()
    tilt, az = df["tilt"].tolist(), df["azimuth"].tolist()
    lk = src.__dict__.setdefault("_columnar_load_rows", {})
    sk = src.__dict__.setdefault("_columnar_solar_rows", {})

    def rows_of(keys, cache, lookup):
        f = _factorize_rows(*keys)
        if f is None:
            out = np.empty(n, np.int64)
            for i, k in enumerate(zip(*keys)):
                r = cache.get(k)
                out[i] = r if r is not None else cache.setdefault(k, lookup(*k))
            return out
        codes, first = f
        rows = np.empty(first.size, np.int64)
        for j, i in enumerate(first.tolist()):
            k = tuple(c[i] for c in keys)
            r = cache.get(k)
            rows[j] = r if r is not None else cache.setdefault(k, lookup(*k))
        return rows[codes]
    cols["load_row"] = rows_of((bldg, sector, state), lk, lambda b_, s_, t_: src.load_row(
        {"bldg_id": b_, "sector_abbr": s_, "state_abbr": t_})).astype(cols["load_row"].dtype)
    cols["cf_row"] = rows_of((gid, tilt, az), sk, lambda g_, t_, a_: src.solar_row(
        {"solar_re_9809_gid": g_, "tilt": t_, "azimuth": a_})).astype(cols["cf_row"].dtype)
    # tariffs: content key once per distinct dict / string object
    from .tariff import tariff_key
    tdict = df["tariff_dict"].tolist()
    tkey: Dict[int, str] = {}
    eia = df["eia_id"].tolist()
    mult = _num(df["elec_price_multiplier"])
    whl = df["wholesale_prices"].tolist() if "wholesale_prices" in df else [None] * n
    W = b.wholesale
    # one resolution per distinct (tariff object, CA?, eia_id, sector): rows
    # repeat these combinations (pandas merges share the objects), and
    # resolving a combination at its first row keeps the tariff and switch
    # tables in the row-by-row order of first use
    ca_l = is_ca.tolist()

    def resolve(i):
        raw, ca, e = tdict[i], ca_l[i], eia[i]
        key = tkey.get(id(raw))
        if key is None:
            key = tkey[id(raw)] = tariff_key(raw)
        t0 = b.tariffs.add(raw, ca, key=key)
        so, sc = b.switches.candidates("solar", e, sector[i], ca)
        to, tc = b.switches.candidates("storage", e, sector[i], ca)
        return (t0, so, sc, to, tc)
    f = _factorize_rows([id(x) for x in tdict], ca_l, eia, sector)
    if f is not None:        # distinct combinations in first-use order, then mapped back
        codes, first = f
        res = np.array([resolve(i) for i in first.tolist()], np.int64).reshape(-1, 5)[codes]
    else:                    # an unhashable eia_id: the row-by-row memo
        memo: Dict[Tuple, Tuple[int, int, int, int, int]] = {}
        out: List[Tuple[int, int, int, int, int]] = []
        for i in range(n):
            try:
                ck = (id(tdict[i]), ca_l[i], eia[i], sector[i])
                hit = memo.get(ck)
            except TypeError:          # unhashable eia_id: resolve the row on its own
                ck, hit = None, None
            if hit is None:
                hit = resolve(i)
                if ck is not None:
                    memo[ck] = hit
            out.append(hit)
        res = np.array(out, np.int64).reshape(n, 5)
    cols["tariff0"] = res[:, 0].astype(cols["tariff0"].dtype)
    cols["sw_solar_off"] = res[:, 1].astype(cols["sw_solar_off"].dtype)
    cols["sw_solar_cnt"] = res[:, 2].astype(cols["sw_solar_cnt"].dtype)
    cols["sw_storage_off"] = res[:, 3].astype(cols["sw_storage_off"].dtype)
    cols["sw_storage_cnt"] = res[:, 4].astype(cols["sw_storage_cnt"].dtype)
    # wholesale rows do not interleave with the tables above: resolved whole
    cols["wholesale_row"] = W.add_frame(whl, mult, is_ca).astype(cols["wholesale_row"].dtype)
    cols["flags"] = (is_res.astype(np.uint8) | (is_ca.astype(np.uint8) << 1)).astype(np.uint8)
    cols["econ_life"] = df["economic_lifetime_yrs"].astype(np.int64).to_numpy().astype(np.int32)
    cols["loan_term"] = df["loan_term_yrs"].astype(np.int64).to_numpy().astype(np.int32)
    for name, ref in (("load_kwh", "load_kwh_per_customer_in_bin"), ("inflation", "inflation_rate"),
                      ("pv_deg", "pv_degradation_factor"), ("escalator", "elec_price_escalator"),
                      ("down_payment", "down_payment_fraction"), ("tax_rate", "tax_rate"),
                      ("real_discount", "real_discount_rate"), ("itc_frac", "itc_fraction_of_capex"),
                      ("capex", "system_capex_per_kw"), ("capex_combined", "system_capex_per_kw_combined"),
                      ("batt_capex_kwh", "batt_capex_per_kwh_combined"), ("ccm", "cap_cost_multiplier"),
                      ("vor", "value_of_resiliency_usd")):
        cols[name] = _num(df[ref])
    cols["price_mult"] = mult
    cols["scratch_slot"] = np.full(n, -1, np.int32)
    assign_scratch(cols, b.tariffs.array(), b.switches.array())
    b.frame_columns = cols
    return b
