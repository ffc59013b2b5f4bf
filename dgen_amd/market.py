"""Per-year agent attributes and first-year market seeding on the device
(SURVEY 8(f)-3 and the seeding half of 8(f)-1).

The reference rebuilds the agent frame's economic columns every model year
with a chain of pandas left merges (``agent_mutation/elec.py`` ``apply_*``,
called at ``dgen_model.py:252-292``) and seeds the first year's market from
observed state capacities (``elec.estimate_initial_market_shares``,
``elec.py:701-765``, called at ``dgen_model.py:390-393``).  Here:

* :class:`YearTables` compiles, once per model year and on the host, each
  lookup table to a dense array indexed by a per-agent key code that is built
  once per run.  Every per-row value is produced by the reference's own
  expression on its own table (the escalator CAGR of ``elec.py:64-73``
  included, positional final-year alignment and all), so the device's work is
  a pure gather and the result is bit-exact to the merges.
* ``dgen_year_inputs`` (``k_year_inputs``) gathers those rows into the
  resident SoA columns ``dgen_size_agents`` reads, plus the loop's customers
  and load in bin (``apply_load_growth``'s products are the only arithmetic).
* ``dgen_initial_market_shares`` (``k_initial_shares``) runs pandas'
  Kahan-compensated group sum per (state, sector, tech) group in frame order
  and each agent's portion of its state's starting capacities.

A key with more than one matching row would make the reference's merge
duplicate agents; it is refused here (``ValueError``).  A key with no row is
NaN (reals) / -1 (ints), as a left merge leaves it.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd

from . import _lib

YS_COLS = ["system_capex_per_kw", "system_capex_per_kw_combined", "batt_capex_per_kwh_combined",
           "pv_degradation_factor", "itc_fraction_of_capex", "economic_lifetime_yrs", "loan_term_yrs",
           "down_payment_fraction", "real_discount_rate", "tax_rate"]          # DGEN_YS_* order
YC_COLS = ["load_multiplier", "elec_price_multiplier", "elec_price_escalator"]  # DGEN_YC_* order
FIN_COLS = ["economic_lifetime_yrs", "loan_term_yrs", "down_payment_fraction", "real_discount_rate",
            "tax_rate"]

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64


class YearKeys(ctypes.Structure):
    _fields_ = [("k_sector", _vp), ("k_sector_county", _vp), ("k_state_sector", _vp), ("k_county", _vp),
                ("is_res", _vp), ("load_kwh_initial", _vp), ("customers_initial", _vp),
                ("load_in_bin_initial", _vp)]


class YearTablesC(ctypes.Structure):
    _fields_ = [("by_sector", _vp), ("by_sector_county", _vp), ("by_state_sector", _vp),
                ("wholesale_row", _vp), ("n_sector", _i64), ("n_sector_county", _i64),
                ("n_state_sector", _i64), ("n_county", _i64), ("inflation_rate", ctypes.c_double)]


YEAR_OUT_F64 = ["load_kwh", "price_mult", "escalator", "inflation", "pv_deg", "capex", "capex_combined",
                "batt_capex_kwh", "itc_frac", "down_payment", "real_discount", "tax_rate", "vor"]
YEAR_OUT_I32 = ["econ_life", "loan_term", "wholesale_row"]
YEAR_OUT_LOOP = ["customers_in_bin", "load_kwh_in_bin"]


class YearOut(ctypes.Structure):
    _fields_ = [(k, _vp) for k in YEAR_OUT_F64 + YEAR_OUT_I32 + YEAR_OUT_LOOP]


INIT_OUT = ["adopters_cum_last_year", "system_kw_cum_last_year", "batt_kw_cum_last_year",
            "batt_kwh_cum_last_year", "market_share_last_year", "market_value_last_year",
            "initial_number_of_adopters", "initial_pv_kw", "initial_batt_kw", "initial_batt_kwh",
            "initial_market_share", "initial_market_value"]


class InitIn(ctypes.Structure):
    _fields_ = [("developable_agent_weight", _vp), ("system_capex_per_kw", _vp)]


class InitOut(ctypes.Structure):
    _fields_ = [(k, _vp) for k in INIT_OUT] + [("developable_customers_in_state", _vp), ("agent_count", _vp)]


CAP_COLS = ["system_mw", "batt_mw", "batt_mwh", "pv_systems_count", "batt_systems_count"]


def _bind(L):
    L.dgen_year_inputs.restype = ctypes.c_int32
    L.dgen_year_inputs.argtypes = [_vp, ctypes.POINTER(YearKeys), ctypes.POINTER(YearTablesC),
                                   ctypes.POINTER(YearOut), _i64, _vp]
    L.dgen_initial_market_shares.restype = ctypes.c_int32
    L.dgen_initial_market_shares.argtypes = [_vp, ctypes.POINTER(InitIn), ctypes.POINTER(InitOut), _vp, _vp,
                                             _vp, _i64, _vp]
    return L


def _codes(keys: Sequence[Tuple]) -> Tuple[np.ndarray, List[Tuple]]:
    """Dense codes of the distinct keys (first-appearance order)."""
    uniq: Dict[Tuple, int] = {}
    code = np.empty(len(keys), np.int32)
    for i, k in enumerate(keys):
        code[i] = uniq.setdefault(k, len(uniq))
    return code, list(uniq.keys())


def _index_unique(df: pd.DataFrame, on: List[str], what: str) -> Dict[Tuple, int]:
    """Row position of every key of `df` on columns `on`; a repeated key is
    refused (the reference's merge would duplicate the agents matching it)."""
    idx: Dict[Tuple, int] = {}
    for pos, key in enumerate(zip(*[df[c].tolist() for c in on])):
        if key in idx:
            raise ValueError(f"{what}: key {dict(zip(on, key))} appears more than once; the reference's "
                             f"left merge would duplicate the agents that match it")
        idx[key] = pos
    return idx


def _lookup(df: pd.DataFrame, on: List[str], keys: Sequence[Tuple], cols: List[str], what: str) -> np.ndarray:
    """[len(keys), len(cols)] float64: the matching row's values, NaN on a miss."""
    idx = _index_unique(df, on, what)
    out = np.full((len(keys), len(cols)), np.nan)
    vals = [df[c].to_numpy(dtype=np.float64) for c in cols]
    for r, k in enumerate(keys):
        p = idx.get(k)
        if p is not None:
            for j, v in enumerate(vals):
                out[r, j] = v[p]
    return out


def elec_price_rows(traj: pd.DataFrame, year: int) -> Tuple[pd.DataFrame, pd.DataFrame]:
    """The two frames apply_elec_price_multiplier_and_escalator merges
    (elec.py:56-78), by the reference's own operations: this year's
    multipliers, and the escalator = clip((final / year_cap multiplier) **
    (1 / (final_year - year_cap)) - 1, -0.01, 0.01) with year_cap = min(year,
    2040) and the final year's values aligned by POSITION (reset_index)."""
    mult = traj[traj["year"] == year].reset_index(drop=True)
    year_cap = min(year, 2040)
    esc = traj[traj["year"] == year_cap].reset_index(drop=True)
    final_year = np.max(traj["year"])
    final = traj[traj["year"] == final_year].reset_index(drop=True)
    esc["final_year_values"] = final["elec_price_multiplier"].reset_index(drop=True)
    esc["elec_price_escalator"] = (esc["final_year_values"] / esc["elec_price_multiplier"]) ** (
        1.0 / (final_year - year_cap)) - 1.0
    esc["elec_price_escalator"] = np.clip(esc["elec_price_escalator"], -.01, .01)
    return mult, esc


class YearTables:
    """Per-run key codes + per-year dense tables (host), see the module doc.

    frame: the agents' static attributes (state_abbr, sector_abbr, county_id,
    and 'tech', default 'solar'), in device or caller order -- whatever order
    the key arrays are uploaded in.  tables: the reference's input frames by
    role: load_growth (year, sector_abbr, county_id, load_multiplier),
    elec_price (year, sector_abbr, county_id, elec_price_multiplier),
    pv_tech (year, sector_abbr, pv_degradation_factor), pv_price (year,
    sector_abbr, system_capex_per_kw), pv_plus_batt_price (year, sector_abbr,
    system_capex_per_kw, batt_capex_per_kwh), vor (state_abbr, sector_abbr,
    value_of_resiliency_usd), financing (year, sector_abbr, FIN_COLS), itc
    (year, tech, sector_abbr, itc_fraction_of_capex), and optionally
    wholesale_row: {(county_id, year): row of the engine's wholesale table}.
    """

    def __init__(self, frame: pd.DataFrame, tables: Dict[str, object], inflation_rate: float):
        self.t = tables
        self.inflation_rate = float(inflation_rate)
        st = frame["state_abbr"].tolist()
        sec = frame["sector_abbr"].tolist()
        cty = [int(c) for c in frame["county_id"].tolist()]
        self.tech = frame["tech"].tolist() if "tech" in frame else ["solar"] * len(sec)
        self.k_sector, self.sectors = _codes([(s, t) for s, t in zip(sec, self.tech)])
        self.k_sector_county, self.sector_counties = _codes(list(zip(sec, cty)))
        self.k_state_sector, self.state_sectors = _codes(list(zip(st, sec)))
        self.k_county, self.counties = _codes([(c,) for c in cty])
        self.is_res = np.array([s == "res" for s in sec], np.uint8)

    def compile(self, year: int) -> Dict[str, np.ndarray]:
        # each table restricted to the year first (its keys carry the year);
        # the elec price frames keep every year for the CAGR
        t = {k: (v[v["year"] == year] if isinstance(v, pd.DataFrame) and "year" in v and k != "elec_price"
                 else v) for k, v in self.t.items()}
        sk = [(year, s) for s, _ in self.sectors]
        by_sector = np.concatenate([
            _lookup(t["pv_price"], ["year", "sector_abbr"], sk, ["system_capex_per_kw"], "pv prices"),
            _lookup(t["pv_plus_batt_price"], ["year", "sector_abbr"], sk,
                    ["system_capex_per_kw", "batt_capex_per_kwh"], "pv+battery prices"),
            _lookup(t["pv_tech"], ["year", "sector_abbr"], sk, ["pv_degradation_factor"], "pv tech"),
            _lookup(t["itc"], ["year", "tech", "sector_abbr"], [(year, tc, s) for s, tc in self.sectors],
                    ["itc_fraction_of_capex"], "itc options"),
            _lookup(t["financing"], ["year", "sector_abbr"], sk, FIN_COLS, "financing terms"),
        ], axis=1)
        sck = [(year, s, c) for s, c in self.sector_counties]
        lg = _lookup(t["load_growth"], ["year", "sector_abbr", "county_id"], sck, ["load_multiplier"],
                     "load growth")
        mult, esc = elec_price_rows(t["elec_price"], year)
        pm = _lookup(mult, ["sector_abbr", "county_id"], self.sector_counties, ["elec_price_multiplier"],
                     "elec price multipliers")
        pe = _lookup(esc, ["sector_abbr", "county_id"], self.sector_counties, ["elec_price_escalator"],
                     "elec price escalators")
        by_sc = np.concatenate([lg, pm, pe], axis=1)
        vor = _lookup(t["vor"], ["state_abbr", "sector_abbr"], self.state_sectors,
                      ["value_of_resiliency_usd"], "value of resiliency")[:, 0]
        wr = None
        wmap = t.get("wholesale_row")
        if wmap is not None:
            wr = np.array([int(wmap.get((c, year), -1)) for (c,) in self.counties], np.int32)
        return {"by_sector": np.ascontiguousarray(by_sector), "by_sector_county": np.ascontiguousarray(by_sc),
                "by_state_sector": np.ascontiguousarray(vor), "wholesale_row": wr}

    def gather_host(self, year: int, load_kwh0, customers0, load_in_bin0) -> Dict[str, np.ndarray]:
        """The device gather restated on the host (tests): same rows, same
        products as k_year_inputs."""
        c = self.compile(year)
        S, C = c["by_sector"][self.k_sector], c["by_sector_county"][self.k_sector_county]
        mult = C[:, 0]
        res = self.is_res.astype(bool)
        toint = lambda v: np.where(np.isnan(v), -1, np.nan_to_num(v)).astype(np.int32)
        out = {"load_kwh": np.where(res, load_kwh0 * mult, load_kwh0),
               "customers_in_bin": np.where(res, customers0, customers0 * mult),
               "load_kwh_in_bin": load_in_bin0 * mult, "price_mult": C[:, 1], "escalator": C[:, 2],
               "inflation": np.full(len(mult), self.inflation_rate), "capex": S[:, 0], "capex_combined": S[:, 1],
               "batt_capex_kwh": S[:, 2], "pv_deg": S[:, 3], "itc_frac": S[:, 4], "econ_life": toint(S[:, 5]),
               "loan_term": toint(S[:, 6]), "down_payment": S[:, 7], "real_discount": S[:, 8],
               "tax_rate": S[:, 9], "vor": c["by_state_sector"][self.k_state_sector]}
        if c["wholesale_row"] is not None:
            out["wholesale_row"] = c["wholesale_row"][self.k_county]
        return out


def financing_max_years(by_sector: np.ndarray, k_sector, year: int) -> int:
    """Largest economic lifetime the agents (sector keys `k_sector`) gather
    from a compiled year's by_sector table; the lifetimes and loan terms they
    use must lie in [1, MAXY] (a merge miss is NaN and is rejected, as the
    upload-time checks would reject it)."""
    used = np.unique(np.asarray(k_sector, np.int64))
    if used.size == 0:
        return 0
    terms = np.asarray(by_sector)[used][:, [5, 6]]
    if not np.all(np.isfinite(terms)) or terms.min() < 1 or terms.max() > _lib.MAXY:
        raise ValueError(f"financing terms for {year}: economic lifetime / loan term outside "
                         f"[1, {_lib.MAXY}] or missing (merge miss)")
    return int(terms[:, 0].max())


class YearInputs:
    """Device side of YearTables: key codes and initial columns resident on the
    GPU, per-year tables uploaded (cached) and gathered by dgen_year_inputs."""

    def __init__(self, engine, tables: YearTables, load_kwh0, customers0, load_in_bin0):
        import torch
        self.eng, self.yt = engine, tables
        self.L = _bind(engine.lib)
        dev = engine.dev
        i32 = lambda a: torch.as_tensor(np.asarray(a, np.int32), device=dev)
        f64 = lambda a: torch.as_tensor(np.asarray(a, np.float64), device=dev)
        self._keep = {"k_sector": i32(tables.k_sector), "k_sector_county": i32(tables.k_sector_county),
                      "k_state_sector": i32(tables.k_state_sector), "k_county": i32(tables.k_county),
                      "is_res": torch.as_tensor(tables.is_res, device=dev), "load_kwh_initial": f64(load_kwh0),
                      "customers_initial": f64(customers0), "load_in_bin_initial": f64(load_in_bin0)}
        self.keys = YearKeys(**{k: v.data_ptr() for k, v in self._keep.items()})
        self._years: Dict[int, Tuple[YearTablesC, Dict]] = {}

    def _tables(self, year: int):
        import torch
        hit = self._years.get(year)
        if hit is None:
            c = self.yt.compile(year)
            dev = self.eng.dev
            keep = {k: torch.as_tensor(v, device=dev) for k, v in c.items() if v is not None}
            tc = YearTablesC(by_sector=keep["by_sector"].data_ptr(),
                             by_sector_county=keep["by_sector_county"].data_ptr(),
                             by_state_sector=keep["by_state_sector"].data_ptr(),
                             wholesale_row=keep["wholesale_row"].data_ptr() if "wholesale_row" in keep else None,
                             n_sector=len(self.yt.sectors), n_sector_county=len(self.yt.sector_counties),
                             n_state_sector=len(self.yt.state_sectors),
                             n_county=len(self.yt.counties) if "wholesale_row" in keep else 0,
                             inflation_rate=self.yt.inflation_rate)
            # the financing lifetimes this shard's agents gather: the sizing
            # kernels pick their lanes-per-agent form from the batch maximum,
            # so it is refreshed every year (a merge miss is NaN -> rejected)
            max_years = financing_max_years(c["by_sector"], self.yt.k_sector, year)
            hit = self._years[year] = (tc, keep, max_years)
        return hit[0]

    def max_years(self, year: int) -> int:
        """Largest economic lifetime any agent of the shard gathers in `year`."""
        self._tables(year)
        return self._years[year][2]

    def apply(self, year: int, cols: Dict[str, object], loop: Dict[str, object]):
        """Write year `year`'s attributes into the device agent columns `cols`
        (the AgentBatch.cols names) and the loop columns `loop`
        (customers_in_bin, load_kwh_in_bin), stream-ordered."""
        tc = self._tables(year)
        ptr = {k: cols[k].data_ptr() for k in YEAR_OUT_F64 + ["econ_life", "loan_term"]}
        ptr["wholesale_row"] = cols["wholesale_row"].data_ptr() if tc.wholesale_row else None
        ptr.update({k: loop[k].data_ptr() for k in YEAR_OUT_LOOP})
        out = YearOut(**ptr)
        n = len(self.yt.k_sector)
        _lib.check(self.L.dgen_year_inputs(self.eng.ctx, ctypes.byref(self.keys), ctypes.byref(tc),
                                           ctypes.byref(out), n, self.eng.stream_handle()), "dgen_year_inputs")


def initial_market_shares(engine, state, sector, tech, developable_agent_weight, system_capex_per_kw,
                          caps: pd.DataFrame, dev_index: Optional[np.ndarray] = None):
    """estimate_initial_market_shares (elec.py:701-765) on device.  state /
    sector / tech: host sequences in frame order (the order pandas' group sums
    visit rows); the two value columns are device float64 tensors, row
    dev_index[i] holding frame row i (default: the same order); outputs are in
    the value columns' order.  caps: the state starting
    capacities frame (state_abbr, sector_abbr, CAP_COLS).  Returns a dict of
    device tensors (INIT_OUT + per-group developable_customers_in_state and
    agent_count, groups in first-appearance order)."""
    import torch
    from .dist import group_order
    L = _bind(engine.lib)
    n = len(state)
    keys = list(zip(state, sector, tech))
    perm, seg_off, uniq = group_order(keys)
    capk = [(s, c) for s, c, _ in uniq]
    cap = _lookup(caps, ["state_abbr", "sector_abbr"], capk, CAP_COLS, "state starting capacities")
    dev = engine.dev
    rows = perm.astype(np.int64) if dev_index is None else np.asarray(dev_index, np.int64)[perm]
    keep = {"idx": torch.as_tensor(rows, device=dev),
            "seg": torch.as_tensor(seg_off, device=dev),
            "caps": torch.as_tensor(np.ascontiguousarray(cap), device=dev)}
    out = {k: torch.empty(n, dtype=torch.float64, device=dev) for k in INIT_OUT}
    out["developable_customers_in_state"] = torch.empty(len(uniq), dtype=torch.float64, device=dev)
    out["agent_count"] = torch.empty(len(uniq), dtype=torch.int64, device=dev)
    w = developable_agent_weight.contiguous()
    cx = system_capex_per_kw.contiguous()
    ci = InitIn(developable_agent_weight=w.data_ptr(), system_capex_per_kw=cx.data_ptr())
    co = InitOut(**{k: v.data_ptr() for k, v in out.items()})
    _lib.check(L.dgen_initial_market_shares(engine.ctx, ctypes.byref(ci), ctypes.byref(co),
                                            keep["idx"].data_ptr(), keep["seg"].data_ptr(),
                                            keep["caps"].data_ptr(), len(uniq), engine.stream_handle()),
               "dgen_initial_market_shares")
    torch.cuda.current_stream(dev).synchronize()
    out["groups"] = uniq
    return out
