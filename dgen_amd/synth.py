"""Synthetic agent populations: the reference's DB and agent
files are remote downloads, so every benchmark / scale test runs on
populations generated here with numpy PCG64, seed = 20260000 + config number.

Profiles: diurnal x seasonal x lognormal load shapes normalised to 1 (float32),
solar cf x 1e6 (int32, 1100-1900 kWh/kW-yr, zero at night), per-county 8760
wholesale $/kWh.  Scalars: the 2026 rows of the reference's input CSVs
(financing_atb_FY23.csv:14, pv_price_atb23_mid.csv:14,
pv_plus_batt_prices_FY23_mid.csv:14, pv_tech_performance_defaultFY19.csv:14).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import pandas as pd

from . import _lib
from .columnar import assign_scratch, empty_columns
from .engine import SWITCH_DTYPE
from .tariff import TariffTable

NH = _lib.NH

CONFIGS = {
    # name: (config number, sector mix, tariff metering, description)
    "de_res": (1, "res", "nem", "DE-like residential PV-only stand-in (50k)"),
    "ca_res_storage": (2, "res", "ca", "CA-like residential PV+storage stand-in (200k)"),
    "res_1m_nem_tou": (3, "res", "nem", "synthetic 1M residential, NEM TOU tariffs"),
    "com_8m": (4, "com", "nem", "synthetic commercial with battery"),
    # C4 extension mode: the reference keeps demand charges off (ff:35); here
    # they are compiled and billed (parity unpinned)
    "com_dc_batt": (4, "com", "nem_dc", "synthetic commercial, demand charges billed, with battery"),
    "national_mixed": (5, "mixed", "mixed", "national mixed population"),
    # parity case (not a bench line): tariffs spread over SAM's metering
    # options 0-4 (the reference passes ur_metering_option through, ff:586)
    "metering_mix": (6, "mixed", "all", "mixed population, metering options 0-4"),
    # parity case: commercial tariffs whose tiers are in kWh/kW (unit 1) or
    # kWh/kW daily (unit 3) on 60 %, caps scaled by the month's peak import
    "com_kwkw": (7, "com", "kwkw", "commercial, kWh/kW tier units"),
}


@dataclass
class Population:
    shapes: np.ndarray           # float32 [R, 8760]
    cfs: np.ndarray              # int32 [C, 8760]
    wholesale: Optional[np.ndarray]  # float64 [W, 8760]
    tariffs: np.ndarray          # TARIFF_DTYPE
    switches: np.ndarray         # SWITCH_DTYPE
    cols: Dict[str, np.ndarray]  # agent SoA columns
    n_scratch: int
    config: str
    state_ix: Optional[np.ndarray] = None   # int16 index into STATES per agent
    demand: Optional[np.ndarray] = None     # DEMAND_DTYPE (demand-charge configs)
    county_ix: Optional[np.ndarray] = None  # int32 county per agent (wholesale row of non-CA agents)

    @property
    def skip_demand_charges(self) -> int:
        """EngineConfig.skip_demand_charges the population is meant for."""
        return 0 if self.demand is not None and self.demand.size else 1


def load_shapes(rng, n_rows: int, commercial: bool) -> np.ndarray:
    hod = np.arange(NH) % 24
    doy = np.arange(NH) // 24
    dow = doy % 7
    out = np.empty((n_rows, NH), dtype=np.float32)
    step = 256
    for s in range(0, n_rows, step):
        k = min(step, n_rows - s)
        ph = rng.uniform(-2.0, 2.0, (k, 1))
        amp = rng.uniform(0.3, 0.9, (k, 1))
        sea = rng.uniform(0.1, 0.5, (k, 1))
        if commercial:
            occ = ((hod >= 7) & (hod <= 19) & (dow < 5)).astype(float)
            diurnal = 0.45 + amp * occ + 0.05 * np.sin((hod - 12 - ph) / 24 * 2 * np.pi)
        else:
            diurnal = (1.0 + amp * np.sin((hod - 7 - ph) / 24 * 2 * np.pi) ** 2
                       + 0.4 * amp * ((hod >= 17) & (hod <= 21)))
        seasonal = 1.0 + sea * np.cos((doy - 200 + 20 * ph) / 365 * 2 * np.pi)
        noise = rng.lognormal(0.0, 0.25, (k, NH))
        x = diurnal * seasonal * noise
        out[s:s + k] = (x / x.sum(axis=1, keepdims=True)).astype(np.float32)
    return out


def solar_cfs(rng, n_rows: int) -> np.ndarray:
    hod = np.arange(NH) % 24
    doy = np.arange(NH) // 24
    out = np.empty((n_rows, NH), dtype=np.int32)
    step = 256
    for s in range(0, n_rows, step):
        k = min(step, n_rows - s)
        lat = rng.uniform(-0.8, 0.8, (k, 1))
        daylen = 12.0 + 3.0 * np.cos((doy - 172) / 365 * 2 * np.pi) * (1 + 0.3 * lat)
        rise = 12.0 - daylen / 2
        t = (hod + 0.5 - rise) / daylen
        sun = np.clip(np.sin(np.pi * t), 0.0, None) * ((t > 0) & (t < 1))
        cloud = np.clip(rng.normal(0.85, 0.22, (k, NH)), 0.05, 1.0)
        cf = sun * cloud
        target = rng.uniform(1100.0, 1900.0, (k, 1))
        cf = cf * (target / cf.sum(axis=1, keepdims=True))
        out[s:s + k] = np.round(np.clip(cf, 0.0, 1.0) * 1e6).astype(np.int32)
    return out


def wholesale_rows(rng, n_rows: int) -> np.ndarray:
    hod = np.arange(NH) % 24
    doy = np.arange(NH) // 24
    base = rng.uniform(0.02, 0.08, (n_rows, 1))
    w = base * (1.0 + 0.35 * np.sin((hod - 14) / 24 * 2 * np.pi)[None, :]
                + 0.15 * np.cos((doy - 200) / 365 * 2 * np.pi)[None, :])
    w += rng.normal(0.0, 0.003, (n_rows, NH))
    return np.clip(w, 0.005, None)


def random_tariffs(rng, n: int, metering: str):
    """256-ish synthetic URDB-style tariffs: P 1..4, T 1..3 (mostly BIG caps),
    prices U[0.06, 0.40] $/kWh, fixed U[0, 25] $/month; legacy e_* and ur_*
    forms mixed.  metering: 'nem' -> mo 0; 'nb' -> mo 2; 'mixed' -> 20 % mo 2;
    'all' -> uniform over options 0-4."""
    out = []
    for k in range(n):
        P = int(rng.integers(1, 5))
        T = int(rng.integers(1, 4))
        prices = np.sort(np.round(rng.uniform(0.06, 0.40, (T, P)), 5), axis=0)
        fixed = float(np.round(rng.uniform(0.0, 25.0), 2))
        on0 = int(rng.integers(12, 18))
        wk = np.zeros((12, 24), dtype=int)
        for p in range(1, P):
            wk[:, (on0 + 2 * p) % 24:(on0 + 2 * p + 3) % 24 or 24] = p
        we = np.zeros((12, 24), dtype=int)
        if metering == "all":
            mo = int(rng.integers(0, 5))
        else:
            mo = 0 if metering in ("nem", "nem_dc") else (2 if metering == "nb" else int(rng.random() < 0.2) * 2)
        unit = 0
        if metering == "kwkw":
            unit = int(rng.choice([1, 3, 0], p=[0.35, 0.25, 0.40]))
            if unit and T == 1:
                T = 2
                prices = np.sort(np.round(rng.uniform(0.06, 0.40, (T, P)), 5), axis=0)
        lv = None
        if T > 1:
            if unit == 1:        # kWh per kW of the month's peak
                lv = np.sort(rng.choice([120.0, 200.0, 300.0, 450.0], size=(T, P)), axis=0)
            elif unit == 3:      # kWh per kW per day
                lv = np.sort(rng.choice([4.0, 7.0, 10.0, 15.0], size=(T, P)), axis=0)
            else:
                lv = np.sort(rng.choice([250.0, 400.0, 600.0, 900.0], size=(T, P)), axis=0)
            lv[-1, :] = 1e38
        if k % 2 == 0:
            d = {"e_prices": prices.tolist(), "e_wkday_12by24": wk.tolist(),
                 "e_wkend_12by24": we.tolist(), "fixed_charge": fixed, "ur_metering_option": mo}
            if lv is not None:
                d["e_levels"] = lv.tolist()
            if unit:
                d["energy_rate_unit"] = {1: "kWh/kW", 3: "kWh/kW daily"}[unit]
        else:
            rows = [[p + 1, t + 1, 1e38 if lv is None else float(lv[t, p]), unit, float(prices[t, p]), 0.0]
                    for p in range(P) for t in range(T)]
            d = {"ur_ec_tou_mat": rows, "ur_ec_sched_weekday": (wk + 1).tolist(),
                 "ur_ec_sched_weekend": (we + 1).tolist(), "ur_monthly_fixed_charge": fixed,
                 "ur_metering_option": mo}
        if metering == "nem_dc":
            # monthly flat demand charge (1-2 tiers, $/kW) on every tariff, a
            # 2-period TOU demand charge (afternoon peak) on half of them
            nt = int(rng.integers(1, 3))
            fp = np.round(rng.uniform(4.0, 16.0, nt), 2)
            caps = [float(rng.choice([50.0, 100.0, 250.0]))] if nt == 2 else []
            d["ur_dc_flat_mat"] = [[m, t + 1, (caps + [1e38])[t], float(fp[t])]
                                   for m in range(12) for t in range(nt)]
            if rng.random() < 0.5:
                on = int(rng.integers(11, 15))
                d["ur_dc_tou_mat"] = [[1, 1, 1e38, float(np.round(rng.uniform(0.0, 3.0), 2))],
                                      [2, 1, 1e38, float(np.round(rng.uniform(5.0, 18.0), 2))]]
                d["ur_dc_sched_weekday"] = [[2 if on <= h < on + 6 else 1 for h in range(24)]] * 12
                d["ur_dc_sched_weekend"] = [[1] * 24 for _ in range(12)]
        out.append(d)
    return out


STATES = ["AL", "AZ", "AR", "CA", "CO", "CT", "DE", "FL", "GA", "ID", "IL", "IN", "IA", "KS", "KY",
          "LA", "ME", "MD", "MA", "MI", "MN", "MS", "MO", "MT", "NE", "NV", "NH", "NJ", "NM", "NY",
          "NC", "ND", "OH", "OK", "OR", "PA", "RI", "SC", "SD", "TN", "TX", "UT", "VT", "VA", "WA",
          "WV", "WI", "WY", "DC", "AK", "HI"]


# Approximate households per state (millions, 2020 census order of magnitude),
# STATES order: the "census" state mix of a national population, so that state
# sizes are as uneven as the real ones (CA and TX together ~18 %, WY ~0.2 %).
STATE_HOUSEHOLDS_M = np.array([
    1.93, 2.74, 1.17, 13.30, 2.23, 1.40, 0.38, 8.23, 3.83, 0.66, 4.91, 2.62, 1.27, 1.13, 1.74,
    1.74, 0.57, 2.23, 2.62, 3.98, 2.21, 1.11, 2.43, 0.43, 0.77, 1.13, 0.53, 3.27, 0.80, 7.42,
    4.01, 0.32, 4.68, 1.49, 1.64, 5.11, 0.41, 1.96, 0.35, 2.63, 10.00, 1.03, 0.26, 3.15, 2.90,
    0.73, 2.37, 0.23, 0.29, 0.25, 0.46])


@dataclass
class PopTables:
    """The tables a population's agents index (profiles, wholesale rows,
    compiled tariffs, DG switch rows), shared by every agent drawn against them
    (national_tables / make_population(tables=...)): one national population
    generated state by state, each rank drawing only its own pieces."""
    config: str
    shapes: np.ndarray
    cfs: np.ndarray
    wholesale: np.ndarray
    tt: object                       # TariffTable
    base_idx: np.ndarray
    ca_idx: np.ndarray
    n_res_shapes: int
    n_com_shapes: int
    n_cf: int
    n_counties: int
    n_tariffs: int
    switches: Optional[np.ndarray] = None
    sw_first: Optional[np.ndarray] = None     # [n_util, is_res, is_ca] -> switch row (-1: none)


N_UTIL = 3000


def _switch_rows(rng, n_tariffs: int, base_idx, ca_idx):
    """10 % of (utility, sector) get one DG rate-switch row (solar)."""
    has_dg = rng.random((N_UTIL, 2)) < 0.10
    sw = []
    first = np.full((N_UTIL, 2, 2), -1, dtype=np.int64)   # [util, is_res, is_ca] -> switch index
    for u in range(N_UTIL):
        for r in range(2):
            if not has_dg[u, r]:
                continue
            lim = 10.0 if r == 1 else 200.0
            k = int(rng.integers(0, n_tariffs))
            otc = float(rng.uniform(0.0, 500.0))
            for c in range(2):
                rec = np.zeros((), dtype=SWITCH_DTYPE)
                rec["min_kw"], rec["max_kw"], rec["one_time_charge"] = 0.0, lim, otc
                rec["tariff"] = ca_idx[k] if c else base_idx[k]
                first[u, r, c] = len(sw)
                sw.append(rec)
    switches = np.stack(sw).astype(SWITCH_DTYPE) if sw else np.zeros(0, dtype=SWITCH_DTYPE)
    return switches, first


def _tables(rng, config: str, n_res_shapes: int, n_com_shapes: int, n_cf: int, n_counties: int,
            n_tariffs: int) -> PopTables:
    _, _, metering, _ = CONFIGS[config]
    res_shapes = load_shapes(rng, n_res_shapes, commercial=False)
    com_shapes = load_shapes(rng, n_com_shapes, commercial=True)
    shapes = np.concatenate([res_shapes, com_shapes])
    cfs = solar_cfs(rng, n_cf)
    wholesale = wholesale_rows(rng, n_counties)
    tt = TariffTable(skip_demand_charges=False if metering == "nem_dc" else None)
    raw = random_tariffs(rng, n_tariffs, "nem" if metering in ("nem", "ca") else metering)
    base_idx = np.array([tt.add(d, False) for d in raw], dtype=np.int32)
    ca_idx = np.array([tt.add(d, True) for d in raw], dtype=np.int32)
    return PopTables(config=config, shapes=shapes, cfs=cfs, wholesale=wholesale, tt=tt, base_idx=base_idx,
                     ca_idx=ca_idx, n_res_shapes=n_res_shapes, n_com_shapes=n_com_shapes, n_cf=n_cf,
                     n_counties=n_counties, n_tariffs=n_tariffs)


def national_tables(config: str = "national_mixed", seed: Optional[int] = None,
                    n_res_shapes: int = 4096, n_com_shapes: int = 2048, n_cf: int = 2048,
                    n_counties: int = 3100, n_tariffs: int = 256) -> PopTables:
    """The shared tables of a population generated piece by piece
    (make_population(..., tables=T, agent_seed=...)): profiles and tariffs
    from the config's stream, the DG switch rows from their own stream."""
    cnum = CONFIGS[config][0]
    s0 = 20260000 + cnum if seed is None else seed
    T = _tables(np.random.default_rng(s0), config, n_res_shapes, n_com_shapes, n_cf, n_counties, n_tariffs)
    T.switches, T.sw_first = _switch_rows(np.random.default_rng(s0 + 2), n_tariffs, T.base_idx, T.ca_idx)
    return T


def make_population(config: str, n_agents: int, seed: Optional[int] = None,
                    n_res_shapes: int = 4096, n_com_shapes: int = 2048, n_cf: int = 2048,
                    n_counties: int = 3100, n_tariffs: int = 256,
                    state_pool: Optional[np.ndarray] = None,
                    state_mix: str = "uniform", tables: Optional[PopTables] = None,
                    agent_seed: Optional[int] = None) -> Population:
    """Synthetic population of `config`.  `state_pool` (indices into
    STATES) restricts the agents' states, e.g. to the states one rank of the
    model-year loop owns (year_loop.rank_states); CA agents take the NEM3 path.
    state_mix (mixed configs): "uniform" (every state equally likely, the
    default stream) or "census" (states drawn in proportion to
    STATE_HOUSEHOLDS_M, renormalised over the pool).  tables (with
    agent_seed): draw the agents alone, from their own stream, against shared
    tables (national_tables; the table-size arguments are then ignored)."""
    if config not in CONFIGS:
        raise KeyError(f"unknown config {config!r}; one of {sorted(CONFIGS)}")
    cnum, sector, metering, _ = CONFIGS[config]
    if tables is None:
        rng = np.random.default_rng(20260000 + cnum if seed is None else seed)
        T = _tables(rng, config, n_res_shapes, n_com_shapes, n_cf, n_counties, n_tariffs)
    else:
        if agent_seed is None or tables.config != config:
            raise ValueError("shared tables need their own config and an agent_seed")
        T = tables
        rng = np.random.default_rng(agent_seed)
    n = int(n_agents)
    n_res_shapes, n_com_shapes, n_cf = T.n_res_shapes, T.n_com_shapes, T.n_cf
    n_counties, n_tariffs = T.n_counties, T.n_tariffs
    base_idx, ca_idx = T.base_idx, T.ca_idx

    if sector == "res":
        is_res = np.ones(n, dtype=bool)
    elif sector == "com":
        is_res = np.zeros(n, dtype=bool)
    else:
        is_res = rng.random(n) < 0.75
    if metering == "ca":
        is_ca = np.ones(n, dtype=bool)
    elif sector == "mixed" or metering == "mixed":
        pool = np.arange(len(STATES)) if state_pool is None else np.asarray(state_pool, np.int64)
        if len(pool) == 0:
            raise ValueError("empty state pool")
        if state_mix == "census":
            w = STATE_HOUSEHOLDS_M[pool]
            state_ix = pool[np.minimum(np.searchsorted(np.cumsum(w / w.sum()), rng.random(n), side="right"),
                                       len(pool) - 1)]
        elif state_mix == "uniform":
            state_ix = pool[rng.integers(0, len(pool), n)]
        else:
            raise ValueError(f"unknown state_mix {state_mix!r}")
        is_ca = state_ix == STATES.index("CA")
    else:
        is_ca = np.zeros(n, dtype=bool)

    cols = empty_columns(n)
    cols["load_row"] = np.where(is_res, rng.integers(0, n_res_shapes, n),
                                n_res_shapes + rng.integers(0, n_com_shapes, n)).astype(np.int32)
    cols["cf_row"] = rng.integers(0, n_cf, n).astype(np.int32)
    county = rng.integers(0, n_counties, n).astype(np.int32)
    cols["wholesale_row"] = np.where(is_ca, -1, county).astype(np.int32)
    tix = rng.integers(0, n_tariffs, n)
    cols["tariff0"] = np.where(is_ca, ca_idx[tix], base_idx[tix]).astype(np.int32)
    cols["flags"] = (is_res.astype(np.uint8) | (is_ca.astype(np.uint8) << 1)).astype(np.uint8)
    res_load = rng.lognormal(np.log(10000.0), 0.35, n)
    com_load = np.clip(rng.lognormal(np.log(150000.0), 1.2, n), 1e4, 5e7)
    cols["load_kwh"] = np.where(is_res, res_load, com_load)
    cols["price_mult"] = rng.uniform(0.9, 1.1, n)
    cols["econ_life"] = np.full(n, 25, dtype=np.int32)
    cols["loan_term"] = np.where(is_res, 20, 30).astype(np.int32)
    cols["inflation"] = np.full(n, 0.025)
    cols["pv_deg"] = np.full(n, 0.005)
    cols["escalator"] = rng.uniform(-0.01, 0.01, n)
    cols["down_payment"] = np.where(is_res, 0.3, 1.0)
    cols["tax_rate"] = np.full(n, 0.2574)
    cols["real_discount"] = np.where(is_res, 0.05, 0.0378)
    cols["itc_frac"] = np.full(n, 0.3)
    cols["capex"] = np.where(is_res, 4637.5, 1672.9)
    cols["capex_combined"] = np.where(is_res, 4500.0, 1600.0)
    cols["batt_capex_kwh"] = np.where(is_res, 431.0, 197.3)
    cols["ccm"] = rng.uniform(0.9, 1.2, n)
    cols["vor"] = np.where(rng.random(n) < 0.2, rng.uniform(0.0, 300.0, n), 0.0)

    util = rng.integers(0, N_UTIL, n)
    if T.switches is None:           # one stream: the switch rows follow the agents' draws
        switches, first = _switch_rows(rng, n_tariffs, base_idx, ca_idx)
    else:
        switches, first = T.switches, T.sw_first
    idx = first[util, is_res.astype(int), is_ca.astype(int)]
    cols["sw_solar_off"] = np.where(idx >= 0, idx, 0).astype(np.int32)
    cols["sw_solar_cnt"] = (idx >= 0).astype(np.int32)
    cols["sw_storage_off"] = np.zeros(n, dtype=np.int32)
    cols["sw_storage_cnt"] = np.zeros(n, dtype=np.int32)
    tt = T.tt
    tariffs = tt.array()
    n_scratch = assign_scratch(cols, tariffs, switches)
    if not (sector == "mixed" or metering == "mixed"):
        # states of the single-market configs from their own stream, so the
        # population above is unchanged: CA for the CA stand-in, else non-CA
        srng = np.random.default_rng((20260000 + cnum if seed is None else seed) + 1)
        pool = np.asarray([i for i in range(len(STATES)) if STATES[i] != "CA"]
                          if state_pool is None else state_pool, np.int64)
        if metering == "ca":
            pool = np.asarray([STATES.index("CA")])
        state_ix = pool[srng.integers(0, len(pool), n)]
    return Population(shapes=T.shapes, cfs=T.cfs, wholesale=T.wholesale, tariffs=tariffs,
                      switches=switches, cols=cols, n_scratch=n_scratch, config=config,
                      state_ix=state_ix.astype(np.int16),
                      demand=tt.demand_array() if metering == "nem_dc" else None,
                      county_ix=county)


def subset(pop: Population, idx) -> Population:
    """The agents `idx` of a population (same profile / tariff / switch
    tables), scratch slots re-assigned: e.g. one rank's states of a national
    population (year_loop.rank_states)."""
    idx = np.asarray(idx, np.int64)
    cols = {k: np.asarray(v)[idx].copy() for k, v in pop.cols.items()}
    n_scratch = assign_scratch(cols, pop.tariffs, pop.switches)
    pick = lambda a: None if a is None else np.asarray(a)[idx].copy()
    return Population(shapes=pop.shapes, cfs=pop.cfs, wholesale=pop.wholesale, tariffs=pop.tariffs,
                      switches=pop.switches, cols=cols, n_scratch=n_scratch, config=pop.config,
                      state_ix=pick(pop.state_ix), demand=pop.demand, county_ix=pick(pop.county_ix))


def reference_frame(n: int, seed: int = 20260811, n_load: int = 512, n_cf: int = 256, n_counties: int = 64,
                    n_tariffs: int = 64, n_util: int = 300):
    """An agent DataFrame in the reference's schema (the columns
    calc_system_size_and_performance reads, ff:330-421) with the objects a
    merged agent file carries: tariff dicts and per-county wholesale arrays
    shared by the rows that merged them, profile keys into a ProfileStore,
    and a rate_switch_table (elec.py:828-836 columns).  Returns (df, store,
    switch_table).  For the drop-in path's tests and bench_dropin.py."""
    from .profiles import ProfileStore
    rng = np.random.default_rng(seed)
    shapes = np.concatenate([load_shapes(rng, n_load // 2, False), load_shapes(rng, n_load - n_load // 2, True)])
    cfs = solar_cfs(rng, n_cf)
    whl = wholesale_rows(rng, n_counties)
    whl_obj = [whl[c] for c in range(n_counties)]          # one array object per county
    raws = random_tariffs(rng, n_tariffs, "mixed")
    is_res = rng.random(n) < 0.8
    st = np.array(STATES)[rng.integers(0, len(STATES), n)]
    store = ProfileStore()
    lrow = np.where(is_res, rng.integers(0, n_load // 2, n), n_load // 2 + rng.integers(0, n_load - n_load // 2, n))
    crow = rng.integers(0, n_cf, n)
    keys_l = {}
    bldg = np.empty(n, np.int64)
    for i in range(n):
        k = (int(lrow[i]) + 100000, "res" if is_res[i] else "com", str(st[i]))
        if k not in keys_l:
            keys_l[k] = store.add_load(k, shapes[lrow[i]])
        bldg[i] = k[0]
    for j in range(n_cf):
        store.add_solar((j + 7000, 25, 180), cfs[j])
    county = rng.integers(0, n_counties, n)
    eia = rng.integers(0, n_util, n)
    tix = rng.integers(0, n_tariffs, n)
    df = pd.DataFrame({
        "agent_id": np.arange(n) * 2 + 1, "sector_abbr": np.where(is_res, "res", "com"), "state_abbr": st,
        "bldg_id": bldg, "solar_re_9809_gid": crow + 7000, "tilt": 25, "azimuth": 180, "eia_id": eia,
        "tariff_id": tix + 1000, "tariff_dict": [raws[k] for k in tix], "county_id": county,
        "wholesale_prices": [whl_obj[c] for c in county],
        "load_kwh_per_customer_in_bin": np.where(is_res, rng.lognormal(np.log(10000.0), 0.35, n),
                                                 np.clip(rng.lognormal(np.log(150000.0), 1.2, n), 1e4, 5e7)),
        "elec_price_multiplier": rng.uniform(0.9, 1.1, n), "elec_price_escalator": rng.uniform(-0.01, 0.01, n),
        "economic_lifetime_yrs": 25, "loan_term_yrs": np.where(is_res, 20, 30), "inflation_rate": 0.025,
        "pv_degradation_factor": 0.005, "down_payment_fraction": np.where(is_res, 0.3, 1.0), "tax_rate": 0.2574,
        "real_discount_rate": np.where(is_res, 0.05, 0.0378), "itc_fraction_of_capex": 0.3,
        "system_capex_per_kw": np.where(is_res, 4637.5, 1672.9),
        "system_capex_per_kw_combined": np.where(is_res, 4500.0, 1600.0),
        "batt_capex_per_kwh_combined": np.where(is_res, 431.0, 197.3), "cap_cost_multiplier": rng.uniform(0.9, 1.2, n),
        "value_of_resiliency_usd": np.where(rng.random(n) < 0.2, rng.uniform(0.0, 300.0, n), 0.0),
        "customers_in_bin": rng.uniform(10, 500, n),
    }).set_index("agent_id", drop=False)
    rows = []
    for u in range(n_util):
        for rc in ("R", "C"):
            if rng.random() < 0.1:
                k = int(rng.integers(0, n_tariffs))
                rows.append({"tech": "solar", "rate_id_alias": 5000 + len(rows), "json": raws[k], "eia_id": u,
                             "res_com": rc, "min_kw_limit": 0.0, "max_kw_limit": 10.0 if rc == "R" else 200.0,
                             "one_time_charge": float(rng.uniform(0, 500))})
    return df, store, pd.DataFrame(rows)


# ------------------------------------------------ national population by pieces
STATE_SEED0 = 20265000          # agents of state s: default_rng(STATE_SEED0 + 7919 * s)
CUST_SEED0 = 20266000           # customers in bin of state s: default_rng(CUST_SEED0 + 7919 * s)


def _state_seed(s: int, seed0: int) -> int:
    return int(seed0) + 7919 * int(s)


def state_member_sectors(config: str, s: int, n_s: int, seed0: int = STATE_SEED0) -> np.ndarray:
    """Sector code (0 res, 1 com) of every member of state s of a national
    population by pieces: the first draw of the state's agent stream, so any
    rank can know a split state's groups without generating its agents."""
    sector = CONFIGS[config][1]
    if sector == "res":
        return np.zeros(int(n_s), np.int64)
    if sector == "com":
        return np.ones(int(n_s), np.int64)
    return np.where(np.random.default_rng(_state_seed(s, seed0)).random(int(n_s)) < 0.75, 0, 1).astype(np.int64)


def state_id_base(sizes) -> np.ndarray:
    """First agent_id of each state (ids are state-major, members in order)."""
    sizes = np.asarray(sizes, np.int64)
    return np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)


def shard_population(tables: PopTables, plan, rank: int, seed0: int = STATE_SEED0,
                     cust_seed0: int = CUST_SEED0):
    """One rank's agents of a national population by pieces (partition.
    ShardPlan): state s's agents are make_population(state_pool=[s]) drawn
    from their own stream against the shared tables, sliced to the rank's
    member range.  Returns (Population, loop agent columns: agent_id (state-
    major global ids), state, sector, county, customers_in_bin, member)."""
    sizes = np.asarray(plan.sizes, np.int64)
    base = state_id_base(sizes)
    cols, county, st, mem, cust, aid = [], [], [], [], [], []
    for s, lo, hi in plan.pieces[rank]:
        n_s = int(sizes[s])
        p = make_population(tables.config, n_s, tables=tables, agent_seed=_state_seed(s, seed0),
                            state_pool=[s], state_mix="uniform")
        sl = slice(lo, hi)
        cols.append({k: np.asarray(v)[sl] for k, v in p.cols.items()})
        county.append(np.asarray(p.county_ix)[sl])
        st.append(np.full(hi - lo, s, np.int64))
        mem.append(np.arange(lo, hi, dtype=np.int64))
        aid.append(base[s] + np.arange(lo, hi, dtype=np.int64))
        is_res = (np.asarray(p.cols["flags"]) & 1).astype(bool)
        crng = np.random.default_rng(_state_seed(s, cust_seed0))
        c = np.where(is_res, crng.lognormal(np.log(400.0), 0.5, n_s), crng.lognormal(np.log(40.0), 0.5, n_s))
        cust.append(c[sl])
    keys = list(cols[0].keys()) if cols else list(empty_columns(0).keys())
    merged = {k: np.concatenate([c[k] for c in cols]) if cols else empty_columns(0)[k] for k in keys}
    tariffs = tables.tt.array()
    n_scratch = assign_scratch(merged, tariffs, tables.switches)
    state = np.concatenate(st) if st else np.zeros(0, np.int64)
    metering = CONFIGS[tables.config][2]
    pop = Population(shapes=tables.shapes, cfs=tables.cfs, wholesale=tables.wholesale, tariffs=tariffs,
                     switches=tables.switches, cols=merged, n_scratch=n_scratch, config=tables.config,
                     state_ix=state.astype(np.int16),
                     demand=tables.tt.demand_array() if metering == "nem_dc" else None,
                     county_ix=np.concatenate(county) if county else np.zeros(0, np.int32))
    sector = np.where((np.asarray(merged["flags"]) & 1) != 0, 0, 1).astype(np.int64)
    agents = {"agent_id": np.concatenate(aid) if aid else np.zeros(0, np.int64), "state": state,
              "sector": sector, "county": np.asarray(pop.county_ix, np.int64),
              "customers_in_bin": np.concatenate(cust) if cust else np.zeros(0),
              "member": np.concatenate(mem) if mem else np.zeros(0, np.int64)}
    return pop, agents


def split_state_members(config: str, plan, seed0: int = STATE_SEED0):
    """({s: member sectors}, {s: member agent ids}) of every split state of
    the plan (partition.split_groups' inputs), the same on every rank."""
    base = state_id_base(plan.sizes)
    sec, ids = {}, {}
    for s in plan.split_states():
        n_s = int(plan.sizes[s])
        sec[s] = state_member_sectors(config, s, n_s, seed0)
        ids[s] = base[s] + np.arange(n_s, dtype=np.int64)
    return sec, ids
