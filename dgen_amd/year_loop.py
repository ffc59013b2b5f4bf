"""Device model-year loop (BASELINE config C5).

The reference's year loop (`dgen_model.py:245-462`) restricted to the hot path
and the steps that consume it, kept resident on the GPU from one model year to
the next:

    per-year inputs      elec.apply_* merges (elec.py:29-409, dgen_model.py:252-292)
                         -> dgen_year_inputs: per-year tables compiled on the
                         host (dgen_amd.market.YearTables), gathered into the
                         resident SoA columns (prices, financing, ITC,
                         degradation, escalator, load growth, VOR); the frame
                         is rebuilt from its base columns every year
                         (dgen_model.py:245-247)
    first-year market    elec.estimate_initial_market_shares (elec.py:701-765,
                         dgen_model.py:390-393) -> dgen_initial_market_shares
                         from the state starting capacities
    sizing               size_chunk -> dgen_size_agents (dgen_model.py:309-384)
    max market share     calc_max_market_share (ff:1264-1310) -> k_max_market_share
    diffusion            calc_diffusion_solar (diffusion_functions_elec.py:24-156)
                         -> k_diffusion
    battery attachment   _allocate_battery_adopters_integer
                         (attachment_rate_functions.py:58-138) -> k_batt_attach
                         over (state, sector) groups
    state hourly export  export_state_hourly_with_storage_mix (:141-206)
                         -> k_export_weights + k_state_hourly
    state totals         last_year_installed_capacity groupby state
                         (dgen_model.py:437-440) -> k_segment_sums, then ONE
                         all-reduce per year (RCCL over xGMI on GPU tensors)
    carry                market_last_year (diffusion_functions_elec.py:131-150,
                         dgen_model.py:417-427): last year's market share,
                         adopters, market value and cumulative PV / battery
                         capacity stay on device as the next year's inputs

Sharding: a rank owns pieces of states -- whole states (`rank_states`, or a
dgen_amd.partition.ShardPlan) or member ranges of a state split across ranks
for balance (plan_partition).  Per-state totals and 8760-h rows are sums of
fixed 8192-member chunk partials in chunk order (bit-identical however the
states are cut), merged by ONE all-reduce per year; a split state's
(state, sector) attachment groups gather their new adopters (one more
all-reduce of disjoint positions) and are allocated whole on every rank that
holds a piece (the reference allocates on the gathered frame,
dgen_model.py:408-427).  The first model year gathers the split groups'
developable weights the same way for the initial market shares.  A year is a
generator of exchange requests (`year_steps`): run_year drives it with the
process group's all-reduce, `run_lockstep` with an in-process sum over shards
(tests).  Nothing here runs on the CPU except index bookkeeping done once.

Synthetic stand-ins (the DB tables are not available offline): Bass
parameters per (state, sector), the max-market-share curves, storage
attachment rates per state, customers per agent, the per-year input tables
(built from the 2026 rows of the reference's input CSVs with learning /
growth trajectories) and the state starting capacities
(`LoopTables.synthetic`).  The developable weight is the agent's customers
in bin, as calculate_developable_customers_and_load sets it (elec.py:414-423).
"""
from __future__ import annotations

import ctypes
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import pandas as pd

from . import _lib
from .attachment import ATTACH_IN, ATTACH_OUT, AttachIn, AttachOut
from .attachment import _bind as _bind_attach
from .attachment import export_weights, state_hourly, state_hourly_combined, string_ranks
from .diffusion import DIFF_IN, DIFF_OUT, DiffIn, DiffOut, MmsTable, mms_table
from .diffusion import _bind as _bind_diff
from .dist import allreduce_sum
from .partition import REDUCE_CHUNK, ChunkLayout, SplitGroups, chunk_layout
from .synth import STATES

SECTORS = ("res", "com")
TOTAL_COLS = ["system_kw_cum", "batt_kw_cum", "batt_kwh_cum", "number_of_adopters", "n_agents"]
LOOP_YEARS = (2022, 2050)       # the years the synthetic input tables cover


# Brent depth bound E as a function of L = load / naep (kW) with the optimum at
# the bracket's bound (scipy 1.15.3 probes): the sizing work
# of an agent is one hourly scan plus E objective evaluations
E_BOUND_L = np.array([3.0, 5.0, 7.5, 10.0, 20.0, 50.0, 100.0, 200.0, 500.0, 1000.0, 4444.0])
E_BOUND_E = np.array([1.0, 2.0, 2.0, 3.0, 4.0, 6.0, 8.0, 9.0, 11.0, 13.0, 16.0])
# device cost of one evaluation relative to the agent's hourly scan (C3 at 1M:
# k_size 9.3 ms over ~2.5 evaluations per agent vs k_hourly_batt 25 ms)
EVAL_COST = 0.15


def predicted_work(load_kwh, naep) -> np.ndarray:
    """Predicted device work per agent: 1 (the 8760-h scan) + EVAL_COST x the
    Brent-depth bound E(L), L = load_kwh / naep, interpolated in log L."""
    L = np.asarray(load_kwh, np.float64) / np.maximum(np.asarray(naep, np.float64), 1e-9)
    E = np.interp(np.log(np.maximum(L, 1e-12)), np.log(E_BOUND_L), E_BOUND_E)
    return 1.0 + EVAL_COST * E


def population_work(pop) -> np.ndarray:
    """predicted_work of a synth.Population's agents (naep from its cf rows)."""
    naep = np.asarray(pop.cfs, np.float64).sum(axis=1) / 1e6
    return predicted_work(pop.cols["load_kwh"], naep[np.asarray(pop.cols["cf_row"], np.int64)])


def balanced_states(state_work, world: int) -> List[np.ndarray]:
    """Whole states onto `world` ranks, largest predicted work first, each to
    the rank with the least work so far (ties: the lowest rank); every rank
    computes the same assignment from the same weights.  Returns each rank's
    states, ascending."""
    w = np.asarray(state_work, np.float64)
    if world < 1:
        raise ValueError("bad world")
    load = np.zeros(world)
    owner = np.empty(w.size, np.int64)
    for s in np.argsort(-w, kind="stable"):
        r = int(np.argmin(load))
        owner[s] = r
        load[r] += w[s]
    return [np.nonzero(owner == r)[0].astype(np.int64) for r in range(world)]


def rank_states(rank: int, world: int, n_states: int = len(STATES),
                state_work=None) -> np.ndarray:
    """States owned by `rank` (every state on exactly one rank; whole states
    keep the attachment groups and state sums local).  With `state_work`
    (predicted work per state, e.g. the bincount of population_work over the
    agents' states) the states are balanced by it
    (balanced_states); without, s % world == rank."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank / world")
    if state_work is not None:
        w = np.asarray(state_work, np.float64)
        if w.size != n_states:
            raise ValueError("state_work must have one entry per state")
        return balanced_states(w, world)[rank]
    return np.arange(rank, n_states, world, dtype=np.int64)


def merge_state_rows(local_rows, local_states: Sequence[int], n_states: int):
    """Scatter this rank's per-state rows [S_local, k] into the full [n_states, k]
    table and all-reduce (SUM) it over the process group: states are disjoint
    across ranks, so the sum is the gather (RCCL on GPU tensors, gloo on CPU)."""
    import torch
    full = torch.zeros((n_states,) + tuple(local_rows.shape[1:]), dtype=local_rows.dtype,
                       device=local_rows.device)
    if len(local_states):
        idx = torch.as_tensor(np.asarray(local_states, np.int64), device=local_rows.device)
        full.index_copy_(0, idx, local_rows)
    return allreduce_sum(full)


@dataclass
class LoopTables:
    """Per-(state, sector) Bass parameters, max-market-share curves (the
    reference's max_market_share_df format), per-state storage attachment
    rates; identical on every rank (fixed seed)."""
    bass: pd.DataFrame
    mms_df: pd.DataFrame
    attach_rate: np.ndarray                  # [n_states]
    inputs: Dict[str, pd.DataFrame] = field(default_factory=dict)   # market.YearTables roles
    inflation_rate: float = 0.025
    caps: Optional[pd.DataFrame] = None      # state starting capacities (elec.py:621-652)

    @staticmethod
    def synthetic_inputs(rng, n_counties: int = 3100):
        """Per-year input tables in the reference's formats (market.YearTables
        roles), from the 2026 rows of its CSVs (capex
        pv_price_atb23_mid.csv:14, battery pv_plus_batt_prices_FY23_mid.csv:14,
        financing_atb_FY23.csv:14, degradation pv_tech_performance_defaultFY19
        .csv:14) with learning / growth trajectories; ITC steps down after
        2032 as the federal schedule does."""
        years = np.arange(LOOP_YEARS[0], LOOP_YEARS[1] + 1)
        k = (years - 2026).astype(np.float64)
        sec = list(SECTORS)
        capex = {"res": 4637.5, "com": 1672.9}
        comb = {"res": 4500.0, "com": 1600.0}
        batt = {"res": 431.0, "com": 197.3}
        pv_price = pd.DataFrame([{"year": int(y), "sector_abbr": s, "system_capex_per_kw": capex[s] * 0.98 ** kk}
                                 for y, kk in zip(years, k) for s in sec])
        pvb = pd.DataFrame([{"year": int(y), "sector_abbr": s, "system_capex_per_kw": comb[s] * 0.98 ** kk,
                             "batt_capex_per_kwh": batt[s] * 0.97 ** kk} for y, kk in zip(years, k) for s in sec])
        pv_tech = pd.DataFrame([{"year": int(y), "sector_abbr": s, "pv_degradation_factor": 0.005}
                                for y in years for s in sec])
        itc = pd.DataFrame([{"year": int(y), "tech": "solar", "sector_abbr": s,
                             "itc_fraction_of_capex": 0.3 if y <= 2032 else (0.26 if y == 2033 else
                                                                            (0.22 if y == 2034 else 0.0))}
                            for y in years for s in sec])
        fin = pd.DataFrame([{"year": int(y), "sector_abbr": s, "economic_lifetime_yrs": 25,
                             "loan_term_yrs": 20 if s == "res" else 30,
                             "down_payment_fraction": 0.3 if s == "res" else 1.0,
                             "real_discount_rate": 0.05 if s == "res" else 0.0378, "tax_rate": 0.2574}
                            for y in years for s in sec])
        cty = np.arange(n_counties)
        rows_lg, rows_ep = [], []
        for s in sec:
            g = rng.uniform(0.5, 1.5, n_counties)
            base = rng.uniform(0.9, 1.1, n_counties)
            drift = rng.uniform(-0.01, 0.015, n_counties)
            for y, kk in zip(years, k):
                rows_lg.append(pd.DataFrame({"year": int(y), "sector_abbr": s, "county_id": cty,
                                             "load_multiplier": 1.0 + 0.01 * kk * g}))
                rows_ep.append(pd.DataFrame({"year": int(y), "sector_abbr": s, "county_id": cty,
                                             "elec_price_multiplier": base * (1.0 + drift) ** kk}))
        vor = pd.DataFrame([{"state_abbr": st, "sector_abbr": s,
                             "value_of_resiliency_usd": float(rng.uniform(0, 300)) if rng.random() < 0.2 else 0.0}
                            for st in STATES for s in sec])
        return {"load_growth": pd.concat(rows_lg, ignore_index=True),
                "elec_price": pd.concat(rows_ep, ignore_index=True), "pv_tech": pv_tech,
                "pv_price": pv_price, "pv_plus_batt_price": pvb, "vor": vor, "financing": fin, "itc": itc}

    @staticmethod
    def synthetic_caps(rng):
        """State starting capacities (the state_starting_capacities_to_model
        table's shape, elec.py:621-652): PV and storage MW / MWh / system
        counts per (state, sector); a few states without a row."""
        rows = []
        for i, st in enumerate(STATES):
            for s in SECTORS:
                if i % 17 == 5:
                    continue
                mw = float(rng.uniform(5, 2500 if s == "res" else 1500))
                rows.append({"state_abbr": st, "sector_abbr": s, "system_mw": mw,
                             "batt_mw": mw * float(rng.uniform(0.0, 0.08)),
                             "batt_mwh": mw * float(rng.uniform(0.0, 0.3)),
                             "pv_systems_count": mw * 1000.0 / (7.0 if s == "res" else 120.0),
                             "batt_systems_count": mw * float(rng.uniform(0, 30))})
        return pd.DataFrame(rows)

    @staticmethod
    def synthetic(seed: int = 20260105, n_counties: int = 3100) -> "LoopTables":
        rng = np.random.default_rng(seed)
        rows = []
        for s in STATES:
            for sec in SECTORS:
                rows.append({"state_abbr": s, "sector_abbr": sec, "tech": "solar",
                             "bass_param_p": float(rng.uniform(0.001, 0.01)),
                             "bass_param_q": float(rng.uniform(0.2, 0.5)),
                             "teq_yr1": float(rng.uniform(1.0, 11.0))})
        bass = pd.DataFrame(rows)
        pb = np.round(np.arange(0, 302) * 0.1, 1)
        pb[-1] = 30.1
        recs = []
        for sec, (a, k) in (("res", (0.93, 0.16)), ("com", (0.85, 0.28))):
            mms = a / (1.0 + np.exp(k * (pb - 8.0))) / (1.0 / (1.0 + np.exp(-k * 8.0)))
            mms = np.minimum(mms, 1.0)
            for p, v in zip(pb, mms):
                recs.append({"payback_period": float(p), "sector_abbr": sec,
                             "max_market_share": float(v), "metric": "payback_period",
                             "source": "synthetic", "business_model": "host_owned"})
        attach = rng.uniform(0.05, 0.35, len(STATES))
        irng = np.random.default_rng(seed + 1)
        return LoopTables(bass=bass, mms_df=pd.DataFrame(recs), attach_rate=attach,
                          inputs=LoopTables.synthetic_inputs(irng, n_counties),
                          caps=LoopTables.synthetic_caps(irng))


def loop_agents(pop, agent_id0: int = 0, seed: int = 20260205) -> Dict[str, np.ndarray]:
    """Per-agent columns of the diffusion / attachment steps for a synthetic
    population (caller order): agent_id, state, sector, county,
    customers_in_bin (the initial customers; apply_load_growth scales the
    non-residential ones per year)."""
    n = len(pop.cols["load_kwh"])
    rng = np.random.default_rng(seed + int(agent_id0))
    is_res = (np.asarray(pop.cols["flags"]) & 1).astype(bool)
    cust = np.where(is_res, rng.lognormal(np.log(400.0), 0.5, n), rng.lognormal(np.log(40.0), 0.5, n))
    county = (np.asarray(pop.county_ix, np.int64) if pop.county_ix is not None
              else np.zeros(n, np.int64))
    return {"agent_id": np.arange(agent_id0, agent_id0 + n, dtype=np.int64),
            "state": np.asarray(pop.state_ix, dtype=np.int64),
            "sector": np.where(is_res, 0, 1).astype(np.int64),
            "county": county, "customers_in_bin": cust}


@dataclass
class YearResult:
    year: int
    totals: object                              # [n_states, 5] float64, all-reduced
    hourly: Optional[object]                    # [n_states, 8760] float64 MW, all-reduced
    seconds: float
    per_agent: Dict[str, object] = field(default_factory=dict)   # device order


class YearLoop:
    """Resident multi-year loop over one rank's shard (see module docstring).

    engine: a loaded Engine (tables set); pop: synth.Population of this rank's
    agents; agents: loop_agents(pop, ...); hourly_export: per-state 8760-h sums
    each year; hourly_chunk: None sizes the shard once with hourly planes and
    exports from them in place (105 KB / agent of HBM), an int sizes the shard
    without planes and re-runs only the 8760-h scan (dgen_hourly_planes) in
    chunks of that many agents into a reusable plane buffer for the export
    (the 2.5M-agents-per-GPU national case).  export: how the per-state
    8760-h rows are made -- "with_batt" (the sizing scan writes the
    with-battery plane alone, 35 KB / agent, and the export recomputes the
    load and PV-only net load from the profile rows: dgen_state_hourly_rows),
    "planes" (the three planes at sizing), "chunked" (hourly_chunk's re-run
    scans), or "auto": with_batt where the scan supports it (daily plan, no
    loss model, no demand machinery) and its plane fits in HBM, else planes
    / chunked as hourly_chunk says.  Every form gives the same rows, bit for
    bit."""

    def __init__(self, engine, pop, agents: Dict[str, np.ndarray], tables: LoopTables,
                 first_year: int = 2026, hourly_export: bool = True,
                 hourly_chunk: Optional[int] = None, order: Optional[np.ndarray] = None,
                 plan=None, split: Optional[SplitGroups] = None, export: str = "auto"):
        import torch
        from .engine import profile_order
        # plan and split come together: a split state's members must be
        # numbered by the plan (agents["member"]) and its groups gathered
        # (split), or its rows, initial shares and allocation go wrong silently
        if split is not None and plan is None:
            raise ValueError("YearLoop: split groups given without the plan they were built from")
        if plan is not None and plan.split_states():
            if split is None:
                raise ValueError(f"YearLoop: the plan splits states {plan.split_states()} across ranks "
                                 "but no split groups were given (partition.split_groups)")
            if "member" not in agents:
                raise ValueError("YearLoop: the plan splits states across ranks but agents['member'] "
                                 "(each agent's index within its state) is missing")
        self.eng, self.tables = engine, tables
        self.first_year = int(first_year)
        self.hourly_export, self.hourly_chunk = bool(hourly_export), hourly_chunk
        n = len(pop.cols["load_kwh"])
        self.n = n
        st_all = np.asarray(agents["state"], np.int64)
        # member index of each agent within its state (caller order); a shard
        # of whole states numbers them itself, a piece of a split state gets
        # them from the plan (agents["member"])
        if "member" in agents:
            member = np.asarray(agents["member"], np.int64)
        else:
            member = np.zeros(n, np.int64)
            for s in np.unique(st_all):
                ix = np.flatnonzero(st_all == s)
                member[ix] = np.arange(ix.size)
        # device order: by (state, reduction chunk), then billing path and
        # profile rows (profile_order): each chunk is one contiguous, canonical
        # run of device rows
        self.chunk = int(plan.chunk) if plan is not None else REDUCE_CHUNK
        gkey = st_all * (1 << 32) + member // self.chunk
        perm = (profile_order(pop.cols, group=gkey) if order is None
                else np.asarray(order, np.int64))
        self.perm = perm
        inv = np.empty(n, np.int64)
        inv[perm] = np.arange(n, dtype=np.int64)
        self.batch = engine.upload_agents(pop.cols, n_scratch=pop.n_scratch, order=perm)
        dev = engine.dev
        f64 = lambda a: torch.as_tensor(np.asarray(a, np.float64)[perm], device=dev)
        # per-year inputs: key codes in device order, initial load / customers
        from .market import YearInputs, YearTables
        frame = pd.DataFrame({"state_abbr": [STATES[s] for s in agents["state"][perm]],
                              "sector_abbr": [SECTORS[c] for c in agents["sector"][perm]],
                              "county_id": np.asarray(agents["county"], np.int64)[perm]})
        self.inv = inv
        self.caller_frame = (list(frame["state_abbr"].to_numpy()[inv]), list(frame["sector_abbr"].to_numpy()[inv]))
        self.year_tables = YearTables(frame, tables.inputs, tables.inflation_rate)
        load0 = np.asarray(pop.cols["load_kwh"], np.float64)[perm]
        cust0 = np.asarray(agents["customers_in_bin"], np.float64)[perm]
        self.year_inputs = YearInputs(engine, self.year_tables, load0, cust0, load0 * cust0)
        self.loop_cols = {k: torch.empty(n, dtype=torch.float64, device=engine.dev)
                          for k in ("customers_in_bin", "load_kwh_in_bin")}
        self.frame = frame
        st, sec = agents["state"], agents["sector"]
        self.state_caller = st
        self.sector_caller = sec
        # per-agent Bass parameters (the reference's merge on (state, sector), :41-44)
        b = tables.bass[tables.bass["tech"] == "solar"].set_index(["state_abbr", "sector_abbr"])
        keys = [(STATES[s], SECTORS[c]) for s, c in zip(st, sec)]
        uk = {k: i for i, k in enumerate(dict.fromkeys(keys))}
        kix = np.array([uk[k] for k in keys], np.int64)
        tab = b.reindex(list(uk.keys()))
        self.bass = {c: f64(tab[src].to_numpy(np.float64)[kix]) for c, src in
                     (("bass_p", "bass_param_p"), ("bass_q", "bass_param_q"), ("teq_yr1", "teq_yr1"))}
        # customers_in_bin / developable weight: the year's loop column
        # (calculate_developable_customers_and_load, elec.py:414-423)
        self.cust = self.loop_cols["customers_in_bin"]
        self.dev_w = self.cust
        # max market share table, curve row per agent (sector)
        mt, rows, fmin, min_pb, max_pb = mms_table(tables.mms_df)
        self.mms_tab = torch.as_tensor(mt, device=dev)
        self.mms_tb = MmsTable(mms=self.mms_tab.data_ptr(), n_rows=mt.shape[0], n_factors=mt.shape[1],
                               factor_min=fmin, pad=0, min_pb=min_pb, max_pb=max_pb)
        self.mms_row = torch.as_tensor(np.array([rows.get(SECTORS[c], -1) for c in sec],
                                                np.int32)[perm], device=dev)
        # (state, sector) attachment groups in caller (reference row) order;
        # the groups of split states are allocated whole from a gather (split)
        self.split = split
        split_states = set(plan.split_states()) if plan is not None else set()
        g_keys = list(zip(st.tolist(), sec.tolist()))
        g_first: Dict = {}
        for i, k in enumerate(g_keys):
            if k[0] in split_states:
                continue
            g_first.setdefault(k, []).append(i)
        g_idx = np.concatenate([np.asarray(v, np.int64) for v in g_first.values()]) if g_first else \
            np.zeros(0, np.int64)
        g_off = [0] + np.cumsum([len(v) for v in g_first.values()]).tolist()
        g_rate = [tables.attach_rate[k[0]] for k in g_first]
        aid_local = string_ranks(agents["agent_id"])[g_idx] if g_idx.size else np.zeros(0, np.int64)
        # split groups this rank holds members of: the whole group is allocated
        # here; own members sit at [own_off, own_off + own_cnt) of the group
        self.sg = []          # (buffer offset, group size, own offset, own device rows [torch])
        aid_parts, pos = [aid_local], int(g_idx.size)
        self.m_local = int(g_idx.size)
        if split is not None:
            for j, (key, G) in enumerate(zip(split.keys, split.size)):
                cnt = int(split.own_cnt[j])
                if cnt == 0:
                    continue
                s_, c_ = key
                own = np.flatnonzero((st == s_) & (sec == c_))           # caller order = member order
                if own.size != cnt:
                    raise ValueError(f"split group {key}: {own.size} members here, plan says {cnt}")
                self.sg.append((int(split.buf_off[j]), int(G), int(split.own_off[j]),
                                torch.as_tensor(inv[own], device=dev), pos))
                aid_parts.append(split.aid_rank[j])
                g_off.append(g_off[-1] + int(G))
                g_rate.append(tables.attach_rate[s_])
                pos += int(G)
        self.m_attach = pos
        self.g_dev = torch.as_tensor(inv[g_idx], device=dev)
        self.g_off = torch.as_tensor(np.asarray(g_off, np.int64), device=dev)
        self.g_n = len(g_off) - 1
        self.g_rate = torch.as_tensor(np.asarray(g_rate, np.float64), device=dev)
        self.aid_rank = torch.as_tensor(np.concatenate(aid_parts).astype(np.int64), device=dev)
        self.n_buf = split.n_buf if split is not None else 0
        # reduction chunks (dgen_amd.partition): fixed 8192-member chunks of each
        # state, device rows ascending within a chunk; per-state rows are the
        # chunk partials summed in chunk order
        self.state_dev_order = st_all[perm]                   # state of each device row
        self.layout: ChunkLayout = chunk_layout(self.state_dev_order, member[perm], len(STATES), plan,
                                                chunk=self.chunk)
        self.s_dev_idx = self.layout.seg_dev
        self.s_off = self.layout.seg_off
        self.s_dev = torch.as_tensor(self.s_dev_idx, device=dev)
        self.local_states = sorted(set(self.state_dev_order.tolist()))
        # carry (market_last_year), device order
        z = lambda: torch.zeros(n, dtype=torch.float64, device=dev)
        self.carry = {k: z() for k in ("market_share_last_year", "adopters_cum_last_year",
                                       "market_value_last_year", "system_kw_cum_last_year",
                                       "batt_kw_cum_last_year", "batt_kwh_cum_last_year")}
        self.export_mode = self._pick_export(engine, n, hourly_export, hourly_chunk, export)
        if self.export_mode == "with_batt":
            self.out = engine.alloc_outputs(n, hourly="with_batt")
        else:
            self.out = engine.alloc_outputs(n, hourly=self.export_mode == "planes")
        self.c_out = engine.c_outputs(self.out)
        if self.export_mode == "chunked":
            ch = min(int(hourly_chunk), max(n, 1))
            self._chunk_planes = {k: torch.empty(_lib.NH * ch, dtype=torch.float32, device=dev)
                                  for k in _lib.OUTPUT_HOURLY}
        self.Ld, self.La = _bind_diff(engine.lib), _bind_attach(engine.lib)

    @staticmethod
    def _pick_export(engine, n: int, hourly_export: bool, hourly_chunk, export: str) -> str:
        if not hourly_export:
            return "none"
        cfg, T = engine.cfg, engine.tables
        dc = T.n_demand > 0 and (cfg.skip_demand_charges == 0 or T.peak_units != 0)
        wo_ok = cfg.batt_loss_model != 1 and cfg.batt_update_hours == 24 and not dc
        legacy = "planes" if hourly_chunk is None else "chunked"
        if export == "auto":
            if not wo_ok:
                return legacy
            import torch
            free, _ = torch.cuda.mem_get_info(engine.dev)
            return "with_batt" if n * _lib.NH * 4 <= 0.6 * free else legacy
        if export == "with_batt" and not wo_ok:
            raise ValueError("export='with_batt' needs the daily plan, no loss model and no demand machinery")
        if export == "chunked" and hourly_chunk is None:
            raise ValueError("export='chunked' needs hourly_chunk")
        if export not in ("with_batt", "planes", "chunked"):
            raise ValueError(f"unknown export mode {export!r}")
        return export

    # --------------------------------------------------------------- steps
    def apply_year_inputs(self, year: int):
        """This year's elec.apply_* merges as device gathers (dgen_year_inputs)
        into the resident SoA columns and the loop's customers / load in bin."""
        self.year_inputs.apply(year, self.batch.cols, self.loop_cols)
        # the year's lifetimes pick the sizing kernels' lanes-per-agent form
        # (k_size / k_batt_finance treat years <= 32 as active in the two-agent
        # form); the chunked export's sub-batches copy it from here
        self.batch.c_agents.max_years = self.year_inputs.max_years(year)

    def _initial_market_steps(self):
        """First model year: elec.estimate_initial_market_shares (elec.py:701-765)
        on device from the state starting capacities, into the carry.  Its
        per-(state, sector, tech) group sums need whole groups: a split group's
        developable weights are gathered (exchange) and the group is computed
        whole here, own members' rows kept (a generator: yields the gather)."""
        import torch
        from .market import initial_market_shares
        caps = self.tables.caps if self.tables.caps is not None else pd.DataFrame(
            columns=["state_abbr", "sector_abbr", "system_mw", "batt_mw", "batt_mwh", "pv_systems_count",
                     "batt_systems_count"])
        st, sec = self.caller_frame          # pandas' group sums visit the frame (caller) order
        n = self.n
        w, cx = self.dev_w, self.batch.cols["capex"]
        if self.split is None or self.n_buf == 0:
            ini = initial_market_shares(self.eng, st, sec, ["solar"] * n, w, cx, caps, dev_index=self.inv)
        else:
            buf = torch.zeros(self.n_buf, dtype=torch.float64, device=self.eng.dev)
            for b0, G, o, rows, _ in self.sg:
                buf[b0 + o:b0 + o + rows.numel()] = w.index_select(0, rows)
            buf = yield buf
            # extended frame: this rank's rows outside split groups, then every
            # split group it holds members of, whole, in group (caller) order
            split_keys = {(k[0], k[1]) for k in self.split.keys}
            stc = np.asarray(self.state_caller, np.int64)
            seco = np.asarray(self.sector_caller, np.int64)
            keep = np.array([(a, b) not in split_keys for a, b in zip(stc.tolist(), seco.tolist())], bool)
            rows_local = np.flatnonzero(keep)
            fst = [st[i] for i in rows_local]
            fsec = [sec[i] for i in rows_local]
            # value columns in frame order: this rank's rows outside split
            # groups, then the gathered groups (the frame and its values have
            # one row each, initial_market_shares' contract)
            loc_dev = torch.as_tensor(self.inv[rows_local], device=self.eng.dev)
            L = int(rows_local.size)
            dev_index = [np.arange(L, dtype=np.int64)]
            vals_w, vals_c = [w.index_select(0, loc_dev)], [cx.index_select(0, loc_dev)]
            ext = L
            take = [(0, loc_dev)]
            for (b0, G, o, rows, _), key in zip(self.sg, [k for k, c in zip(self.split.keys, self.split.own_cnt)
                                                          if c > 0]):
                fst += [STATES[key[0]]] * G
                fsec += [SECTORS[key[1]]] * G
                dev_index.append(np.arange(ext, ext + G, dtype=np.int64))
                vals_w.append(buf[b0:b0 + G])
                cg = torch.zeros(G, dtype=torch.float64, device=self.eng.dev)
                cg[o:o + rows.numel()] = cx.index_select(0, rows)
                vals_c.append(cg)
                take.append((ext + o, rows))
                ext += G
            ini = initial_market_shares(self.eng, fst, fsec, ["solar"] * len(fst), torch.cat(vals_w),
                                        torch.cat(vals_c), caps, dev_index=np.concatenate(dev_index))
            for k in list(ini.keys()):
                v = ini[k]
                if isinstance(v, torch.Tensor) and v.dim() == 1 and v.numel() == ext and k != "agent_count":
                    own = torch.empty(n, dtype=v.dtype, device=v.device)
                    for e0, rows in take:
                        own.index_copy_(0, rows, v[e0:e0 + rows.numel()])
                    ini[k] = own
        c = self.carry
        for k in ("market_share_last_year", "adopters_cum_last_year", "market_value_last_year",
                  "system_kw_cum_last_year", "batt_kw_cum_last_year", "batt_kwh_cum_last_year"):
            c[k].copy_(ini[k])
        return ini

    def initial_market(self, exchange=None):
        return _drive(self._initial_market_steps(), exchange or allreduce_sum)

    def _max_market_share(self):
        import torch
        eng, n = self.eng, self.n
        b = torch.empty(n, dtype=torch.float64, device=eng.dev)
        fct = torch.empty(n, dtype=torch.int64, device=eng.dev)
        mms = torch.empty(n, dtype=torch.float64, device=eng.dev)
        _lib.check(self.Ld.dgen_max_market_share(eng.ctx, ctypes.byref(self.mms_tb),
                                                 self.out["payback_period"].data_ptr(),
                                                 self.mms_row.data_ptr(), n, b.data_ptr(),
                                                 fct.data_ptr(), mms.data_ptr(), eng.stream_handle()),
                   "dgen_max_market_share")
        return mms

    def _diffusion(self, mms, first: bool):
        import torch
        eng, n, c = self.eng, self.n, self.carry
        src = {"max_market_share": mms, "market_share_last_year": c["market_share_last_year"],
               "bass_p": self.bass["bass_p"], "bass_q": self.bass["bass_q"],
               "teq_yr1": self.bass["teq_yr1"], "developable_agent_weight": self.dev_w,
               "system_kw": self.out["system_kw"], "system_capex_per_kw": self.batch.cols["capex"],
               "adopters_cum_last_year": c["adopters_cum_last_year"],
               "market_value_last_year": c["market_value_last_year"],
               "system_kw_cum_last_year": c["system_kw_cum_last_year"]}
        outs = {k: torch.empty(n, dtype=torch.float64, device=eng.dev) for k in DIFF_OUT}
        din = DiffIn(**{k: src[k].data_ptr() for k in DIFF_IN})
        dout = DiffOut(**{k: outs[k].data_ptr() for k in DIFF_OUT})
        _lib.check(self.Ld.dgen_diffusion(eng.ctx, ctypes.byref(din), ctypes.byref(dout), n,
                                          int(first), eng.stream_handle()), "dgen_diffusion")
        return outs

    def _attach_steps(self, new_adopters):
        """Largest-remainder battery adopters per (state, sector) group
        (k_batt_attach).  Split groups: the members' new adopters are gathered
        (yield) and each group is allocated whole, own members' results kept."""
        import torch
        eng, n, g = self.eng, self.n, self.g_dev
        dev = eng.dev
        gathered = None
        if self.n_buf:
            buf = torch.zeros(self.n_buf, dtype=torch.float64, device=dev)
            for b0, G, o, rows, _ in self.sg:
                buf[b0 + o:b0 + o + rows.numel()] = new_adopters.index_select(0, rows)
            gathered = yield buf
        M = self.m_attach

        def col(v, gather=None):
            x = torch.zeros(M, dtype=torch.float64, device=dev)
            if self.m_local:
                x[:self.m_local] = v.index_select(0, g)
            for b0, G, o, rows, p0 in self.sg:
                if gather is not None:
                    x[p0:p0 + G] = gather[b0:b0 + G]
                else:
                    x[p0 + o:p0 + o + rows.numel()] = v.index_select(0, rows)
            return x

        src = {"new_adopters": col(new_adopters, gathered), "aid_rank": self.aid_rank,
               "batt_kw": col(self.out["batt_kw"]), "batt_kwh": col(self.out["batt_kwh"]),
               "batt_kw_cum_last_year": col(self.carry["batt_kw_cum_last_year"]),
               "batt_kwh_cum_last_year": col(self.carry["batt_kwh_cum_last_year"])}
        grp = {k: torch.empty(M, dtype=torch.int64 if k == "added" else torch.float64,
                              device=dev) for k in ATTACH_OUT}
        ci = AttachIn(**{k: src[k].data_ptr() for k in ATTACH_IN})
        co = AttachOut(**{k: grp[k].data_ptr() for k in ATTACH_OUT})
        if self.g_n:
            _lib.check(self.La.dgen_batt_attach(eng.ctx, ctypes.byref(ci), ctypes.byref(co),
                                                self.g_off.data_ptr(), self.g_rate.data_ptr(),
                                                self.g_n, eng.stream_handle()), "dgen_batt_attach")
        res = {}
        for k, v in grp.items():                    # group order -> device order
            d = torch.empty(n, dtype=v.dtype, device=dev)
            if self.m_local:
                d.index_copy_(0, g, v[:self.m_local])
            for b0, G, o, rows, p0 in self.sg:
                d.index_copy_(0, rows, v[p0 + o:p0 + o + rows.numel()])
            res[k] = d
        return res

    def _state_hourly(self, w):
        """[C_local, 8760] MW: each reduction chunk's partial, chunks in layout
        order (combined per state by partition.combine_rows)."""
        import torch
        eng = self.eng
        if self.export_mode == "with_batt":
            from .attachment import state_hourly_rows
            return state_hourly_rows(eng, self.batch, self.c_out, self.out["net_with_batt"], w, self.s_dev,
                                     self.s_off)
        if self.export_mode == "planes":
            planes = (self.out["baseline"], self.out["net_pvonly"], self.out["net_with_batt"])
            return state_hourly(eng, planes, w, self.s_dev_idx, self.s_off)
        # chunked: runs of device rows get their hourly planes from the scan
        # alone (dgen_hourly_planes, from this year's sizing outputs: the run's
        # slices of self.out), then each reduction chunk's members are summed.
        # Reduction chunks are contiguous device-row ranges; a run ends on a
        # chunk boundary, so every chunk partial comes from one run.
        from .engine import AgentBatch
        if getattr(self, "_runs", None) is None:
            off = self.s_off
            starts = np.asarray([int(self.s_dev_idx[off[j]]) for j in range(len(off) - 1)], np.int64)
            ends = np.asarray([int(self.s_dev_idx[off[j + 1] - 1]) + 1 for j in range(len(off) - 1)], np.int64)
            if np.any(ends - starts != np.diff(off)):
                raise RuntimeError("reduction chunks are not contiguous device-row ranges")
            runs, j0 = [], 0
            ch = int(self.hourly_chunk)
            while j0 < len(starts):
                j1 = j0 + 1
                while j1 < len(starts) and ends[j1] - starts[j0] <= ch:
                    j1 += 1
                a, b = int(starts[j0]), int(ends[j1 - 1])
                seg = [(int(s0) - a, int(e0) - a) for s0, e0 in zip(starts[j0:j1], ends[j0:j1])]
                idx = np.concatenate([np.arange(s0, e0) for s0, e0 in seg]).astype(np.int64)
                so = np.concatenate([[0], np.cumsum([e0 - s0 for s0, e0 in seg])]).astype(np.int64)
                runs.append((a, b, idx, so))
                j0 = j1
            self._runs = runs
            mx = max((b - a for a, b, _, _ in runs), default=0)
            # the combined export plane (dgen_export_plane: 8 B per agent-hour,
            # the daily plan without the loss model) or the three float32 planes
            self._comb = eng.cfg.batt_loss_model != 1 and eng.cfg.batt_update_hours != 1
            if self._comb:
                self._chunk_comb = torch.empty(_lib.NH * max(mx, 1), dtype=torch.float64, device=eng.dev)
                self._chunk_planes = {}
            else:
                self._chunk_planes = {k: torch.empty(_lib.NH * max(mx, 1), dtype=torch.float32, device=eng.dev)
                                      for k in _lib.OUTPUT_HOURLY}
        B = self.batch
        parts = []
        for a, b, idx, so in self._runs:
            m = b - a
            cols = {k: v[a:b] for k, v in B.cols.items()}
            ca = _lib.Agents(**{name: cols[name].data_ptr() for name, _ in _lib.AGENT_COLUMNS})
            ca.max_years = B.c_agents.max_years
            sub = AgentBatch(n=m, n_scratch=B.n_scratch, cols=cols, workspace=B.workspace,
                             c_agents=ca, nb_scan=B.nb_scan, tables_gen=B.tables_gen)
            out = {k: v[a:b] for k, v in self.out.items() if v is not None}
            wc = tuple(x[a:b] for x in w)
            if self._comb:
                # the scan writes the per-agent-hour sum terms of the export
                # straight into one plane (no three planes written and re-read);
                # the per-state rows are the three-plane form's, bit for bit
                co = eng.c_outputs(out)
                plane = self._chunk_comb[:_lib.NH * m].view(_lib.NH // 4, m, 4)
                eng.export_plane(sub, co, wc, plane)
                parts.append(state_hourly_combined(eng, plane, idx, so))
                continue
            out.update({k: v[:_lib.NH * m].view(_lib.NH // 4, m, 4)
                        for k, v in self._chunk_planes.items()})
            co = eng.c_outputs(out)
            planes = (out["baseline"], out["net_pvonly"], out["net_with_batt"])
            eng.hourly_planes(sub, co)
            parts.append(state_hourly(eng, planes, wc, idx, so))
        return torch.cat(parts) if parts else torch.zeros((0, _lib.NH), dtype=torch.float64, device=eng.dev)

    def year_steps(self, year: int, keep_per_agent: bool = False):
        """One model year as a generator: it yields the tensors to be summed over
        the ranks (the split groups' gathers, the per-state table) and receives
        the sums; returns the YearResult (run_year / run_lockstep drive it)."""
        import torch
        from .partition import rows_finish, rows_table
        eng = self.eng
        first = year == self.first_year
        torch.cuda.synchronize(eng.dev)
        t0 = time.perf_counter()
        self.apply_year_inputs(year)
        eng.size(self.batch, self.out, self.c_out)
        mms = self._max_market_share()
        if first:
            yield from self._initial_market_steps()
        d = self._diffusion(mms, first)
        att = yield from self._attach_steps(d["new_adopters"])
        hourly_local = None
        if self.hourly_export:
            # the export reads the frame's last-year battery cumulative (:185)
            w = export_weights(eng, self.cust, d["number_of_adopters"],
                               self.carry["batt_kw_cum_last_year"], self.out["batt_kw"], att["added"])
            hourly_local = self._state_hourly(w)
        # per-chunk totals (dgen_model.py:437-440), then per-state rows of totals
        # and hourly sums through one all-reduce (partition.rows_table)
        sd = self.s_dev
        cols = torch.stack([d["system_kw_cum"].index_select(0, sd), att["batt_kw_cum"].index_select(0, sd),
                            att["batt_kwh_cum"].index_select(0, sd),
                            d["number_of_adopters"].index_select(0, sd),
                            torch.ones(self.n, dtype=torch.float64, device=eng.dev)])
        loc = eng.segment_sums(cols, self.s_off)                     # [C_local, 5]
        rows = loc if hourly_local is None else torch.cat([loc, hourly_local], dim=1)
        table = rows_table(rows, self.layout, eng.rows_seq_sum)
        table = yield table
        merged = rows_finish(table, self.layout, eng.rows_seq_sum)
        totals = merged[:, :5].contiguous()
        hourly = merged[:, 5:].contiguous() if hourly_local is not None else None
        per_agent = {}
        if keep_per_agent:
            per_agent = {"max_market_share": mms, **d, **att,
                         **{k + "_in": v.clone() for k, v in self.carry.items()}}
        # market_last_year carry (diffusion :131-150; batt cumulatives dm:417-427)
        c = self.carry
        c["market_share_last_year"].copy_(d["market_share"])
        c["adopters_cum_last_year"].copy_(d["number_of_adopters"])
        c["market_value_last_year"].copy_(d["market_value"])
        c["system_kw_cum_last_year"].copy_(d["system_kw_cum"])
        c["batt_kw_cum_last_year"].copy_(att["batt_kw_cum"])
        c["batt_kwh_cum_last_year"].copy_(att["batt_kwh_cum"])
        torch.cuda.synchronize(eng.dev)
        return YearResult(year=year, totals=totals, hourly=hourly,
                          seconds=time.perf_counter() - t0, per_agent=per_agent)

    def run_year(self, year: int, keep_per_agent: bool = False, exchange=None) -> YearResult:
        """One model year; exchange(t) sums t over the ranks (default: the
        process group's all-reduce, identity without one)."""
        return _drive(self.year_steps(year, keep_per_agent), exchange or allreduce_sum)

    def reset(self):
        """Back to an empty market (before the first model year)."""
        for v in self.carry.values():
            v.zero_()

    def run(self, years: Sequence[int]) -> List[YearResult]:
        return [self.run_year(int(y)) for y in years]


def _drive(gen, exchange):
    """Run a year_steps-style generator, answering each yielded tensor with
    exchange(tensor); returns the generator's value."""
    try:
        req = next(gen)
        while True:
            req = gen.send(exchange(req))
    except StopIteration as e:
        return e.value


def run_lockstep(loops: Sequence["YearLoop"], year: int, keep_per_agent: bool = False):
    """The shards of one model year run in one process, their exchanges summed
    here in shard order (what the all-reduce over their ranks returns): the
    multi-rank loop by construction on one GPU (tests)."""
    import torch
    gens = [lp.year_steps(year, keep_per_agent) for lp in loops]
    reqs = [next(g) for g in gens]
    while True:
        tot = reqs[0].clone()
        for r in reqs[1:]:
            tot += r
        done, nxt = [], []
        for g in gens:
            try:
                nxt.append(g.send(tot.clone()))
            except StopIteration as e:
                done.append(e.value)
        if done:
            if len(done) != len(gens):
                raise RuntimeError("shards disagree on the year's exchanges")
            return done
        reqs = nxt
