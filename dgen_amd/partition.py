"""Rank partition of a national population (BASELINE C5 / C4 at
8 GPUs) with states split across ranks where balance needs it.

The reference shards by agent id (`np.array_split(all_ids, cores)`,
dgen_model.py:326-328) and runs the per-(state, sector) battery allocation
and the per-state sums once, on the gathered frame (dgen_model.py:408-427 ->
attachment_rate_functions.py:58-148, :151-206).  Here a rank owns PIECES:
contiguous member ranges [lo, hi) of states (a state's members in their
caller order), cut so that every rank carries about the same measured device
cost; a state is cut only where no state boundary lies within `tol` of the
balanced cut.  What the reference gets from gathering, the loop gets from two
exchanges per model year (dgen_amd.year_loop):

* per-state totals and 8760-h rows are sums of per-CHUNK partials (fixed
  REDUCE_CHUNK-member chunks of each state, every partial over its members in
  a canonical order) added in chunk order (dgen_rows_seq_sum); cuts fall on
  chunk boundaries, so a split state's chunks are whole on their ranks and
  the state sums to the same bits on any number of ranks;
* a split (state, sector) group's largest-remainder allocation needs the
  whole group (numpy-order group sum, the winners' order): its members'
  new_adopters are gathered (an all-reduce of disjoint positions) and every
  rank holding a piece allocates the whole group, keeping its own members'
  results -- bit-identical to the one-pool allocation.

Per-agent cost model (`cost_per_agent`): measured per billing path on one
MI355X (scripts/calibrate_cost.py, profiles/r04/calibrate/), in ns of device
time per agent: a scan term per path and a per-evaluation term times the
Brent-depth bound E(L).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Tuple

import numpy as np

REDUCE_CHUNK = 8192

# Brent depth bound E as a function of L = load / naep (kW) with the optimum at
# the bracket's bound (scipy 1.15.3 probes)
E_BOUND_L = np.array([3.0, 5.0, 7.5, 10.0, 20.0, 50.0, 100.0, 200.0, 500.0, 1000.0, 4444.0])
E_BOUND_E = np.array([1.0, 2.0, 2.0, 3.0, 4.0, 6.0, 8.0, 9.0, 11.0, 13.0, 16.0])

# Device ns per agent by billing path (engine.path_class: 0 bins / NEM, 1 net
# billing from the scan-built split, 2 other hourly: TS sell rate or demand
# charges) and sector: (scan + battery-case finance, per Brent evaluation of
# the search).  Measured on MI355X by scripts/calibrate_cost.py: each class of
# a national population sized alone, 100k agents (profiles/r04/calibrate/
# cost.log).  The commercial net-billing class had 32k agents, whose fixed
# per-launch costs inflate its scan figure (128 ns): its scan is taken as the
# residential one's.
PATH_COST_NS = {
    # (path, is_res): (scan, per_eval)
    (0, True): (42.8, 4.5),
    (0, False): (42.2, 2.8),
    (1, True): (57.2, 43.3),
    (1, False): (57.2, 37.7),
    (2, True): (125.6, 60.0),
    (2, False): (142.6, 39.0),
}


def brent_depth(load_kwh, naep) -> np.ndarray:
    """E(L) interpolated in log L, L = load_kwh / naep."""
    L = np.asarray(load_kwh, np.float64) / np.maximum(np.asarray(naep, np.float64), 1e-9)
    return np.interp(np.log(np.maximum(L, 1e-12)), np.log(E_BOUND_L), E_BOUND_E)


def cost_per_agent(cols, naep, table=None) -> np.ndarray:
    """Predicted device ns per agent: scan[path, sector] + per_eval[path,
    sector] x E(L) (PATH_COST_NS unless `table` is given)."""
    from .engine import path_class
    tab = PATH_COST_NS if table is None else table
    pc = path_class(cols)
    res = (np.asarray(cols["flags"]) & 1) != 0
    E = brent_depth(cols["load_kwh"], naep)
    out = np.empty(pc.size, np.float64)
    for (p, r), (a, b) in tab.items():
        m = (pc == p) & (res == r)
        out[m] = a + b * E[m]
    return out


def census_sizes(n_global: int, weights=None) -> np.ndarray:
    """Agents per state: n_global shared out in proportion to `weights`
    (default the census households, synth.STATE_HOUSEHOLDS_M) by largest
    remainders, so the sizes add up to n_global exactly."""
    if weights is None:
        from .synth import STATE_HOUSEHOLDS_M as weights
    w = np.asarray(weights, np.float64)
    q = n_global * w / w.sum()
    base = np.floor(q).astype(np.int64)
    rem = int(n_global - base.sum())
    order = np.lexsort((np.arange(w.size), -(q - base)))
    base[order[:rem]] += 1
    return base


@dataclass
class ShardPlan:
    """Per rank, its pieces (state, lo, hi): member ranges of states, in state
    order.  Built identically on every rank (plan_partition)."""
    sizes: np.ndarray                          # agents per state
    pieces: List[List[Tuple[int, int, int]]]
    chunk: int = REDUCE_CHUNK
    rank_cost: List[float] = field(default_factory=list)

    @property
    def world(self) -> int:
        return len(self.pieces)

    def owners(self, s: int) -> List[int]:
        return [r for r, ps in enumerate(self.pieces) if any(p[0] == s for p in ps)]

    def split_states(self) -> List[int]:
        """States whose members sit on more than one rank (ascending)."""
        cnt: Dict[int, int] = {}
        for ps in self.pieces:
            for s, _, _ in ps:
                cnt[s] = cnt.get(s, 0) + 1
        return sorted(s for s, c in cnt.items() if c > 1)

    def n_chunks(self, s: int) -> int:
        return -(-int(self.sizes[s]) // self.chunk)

    def imbalance(self) -> float:
        c = np.asarray(self.rank_cost, np.float64)
        return float(c.max() / c.mean()) if c.size and c.mean() > 0 else 1.0


def plan_partition(sizes, cost_per_member, world: int, chunk: int = REDUCE_CHUNK,
                   tol: float = 0.02) -> ShardPlan:
    """Cut the states (in state order, members in caller order) into `world`
    contiguous runs of about equal cost.  cost_per_member[s]: the predicted
    cost of one agent of state s (its state's mean), or an array per member.
    Each cut lands on a state boundary when one is within tol x the per-rank
    cost of the balanced cut, else on the nearest chunk boundary inside the
    state it falls in (so every chunk stays whole on one rank)."""
    sizes = np.asarray(sizes, np.int64)
    S = sizes.size
    if world < 1:
        raise ValueError("bad world")
    # per-state cumulative cost at each chunk boundary
    bounds = []      # per state: member offsets of its chunk boundaries
    cum = []         # per state: cumulative cost (global) at those offsets
    run = 0.0
    for s in range(S):
        n = int(sizes[s])
        off = np.minimum(np.arange(0, n + chunk, chunk), n)
        off = np.unique(off)
        c = cost_per_member[s]
        if np.ndim(c) == 0:
            cc = run + float(c) * off
        else:
            pre = np.concatenate([[0.0], np.cumsum(np.asarray(c, np.float64))])
            cc = run + pre[off]
        bounds.append(off)
        cum.append(cc)
        run = float(cc[-1]) if n else run
    total = run
    T = total / world
    # cut positions as (state, member offset); (S, 0) = the end
    cuts = [(0, 0)]
    for k in range(1, world):
        x = k * T
        s = 0
        while s < S - 1 and (cum[s][-1] if sizes[s] else cum[s][0]) <= x:
            s += 1
        lo_c, hi_c = cum[s][0], cum[s][-1]
        if sizes[s] == 0 or x - lo_c <= tol * T or (hi_c - x <= tol * T):
            cut = (s, 0) if x - lo_c <= hi_c - x else (s + 1, 0)
        else:
            j = int(np.argmin(np.abs(cum[s] - x)))
            cut = (s, int(bounds[s][j]))
            if cut[1] == 0:
                cut = (s, 0)
            elif cut[1] >= sizes[s]:
                cut = (s + 1, 0)
        if cut < cuts[-1]:
            cut = cuts[-1]
        cuts.append(cut)
    cuts.append((S, 0))
    pieces: List[List[Tuple[int, int, int]]] = []
    cost: List[float] = []

    def at(c):
        s, m = c
        if s >= S:
            return total
        j = int(np.searchsorted(bounds[s], m))
        return float(cum[s][j])

    for r in range(world):
        (s0, m0), (s1, m1) = cuts[r], cuts[r + 1]
        ps = []
        s = s0
        while (s, 0) < (s1, m1) and s < S:
            lo = m0 if s == s0 else 0
            hi = m1 if s == s1 else int(sizes[s])
            if hi > lo:
                ps.append((s, lo, hi))
            s += 1
        pieces.append(ps)
        cost.append(at(cuts[r + 1]) - at(cuts[r]))
    return ShardPlan(sizes=sizes, pieces=pieces, chunk=chunk, rank_cost=cost)


def whole_plan(sizes, chunk: int = REDUCE_CHUNK) -> ShardPlan:
    """One rank holding every state (the one-pool reference of a plan)."""
    sizes = np.asarray(sizes, np.int64)
    return ShardPlan(sizes=sizes, pieces=[[(s, 0, int(n)) for s, n in enumerate(sizes) if n > 0]],
                     chunk=chunk, rank_cost=[1.0])


# ------------------------------------------------------------------ reductions
def chunk_keys(state, member, chunk: int = REDUCE_CHUNK) -> np.ndarray:
    """Chunk index of each agent within its state (member // chunk)."""
    return np.asarray(member, np.int64) // int(chunk)


@dataclass
class ChunkLayout:
    """This rank's chunk segments and how their partial rows combine into
    per-state rows through one all-reduce.

    seg_dev / seg_off: device rows of each local chunk (ascending device index
    within the chunk), chunk segments ordered by (state, chunk); chunk_state /
    chunk_index: each local chunk's state and index.  The exchange table has
    one row per state (rows of states held whole here are pre-combined
    locally) followed by one row per chunk of every split state (global)."""
    seg_dev: np.ndarray
    seg_off: np.ndarray
    chunk_state: np.ndarray
    chunk_index: np.ndarray
    n_states: int
    split_states: List[int]
    split_base: Dict[int, int]       # split state -> first exchange row of its chunks
    n_rows: int                      # exchange table rows
    local_whole: List[int]           # states held whole here (ascending)


def chunk_layout(state_dev, member_dev, n_states: int, plan: ShardPlan = None,
                 chunk: int = REDUCE_CHUNK) -> ChunkLayout:
    """Chunk segments of a rank's device rows (state_dev / member_dev: state and
    member index of each device row)."""
    st = np.asarray(state_dev, np.int64)
    ck = np.asarray(member_dev, np.int64) // int(chunk)
    n = st.size
    key = st * (1 << 32) + ck
    order = np.lexsort((np.arange(n), key))        # by (state, chunk), device index ascending
    k_sorted = key[order]
    starts = np.flatnonzero(np.r_[True, k_sorted[1:] != k_sorted[:-1]]) if n else np.zeros(0, np.int64)
    seg_off = np.concatenate([starts, [n]]).astype(np.int64)
    chunk_state = (k_sorted[starts] >> 32).astype(np.int64) if n else np.zeros(0, np.int64)
    chunk_index = (k_sorted[starts] & ((1 << 32) - 1)).astype(np.int64) if n else np.zeros(0, np.int64)
    split = plan.split_states() if plan is not None else []
    base, row = {}, n_states
    for s in split:
        base[s] = row
        row += plan.n_chunks(s)
    whole = sorted(set(chunk_state.tolist()) - set(split))
    return ChunkLayout(seg_dev=order.astype(np.int64), seg_off=seg_off, chunk_state=chunk_state,
                       chunk_index=chunk_index, n_states=n_states, split_states=split, split_base=base,
                       n_rows=row, local_whole=whole)


def rows_table(chunk_rows, L: ChunkLayout, seq_sum):
    """This rank's exchange table [n_rows, k] from its chunk partials
    [C_local, k] (in L's chunk order): states held whole are combined here
    (their chunks in order), split states' chunks go to their exchange rows;
    every other row is 0, so the ranks' SUM is a gather.  seq_sum(rows,
    seg_off): sequential row sums (Engine.rows_seq_sum, or host_seq_sum)."""
    import torch
    k = chunk_rows.shape[1]
    dev = chunk_rows.device
    table = torch.zeros((L.n_rows, k), dtype=torch.float64, device=dev)
    cs = L.chunk_state
    whole_mask = ~np.isin(cs, L.split_states)
    if whole_mask.any():
        # local chunks of whole states are contiguous per state (ordered by state, chunk)
        sel = np.flatnonzero(whole_mask)
        st = cs[sel]
        starts = np.flatnonzero(np.r_[True, st[1:] != st[:-1]])
        off = np.concatenate([starts, [sel.size]]).astype(np.int64)
        rows = chunk_rows.index_select(0, torch.as_tensor(sel, device=dev))
        comb = seq_sum(rows, off)
        table.index_copy_(0, torch.as_tensor(st[starts], device=dev), comb)
    if (~whole_mask).any():
        sel = np.flatnonzero(~whole_mask)
        dst = np.array([L.split_base[int(cs[i])] + int(L.chunk_index[i]) for i in sel], np.int64)
        table.index_copy_(0, torch.as_tensor(dst, device=dev),
                          chunk_rows.index_select(0, torch.as_tensor(sel, device=dev)))
    return table


def rows_finish(table, L: ChunkLayout, seq_sum):
    """Per-state rows [n_states, k] from the summed exchange table: every split
    state's chunk rows combined in chunk order."""
    import torch
    out = table[:L.n_states].clone()
    if L.split_states:
        base0 = L.n_states
        offs = np.array([L.split_base[s] - base0 for s in L.split_states] + [L.n_rows - base0], np.int64)
        comb = seq_sum(table[base0:].contiguous(), offs)
        out.index_copy_(0, torch.as_tensor(np.asarray(L.split_states, np.int64), device=out.device), comb)
    return out


def combine_rows(chunk_rows, L: ChunkLayout, seq_sum, allreduce):
    """rows_table -> allreduce (in-place SUM over the ranks) -> rows_finish."""
    return rows_finish(allreduce(rows_table(chunk_rows, L, seq_sum)), L, seq_sum)


def host_seq_sum(rows, seg_off):
    """CPU stand-in of Engine.rows_seq_sum (same additions in the same order)."""
    import torch
    out = torch.zeros((len(seg_off) - 1, rows.shape[1]), dtype=torch.float64)
    for s in range(len(seg_off) - 1):
        acc = torch.zeros(rows.shape[1], dtype=torch.float64)
        for r in range(int(seg_off[s]), int(seg_off[s + 1])):
            acc = acc + rows[r]
        out[s] = acc
    return out


# -------------------------------------------------------------- split groups
@dataclass
class SplitGroups:
    """The (state, sector) groups of split states, in a global order every
    rank agrees on: per group its global size, this rank's member offset and
    count (0 when it holds none), the global string ranks of its agent ids
    (the reference's tie-break, attachment_rate_functions.py:125-128) and its
    slice of the gather buffer."""
    keys: List[Tuple[int, int]]
    size: np.ndarray
    own_off: np.ndarray
    own_cnt: np.ndarray
    buf_off: np.ndarray                       # [G + 1] offsets into the gather buffer
    aid_rank: List[np.ndarray]                # per group: string ranks over the whole group

    @property
    def n_buf(self) -> int:
        return int(self.buf_off[-1])


def split_groups(plan: ShardPlan, rank: int, state_sectors: Dict[int, np.ndarray],
                 state_ids: Dict[int, np.ndarray]) -> SplitGroups:
    """state_sectors[s] / state_ids[s]: sector code and agent id of every
    member of split state s (caller order) -- a rank holding a piece of s
    knows them all (the state's agents are generated whole, then sliced)."""
    from .attachment import string_ranks
    keys, size, own_off, own_cnt, ranks = [], [], [], [], []
    mine = {s: (lo, hi) for s, lo, hi in plan.pieces[rank]}
    for s in plan.split_states():
        sec = state_sectors.get(s)
        if sec is None:
            raise ValueError(f"split state {s}: member sectors needed on every rank")
        ids = state_ids[s]
        for c in (0, 1):
            m = np.flatnonzero(np.asarray(sec) == c)
            if m.size == 0:
                continue
            keys.append((s, c))
            size.append(m.size)
            lo, hi = mine.get(s, (0, 0))
            own_off.append(int(np.searchsorted(m, lo)))
            own_cnt.append(int(np.searchsorted(m, hi) - np.searchsorted(m, lo)))
            ranks.append(string_ranks(np.asarray(ids)[m]))
    size = np.asarray(size, np.int64)
    return SplitGroups(keys=keys, size=size, own_off=np.asarray(own_off, np.int64),
                       own_cnt=np.asarray(own_cnt, np.int64),
                       buf_off=np.concatenate([[0], np.cumsum(size)]).astype(np.int64), aid_rank=ranks)
