"""Rank partition with split states (dgen_amd.partition): the
plan, the chunked per-state reductions and the split groups' gathered
allocation, world size 1 vs 2 (gloo) on CPU.  The device pieces (chunk
partials, k_batt_attach) are stood in by host restatements here (the oracle's
largest-remainder allocation, sequential chunk sums); the GPU path is
tests/test_gpu_year_loop.py::test_split_state_shards_reproduce_one_pool."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dgen_amd import partition as P
from dgen_amd.synth import STATES, state_id_base, state_member_sectors


def test_census_sizes_add_up():
    for n in (0, 1, 51, 1000, 2_500_000):
        s = P.census_sizes(n)
        assert s.sum() == n and s.size == len(STATES) and (s >= 0).all()
    s = P.census_sizes(20_000_000)
    assert s[STATES.index("CA")] > s[STATES.index("WY")] * 40


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("tol", [0.0, 0.02])
def test_plan_covers_every_member_once(world, tol):
    sizes = P.census_sizes(300_000)
    cost = np.random.default_rng(1).uniform(1.0, 4.0, sizes.size)
    plan = P.plan_partition(sizes, cost, world, chunk=1024, tol=tol)
    assert plan.world == world
    seen = [np.zeros(n, np.int64) for n in sizes]
    last = (-1, -1)
    for ps in plan.pieces:
        for s, lo, hi in ps:
            assert 0 <= lo < hi <= sizes[s]
            assert (s, lo) > last                      # state order, contiguous runs
            last = (s, lo)
            assert lo % 1024 == 0 and (hi % 1024 == 0 or hi == sizes[s])   # chunk boundaries
            seen[s][lo:hi] += 1
    assert all((v == 1).all() for v in seen)
    # balance: within one chunk's cost of the mean (tol 0), or tol + a chunk
    chunk_cost = 1024 * cost.max()
    mean = sum(plan.rank_cost) / world
    assert max(plan.rank_cost) - mean <= chunk_cost + tol * mean + 1e-6
    if world == 1:
        assert plan.split_states() == []


def test_plan_splits_only_where_needed():
    sizes = P.census_sizes(400_000)
    ca = STATES.index("CA")
    plan = P.plan_partition(sizes, np.ones(sizes.size), 8, chunk=1024, tol=0.02)
    assert plan.imbalance() <= 1.03
    for s in plan.split_states():
        assert len(plan.owners(s)) >= 2
    # a state boundary within tol of a balanced cut is taken instead of a split
    exact = P.plan_partition(sizes, np.ones(sizes.size), 8, chunk=1024, tol=0.0)
    assert len(plan.split_states()) <= len(exact.split_states())
    assert exact.imbalance() <= plan.imbalance() + 1e-12
    # CA alone (10.4 % of the census) is more than a rank's share at 16 ranks: split
    p16 = P.plan_partition(sizes, np.ones(sizes.size), 16, chunk=1024, tol=0.02)
    assert ca in p16.split_states() and p16.imbalance() <= 1.05
    whole = P.whole_plan(sizes)
    assert whole.split_states() == [] and whole.world == 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SIZES_N = 6000
CHUNK = 64


def _rank_data(plan, rank):
    """This rank's agents of the synthetic national set: (state, member, id,
    sector, new_adopters, batt_kw, hourly rows [m, 16])."""
    base = state_id_base(plan.sizes)
    st, mem = [], []
    for s, lo, hi in plan.pieces[rank]:
        st.append(np.full(hi - lo, s, np.int64))
        mem.append(np.arange(lo, hi, dtype=np.int64))
    st = np.concatenate(st) if st else np.zeros(0, np.int64)
    mem = np.concatenate(mem) if mem else np.zeros(0, np.int64)
    aid = base[st] + mem
    sec = np.array([state_member_sectors("national_mixed", s, int(plan.sizes[s]))[m] for s, m in zip(st, mem)],
                   np.int64)
    rng = lambda i: np.random.default_rng(1000 + int(i))
    na = np.array([rng(i).uniform(0.0, 3.0) for i in aid])
    bkw = np.array([rng(i + 7).uniform(1.0, 9.0) for i in aid])
    rows = np.stack([rng(i + 13).normal(0.0, 1.0, 16) for i in aid]) if aid.size else np.zeros((0, 16))
    return st, mem, aid, sec, na, bkw, rows


def _chunk_rows(plan, rank, st, mem, rows):
    """Chunk partials in the layout's order (members summed in member order)."""
    L = P.chunk_layout(st, mem, len(STATES), plan, chunk=CHUNK)
    parts = []
    for j in range(len(L.seg_off) - 1):
        idx = L.seg_dev[L.seg_off[j]:L.seg_off[j + 1]]
        acc = torch.zeros(rows.shape[1], dtype=torch.float64)
        for i in idx[np.argsort(mem[idx])]:
            acc = acc + torch.as_tensor(rows[i])
        parts.append(acc)
    return L, (torch.stack(parts) if parts else torch.zeros((0, rows.shape[1]), dtype=torch.float64))


def _allocate_split(plan, rank, st, sec, aid, na, bkw, rate, allreduce):
    """Own members' battery adopters: groups held whole here allocated on
    their own, split groups gathered and allocated whole (oracle restatement)."""
    from dgen_amd.synth import split_state_members
    from oracle import attach as oa
    secs, ids = split_state_members("national_mixed", plan)
    SG = P.split_groups(plan, rank, secs, ids)
    buf = torch.zeros(SG.n_buf, dtype=torch.float64)
    for j, (s, c) in enumerate(SG.keys):
        own = np.flatnonzero((st == s) & (sec == c))
        assert own.size == SG.own_cnt[j]
        b0 = SG.buf_off[j] + SG.own_off[j]
        buf[b0:b0 + own.size] = torch.as_tensor(na[own])
    buf = allreduce(buf).numpy()
    added = np.zeros(st.size, np.int64)
    split = set(plan.split_states())
    loc = np.flatnonzero(~np.isin(st, list(split)))
    if loc.size:
        r = oa.allocate([STATES[s] for s in st[loc]], sec[loc].tolist(), aid[loc], na[loc], rate[st[loc]],
                        bkw[loc], bkw[loc], np.zeros(loc.size), np.zeros(loc.size))
        added[loc] = r["batt_adopters_added_this_year"]
    for j, (s, c) in enumerate(SG.keys):
        if SG.own_cnt[j] == 0:
            continue
        G = int(SG.size[j])
        gid = ids[s][secs[s] == c]
        r = oa.allocate([STATES[s]] * G, [c] * G, gid, buf[SG.buf_off[j]:SG.buf_off[j] + G], np.full(G, rate[s]),
                        np.ones(G), np.ones(G), np.zeros(G), np.zeros(G))
        own = np.flatnonzero((st == s) & (sec == c))
        added[own] = r["batt_adopters_added_this_year"][SG.own_off[j]:SG.own_off[j] + own.size]
    return added


def _one_pool(sizes):
    whole = P.whole_plan(sizes, chunk=CHUNK)
    st, mem, aid, sec, na, bkw, rows = _rank_data(whole, 0)
    L, cr = _chunk_rows(whole, 0, st, mem, rows)
    ident = lambda t: t
    state_rows = P.combine_rows(cr, L, P.host_seq_sum, ident)
    rate = np.random.default_rng(9).uniform(0.05, 0.35, len(STATES))
    added = _allocate_split(whole, 0, st, sec, aid, na, bkw, rate, ident)
    return dict(zip(aid.tolist(), added.tolist())), state_rows


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sizes = P.census_sizes(SIZES_N)
    cost = np.ones(sizes.size)
    cost[STATES.index("CA")] = 50.0          # the balanced cut falls inside CA
    plan = P.plan_partition(sizes, cost, world, chunk=CHUNK, tol=0.0)
    st, mem, aid, sec, na, bkw, rows = _rank_data(plan, rank)

    def ar(t):
        dist.all_reduce(t)
        return t
    L, cr = _chunk_rows(plan, rank, st, mem, rows)
    state_rows = P.combine_rows(cr, L, P.host_seq_sum, ar)
    rate = np.random.default_rng(9).uniform(0.05, 0.35, len(STATES))
    added = _allocate_split(plan, rank, st, sec, aid, na, bkw, rate, ar)
    q.put((rank, plan.split_states(), dict(zip(aid.tolist(), added.tolist())), state_rows.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_split_states_gloo_world2_match_one_pool():
    """World 2 with cuts inside states (tol 0): per-state rows and every
    agent's battery adopters bit-identical to the one-pool computation."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref_added, ref_rows = _one_pool(P.census_sizes(SIZES_N))
    split = got[0][1]
    assert split, "the world-2 plan must cut a state"
    merged = {}
    for rank, sp, added, rows in got:
        assert sp == split
        assert np.array_equal(rows, ref_rows.numpy()), rank       # every rank holds all state rows
        merged.update(added)
    assert merged == ref_added
    assert sum(ref_added.values()) > 0


def test_year_loop_rejects_plan_split_misuse():
    """YearLoop needs plan and split groups together when the plan cuts a
    state, and the members' within-state numbering from the plan:
    each misuse raises before anything touches the device."""
    import types

    import pytest

    from dgen_amd.year_loop import YearLoop
    sizes = P.census_sizes(SIZES_N)
    cost = np.ones(sizes.size)
    cost[STATES.index("CA")] = 50.0
    plan = P.plan_partition(sizes, cost, 2, chunk=CHUNK, tol=0.0)
    assert plan.split_states()
    pop = types.SimpleNamespace(cols={"load_kwh": np.zeros(4)})
    ag = {"state": np.zeros(4, np.int64), "member": np.arange(4)}
    sg = object()
    with pytest.raises(ValueError, match="no split groups"):
        YearLoop(None, pop, ag, None, plan=plan, split=None)
    with pytest.raises(ValueError, match="without the plan"):
        YearLoop(None, pop, ag, None, plan=None, split=sg)
    with pytest.raises(ValueError, match="member"):
        YearLoop(None, pop, {"state": ag["state"]}, None, plan=plan, split=sg)
