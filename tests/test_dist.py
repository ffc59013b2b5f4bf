"""Multi-rank logic on CPU (gloo, world size 2): np.array_split sharding,
group ordering and the per-(state, sector) totals all-reduce."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dgen_amd.dist import allreduce_sum, group_order, shard_bounds


def test_shard_bounds_match_array_split():
    for n in (0, 1, 7, 10, 1001):
        for world in (1, 2, 3, 8):
            chunks = np.array_split(np.arange(n), world)
            for r in range(world):
                lo, hi = shard_bounds(n, world, r)
                assert list(range(lo, hi)) == chunks[r].tolist()


def test_group_order_contiguous():
    keys = [("DE", "res"), ("CA", "com"), ("DE", "res"), ("CA", "res"), ("CA", "com")]
    perm, off, uniq = group_order(keys)
    assert uniq == [("DE", "res"), ("CA", "com"), ("CA", "res")]
    assert off.tolist() == [0, 2, 4, 5]
    ordered = [keys[i] for i in perm]
    for s, k in enumerate(uniq):
        assert all(x == k for x in ordered[off[s]:off[s + 1]])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(5)
    states = rng.choice(["DE", "CA", "NY"], n)
    sectors = rng.choice(["res", "com"], n)
    kw = rng.uniform(1, 20, n)
    all_keys = sorted(set(zip(states, sectors)))
    lo, hi = shard_bounds(n, world, rank)
    keys = list(zip(states[lo:hi], sectors[lo:hi]))
    perm, off, uniq = group_order(keys)
    local = torch.zeros((len(all_keys), 2), dtype=torch.float64)
    pos = {k: i for i, k in enumerate(all_keys)}
    v = kw[lo:hi][perm]
    for s, k in enumerate(uniq):
        local[pos[k], 0] = float(v[off[s]:off[s + 1]].sum())
        local[pos[k], 1] = float(off[s + 1] - off[s])
    allreduce_sum(local)
    if rank == 0:
        q.put(local.numpy().tolist())
    dist.barrier()
    dist.destroy_process_group()


def test_totals_allreduce_gloo_world2():
    n = 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = np.array(q.get(timeout=120))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    rng = np.random.default_rng(5)
    states = rng.choice(["DE", "CA", "NY"], n)
    sectors = rng.choice(["res", "com"], n)
    kw = rng.uniform(1, 20, n)
    all_keys = sorted(set(zip(states, sectors)))
    for i, k in enumerate(all_keys):
        m = (states == k[0]) & (sectors == k[1])
        assert np.isclose(got[i][0], kw[m].sum(), rtol=1e-12)
        assert got[i][1] == m.sum()


def test_allreduce_identity_without_pg():
    t = torch.ones(3)
    assert allreduce_sum(t) is t


# ---------------------------------------------------------------------------
# model-year loop sharding (dgen_amd.year_loop): whole states per rank, one
# all-reduce of the per-state rows per year
# ---------------------------------------------------------------------------
def test_rank_states_partition():
    from dgen_amd.synth import STATES
    from dgen_amd.year_loop import rank_states
    for world in (1, 2, 3, 8):
        got = np.concatenate([rank_states(r, world) for r in range(world)])
        assert sorted(got.tolist()) == list(range(len(STATES)))
    with pytest.raises(ValueError):
        rank_states(2, 2)


def test_state_pool_population():
    from dgen_amd.synth import STATES, make_population
    from dgen_amd.year_loop import loop_agents, rank_states
    pool = rank_states(1, 8)
    pop = make_population("national_mixed", 500, seed=7, n_res_shapes=8, n_com_shapes=4, n_cf=4,
                          n_counties=4, n_tariffs=8, state_pool=pool)
    assert set(np.unique(pop.state_ix)) <= set(pool.tolist())
    is_ca = (pop.cols["flags"] >> 1) & 1
    assert np.array_equal(is_ca.astype(bool), pop.state_ix == STATES.index("CA"))
    ag = loop_agents(pop, agent_id0=500)
    assert ag["agent_id"][0] == 500 and len(np.unique(ag["agent_id"])) == 500
    assert (ag["customers_in_bin"] > 0).all()
    assert np.array_equal(ag["county"], pop.county_ix)
    # the default (all states) stream is unchanged by the pool option
    a = make_population("national_mixed", 300, seed=9, n_res_shapes=8, n_com_shapes=4, n_cf=4,
                        n_counties=4, n_tariffs=8)
    b = make_population("national_mixed", 300, seed=9, n_res_shapes=8, n_com_shapes=4, n_cf=4,
                        n_counties=4, n_tariffs=8, state_pool=np.arange(len(STATES)))
    assert all(np.array_equal(a.cols[k], b.cols[k]) for k in a.cols)


def _loop_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dgen_amd.year_loop import merge_state_rows, rank_states
    mine = rank_states(rank, world)
    rows = torch.stack([torch.tensor([float(s), 10.0 * s + rank, 1.0], dtype=torch.float64)
                        for s in mine])
    full = merge_state_rows(rows, mine.tolist(), 51)
    q.put((rank, full.numpy().tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_merge_state_rows_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_loop_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    a, b = np.array(res[0]), np.array(res[1])
    assert np.array_equal(a, b)                       # every rank holds the full table
    for s in range(51):
        assert a[s].tolist() == [float(s), 10.0 * s + (s % 2), 1.0]


def test_merge_state_rows_single_process():
    from dgen_amd.year_loop import merge_state_rows
    t = merge_state_rows(torch.ones((2, 3), dtype=torch.float64), [4, 7], 10)
    assert t.shape == (10, 3) and t[4].tolist() == [1.0] * 3 and t.sum().item() == 6.0


def _timed_worker(rank, world, port, q):
    """bench.timed_region under gloo: rank r's steps sleep (r + 1) x 40 ms; every
    rank must report the slowest rank's time (the contract's max over ranks)."""
    import sys
    import time
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []
    el = bench.timed_region(lambda: (calls.append(1), time.sleep(0.04 * (rank + 1))), 3,
                            lambda: None, dist, torch.device("cpu"))
    q.put((rank, el, len(calls)))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_timed_region_max_over_ranks_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timed_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    (r0, el0, c0), (r1, el1, c1) = res
    assert c0 == c1 == 3                      # exactly `steps` timed calls per rank
    assert el0 == el1                         # every rank reports the same (max) time
    assert el0 >= 3 * 0.08 * 0.95             # ... the slower rank's (3 x 80 ms)


# ---------------------------------------------------------------------------
# work-balanced state partition (whole states, balanced by the
# predicted Brent depth E(L) per agent)
# ---------------------------------------------------------------------------
def _census_state_work(n=30_000, seed=11):
    from dgen_amd.synth import STATES, make_population
    from dgen_amd.year_loop import population_work
    pop = make_population("national_mixed", n, seed=seed, n_res_shapes=64, n_com_shapes=32, n_cf=64,
                          n_counties=16, n_tariffs=16, state_mix="census")
    w = population_work(pop)
    return np.bincount(pop.state_ix.astype(np.int64), weights=w, minlength=len(STATES)), pop, w


def test_predicted_work_follows_the_brent_depth_table():
    from dgen_amd.year_loop import E_BOUND_E, E_BOUND_L, EVAL_COST, predicted_work
    assert np.allclose(predicted_work(E_BOUND_L * 1000.0, np.full(E_BOUND_L.size, 1000.0)),
                       1.0 + EVAL_COST * E_BOUND_E)
    w = predicted_work([1e3, 1e4, 1e6, 1e9], [1500.0] * 4)
    assert np.all(np.diff(w) >= 0) and w[0] == 1.0 + EVAL_COST and w[-1] == 1.0 + EVAL_COST * 16


def test_balanced_partition_of_census_states():
    """LPT over whole states by predicted work: every state on one rank, and
    max/mean rank load <= 1.1 for 2-8 ranks on census-sized states (CA and TX
    are ~18 % of the households), where s % world leaves ranks idle."""
    from dgen_amd.synth import STATES
    from dgen_amd.year_loop import balanced_states, rank_states
    sw, _, _ = _census_state_work()
    for world in (1, 2, 3, 4, 8):
        parts = balanced_states(sw, world)
        assert sorted(np.concatenate(parts).tolist()) == list(range(len(STATES)))
        for r in range(world):
            assert np.array_equal(rank_states(r, world, state_work=sw), parts[r])
        load = np.array([sw[p].sum() for p in parts])
        assert load.max() / load.mean() <= 1.1, (world, load)
    rr = np.array([sw[rank_states(r, 8)].sum() for r in range(8)])
    assert rr.max() / rr.mean() > 1.3            # the round-robin split is what this replaces
    with pytest.raises(ValueError):
        rank_states(0, 2, state_work=sw[:10])


def _balance_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dgen_amd.year_loop import rank_states
    sw, pop, w = _census_state_work()          # every rank derives the same weights
    mine = rank_states(rank, world, state_work=sw)
    mask = np.isin(pop.state_ix.astype(np.int64), mine)
    t = torch.zeros(world, dtype=torch.float64)
    t[rank] = float(w[mask].sum())
    n = torch.tensor([float(mask.sum())], dtype=torch.float64)
    allreduce_sum(t)
    allreduce_sum(n)
    q.put((rank, t.numpy().tolist(), float(n.item()), mine.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_balanced_partition_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_balance_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (t, n, m)) for r, t, n, m in (q.get(timeout=180) for _ in procs))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    (t0, n0, m0), (t1, n1, m1) = res[0], res[1]
    assert t0 == t1 and n0 == n1 == 30_000          # all agents on exactly one rank
    assert not set(m0) & set(m1)
    load = np.array(t0)
    assert load.max() / load.mean() <= 1.1, load
