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
