"""The model-year loop's real exchange path with a state cut across ranks:
two processes, a gloo process group whose all-reduce carries the loop's GPU
tensors (dgen_amd.dist.allreduce_sum -- the call RCCL answers on a node), a
plan with tol 0 so the cut falls inside a state.  The split-group gather, the
initial-market gather and the chunk-row exchange then all run through
dist.all_reduce; every per-state total and 8760-h row, and every agent's
diffusion and battery allocation, must equal the one-pool loop bit for bit
(test_gpu_year_loop.py covers the same through run_lockstep)."""
import multiprocessing as mp
import socket

import numpy as np
import pytest

from tests import pool_workers

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_split_state_loop_two_ranks_gloo_match_one_pool():
    from dgen_amd.engine import Engine
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=pool_workers.loop_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got = [q.get(timeout=240) for _ in range(2)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for g in got:
        assert g[1] != "error", g
    assert all(p.exitcode == 0 for p in procs)
    _, one = pool_workers.loop_run(Engine(0), 1, 0)
    split = got[0][1]
    assert split and got[1][1] == split, "the plan must cut a state across the two ranks"
    for yi, (tot, hourly, per) in enumerate(one):
        merged = {k: {} for k in pool_workers.LOOP_KEYS}
        for rank, _, out in got:
            t, h, pa = out[yi]
            assert np.array_equal(t, tot), (rank, yi, "totals")
            assert np.array_equal(h, hourly), (rank, yi, "hourly")
            for k in pool_workers.LOOP_KEYS:
                merged[k].update(pa[k])
        for k in pool_workers.LOOP_KEYS:
            assert merged[k] == per[k], (yi, k)
    assert sum(one[-1][2]["added"].values()) > 0
