"""Spawn-pool helpers for tests/test_pool_devices.py (importable by a spawned
worker: module-level functions only, nothing that touches a GPU)."""
import os

_q = None


def stub_init(q, n_devices, env):
    """Pool initializer: a stubbed device count (the CPU container has no GPU),
    then report which device financial_functions.get_engine would open."""
    global _q
    _q = q
    import torch
    torch.cuda.device_count = lambda: n_devices
    for k, v in env.items():
        os.environ[k] = v
    from dgen_amd import financial_functions as ff
    q.put((os.getpid(), ff.worker_device()))


def noop(x):
    return x


def gpu_init(store):
    """Pool initializer of the GPU rehearsal: the worker's profile source (the
    reference's _init_worker opens a DB connection here, ff:1129-1134)."""
    from dgen_amd import financial_functions as ff
    ff._worker_conn = store


def engine_device(_):
    from dgen_amd import financial_functions as ff
    return os.getpid(), ff.get_engine().device


LOOP_YEARS = (2026, 2027)
LOOP_KEYS = ("market_share", "number_of_adopters", "system_kw_cum", "added", "batt_kw_cum", "batt_kwh_cum")


def loop_setup(plan_world, rank, chunk=64):
    """Tables, plan (cuts inside states: tol 0) and this rank's shard of the
    small national population of the split-state loop tests."""
    import numpy as np
    from dgen_amd import partition as P
    from dgen_amd.synth import STATES, national_tables, shard_population, split_state_members
    T = national_tables(n_res_shapes=64, n_com_shapes=32, n_cf=32, n_counties=16, n_tariffs=48)
    sizes = P.census_sizes(3000)
    cost = np.ones(sizes.size)
    cost[STATES.index("CA")] = 40.0
    if plan_world == 1:
        plan = P.whole_plan(sizes, chunk=chunk)
        sg = None
    else:
        plan = P.plan_partition(sizes, cost, plan_world, chunk=chunk, tol=0.0)
    pop, ag = shard_population(T, plan, rank)
    if plan_world > 1:
        secs, ids = split_state_members("national_mixed", plan)
        sg = P.split_groups(plan, rank, secs, ids)
    return T, plan, pop, ag, sg


def loop_run(engine, plan_world, rank, exchange=None):
    """Run LOOP_YEARS of this rank's YearLoop; per year (totals, hourly, {key:
    per-agent values by agent id})."""
    import numpy as np
    from dgen_amd.year_loop import LoopTables, YearLoop
    T, plan, pop, ag, sg = loop_setup(plan_world, rank)
    engine.load_profiles(T.shapes, T.cfs, T.wholesale)
    engine.set_tariffs(T.tt.array())
    engine.set_switches(T.switches)
    lp = YearLoop(engine, pop, ag, LoopTables.synthetic(), first_year=LOOP_YEARS[0], hourly_export=True,
                  plan=plan, split=sg)
    ids = np.asarray(ag["agent_id"])[lp.perm]
    out = []
    for y in LOOP_YEARS:
        r = lp.run_year(y, keep_per_agent=True, exchange=exchange)
        out.append((r.totals.cpu().numpy(), r.hourly.cpu().numpy(),
                    {k: dict(zip(ids.tolist(), r.per_agent[k].cpu().numpy().tolist())) for k in LOOP_KEYS}))
    return plan.split_states(), out


def loop_rank(rank, world, port, q):
    """One rank of the 2-process split-state loop rehearsal: gloo process group
    (its all-reduce takes the GPU tensors the loop exchanges), one GPU."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from dgen_amd.engine import Engine
        eng = Engine(0)
        split, out = loop_run(eng, world, rank)
        q.put((rank, split, out))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:                     # report, never hang the parent
        q.put((rank, "error", repr(e)))
        raise
