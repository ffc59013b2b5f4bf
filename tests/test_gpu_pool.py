"""The reference's production call shape on the GPU: a spawn pool of workers,
each apply_async'ing size_chunk on an np.array_split chunk of the agent frame
(dgen_model.py:309-384), results concatenated -- the same frame as one
size_chunk over the whole population, and each worker on the device
financial_functions.worker_device() gives it (one GPU here: all on 0; the
rotation over a node's GPUs is tests/test_pool_devices.py)."""
import multiprocessing as mp

import numpy as np
import pandas as pd
import pytest

from dgen_amd import financial_functions as ff
from tests import pool_workers

pytestmark = pytest.mark.gpu


def test_spawn_pool_chunks_equal_one_call():
    from dgen_amd.synth import reference_frame
    df, store, table = reference_frame(6000)
    ff._worker_conn = store
    one, agg = ff.size_chunk(df, None, table, "simple")
    ctx = mp.get_context("spawn")
    cores = 2
    pool = ctx.Pool(processes=cores, initializer=pool_workers.gpu_init, initargs=(store,))
    try:
        chunks = np.array_split(df.index.tolist(), cores)
        res = [pool.apply_async(ff.size_chunk, args=(df.loc[c], None, table, "simple")) for c in chunks]
        devs = pool.map(pool_workers.engine_device, range(cores))
        got = [r.get(timeout=300) for r in res]
    finally:
        pool.close()
        pool.join()
    import torch
    ndev = torch.cuda.device_count()
    assert {d for _, d in devs} <= set(range(ndev))
    frame = pd.concat([g[0] for g in got], axis=0)
    assert list(frame.index) == list(one.index)
    for k in ("system_kw", "npv", "payback_period", "batt_kw", "batt_kwh", "naep"):
        assert np.array_equal(frame[k].to_numpy(float), one[k].to_numpy(float)), k
    for k in ("cash_flow", "utility_bill_w_sys_pv_batt"):
        assert [list(x) for x in frame[k]] == [list(x) for x in one[k]], k
    for k in ("baseline_net_hourly", "adopter_net_hourly_with_batt"):
        assert np.array_equal(np.stack([np.asarray(x) for x in frame[k]]),
                              np.stack([np.asarray(x) for x in one[k]])), k
    # size_chunk's hourly aggregate: the chunks' sums add to the whole frame's
    tot = np.sum([np.asarray(g[1]["net_sum_kw"]) for g in got], axis=0)
    assert np.allclose(tot, np.asarray(agg["net_sum_kw"]), rtol=1e-12, atol=0.0)
