"""Device choice of the drop-in under the reference's own caller: dgen_model.py
spawns LOCAL_CORES pool workers per model year (dgen_model.py:309-317) and
apply_asyncs size_chunk on each np.array_split chunk (:326-375).  Each worker's
Engine must open a different GPU of the node, with dgen_model.py unchanged
(financial_functions.worker_device)."""
import multiprocessing as mp

import pytest

from tests import pool_workers


def _devices(n_workers, n_devices, env=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pool = ctx.Pool(processes=n_workers, initializer=pool_workers.stub_init,
                    initargs=(q, n_devices, dict(env or {})))
    try:
        got = [q.get(timeout=120) for _ in range(n_workers)]
        assert pool.map(pool_workers.noop, range(4)) == list(range(4))
    finally:
        pool.close()
        pool.join()
    assert len({pid for pid, _ in got}) == n_workers
    return sorted(d for _, d in got)


def test_spawn_pool_workers_take_distinct_devices():
    assert _devices(4, 4) == [0, 1, 2, 3]


def test_spawn_pool_larger_than_node_spreads_evenly():
    # 16 workers (the reference's LOCAL_CORES default on a node) over 8 GPUs: 2 each
    d = _devices(16, 8)
    assert [d.count(k) for k in range(8)] == [2] * 8


def test_dgen_devices_list_restricts_rotation():
    assert _devices(4, 8, {"DGEN_DEVICES": "2,5"}) == [2, 2, 5, 5]


def test_local_rank_wins_and_main_process_is_device_0(monkeypatch):
    from dgen_amd import financial_functions as ff
    monkeypatch.delenv("DGEN_DEVICES", raising=False)
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert ff.worker_device() == 3
    monkeypatch.delenv("LOCAL_RANK")
    assert ff.worker_device() == 0            # the main process (cores=None path)
    monkeypatch.setenv("DGEN_DEVICES", "6,7")
    assert ff.worker_device() == 6
    monkeypatch.setenv("DGEN_DEVICES", " , ")
    with pytest.raises(ValueError):
        ff.worker_device()


def test_sub_batch_byte_model():
    """The per-agent HBM figure of the device budget covers the fp64 planes and
    the workspace, and DGEN_MAX_ROWS overrides the budget."""
    import os

    from dgen_amd import _lib
    from dgen_amd import financial_functions as ff

    class E:
        lib = _lib.load()
    per = ff.agent_device_bytes(E)
    assert per >= 3 * 8760 * 8 + int(E.lib.dgen_workspace_bytes(4096, 4096)) // 4096
    assert per < 3 * 8760 * 8 + 200_000
    old = os.environ.get("DGEN_MAX_ROWS")
    os.environ["DGEN_MAX_ROWS"] = "50000"
    try:
        assert ff.device_rows_budget(E) == 50000
    finally:
        if old is None:
            del os.environ["DGEN_MAX_ROWS"]
        else:
            os.environ["DGEN_MAX_ROWS"] = old
