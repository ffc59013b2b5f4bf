"""Device finance-series export (k_finance_series) through the drop-in
function against the reference's own records (tests/golden/finance_series.json),
and straight from the sizing outputs against the oracle restatement.
Bit-exact: the kernel copies values (non-finite -> 0)."""
import numpy as np
import pandas as pd
import pytest
import torch

from dgen_amd import finance_series as gfs
from oracle import finance_series as ofs
from tests.helpers import golden_finance

pytestmark = pytest.mark.gpu


def _frame(rows, index_agent_id):
    df = pd.DataFrame({k: [r[k] for r in rows] for k in rows[0]})
    return df.set_index("agent_id") if index_agent_id else df


@pytest.mark.parametrize("case", ["columns", "index_agent_id"])
def test_export_device_matches_reference(engine, case):
    meta = golden_finance()
    c = next(c for c in meta["cases"] if c["name"] == case)
    seen = []
    got = gfs.export_agent_finance_series("eng", "s", "o", meta["year"],
                                          _frame(c["rows"], c["index_agent_id"]),
                                          writer=lambda r, *a, **k: seen.append((a, k)),
                                          dev_engine=engine)
    ref = c["records"]
    assert len(got) == len(ref)
    assert seen and seen[0][0][3] == c["table"] and seen[0][1]["if_exists"] == c["if_exists"]
    for (_, a), b in zip(got.iterrows(), ref):
        assert (a["agent_id"], a["year"], a["scenario_case"]) == (b["agent_id"], b["year"], b["scenario_case"])
        for k in ("cf_energy_value", "utility_bill_w_sys", "utility_bill_wo_sys"):
            assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k


def test_export_nothing_to_write(engine):
    df = pd.DataFrame({"agent_id": [1, 2], "x": [0.0, 1.0]})
    assert gfs.export_agent_finance_series(None, "s", "o", 2027, df, dev_engine=engine) is None


def test_series_from_sizing_outputs(engine):
    from tests import helpers
    from dgen_amd.engine import outputs_to_host, profile_order
    b, cols, shapes, cfs, ws = helpers.golden_population()
    engine.load_profiles(shapes, cfs, ws)
    engine.set_tariffs(b.tariffs.array())
    engine.set_switches(b.switches.array())
    batch = engine.upload_agents(cols, order=profile_order(cols))
    out = engine.alloc_outputs(batch.n, hourly=False)
    engine.size(batch, out)
    torch.cuda.synchronize()
    h = outputs_to_host(out, batch.perm)
    life = np.asarray(cols["econ_life"])
    got = gfs.series_from_outputs(engine, out, life, batch.perm)
    for ci, (case, names) in enumerate(ofs.CASES):
        for si, key in enumerate(("cfev_pv", "bill_w_pv", "bill_wo_pv")[:3] if ci == 0 else
                                 ("cfev_batt", "bill_w_batt", "bill_wo_batt")):
            g = got[f"{gfs.SERIES[si]}_{case}"]
            for i in range(batch.n):
                ref = ofs.norm25(list(h[key][i, :life[i] + 1]))   # the agent's 26-long list
                assert np.array_equal(g[i], np.asarray(ref)), (case, key, i)


def test_export_stages_series_columns_whole(engine):
    """The drop-in's yearly columns (hourly_column.RowColumn: cells are lists of
    N + 1 values) are staged whole; the records equal those of the same frame
    with plain list cells (the reference's form)."""
    from dgen_amd.hourly_column import yearly_column
    rng = np.random.default_rng(5)
    n = 300
    lens = rng.integers(10, 52, n)
    cols = {}
    for _, names in gfs.CASES:
        for c in names:
            a = rng.normal(size=(n, 51)) * 100
            a[rng.random((n, 51)) < 0.02] = np.inf
            cols[c] = a
    aid = rng.permutation(10_000)[:n]
    fast = pd.DataFrame({"agent_id": aid, **{c: yearly_column(a, lens) for c, a in cols.items()}})
    slow = pd.DataFrame({"agent_id": aid, **{c: [list(a[i, :lens[i]]) for i in range(n)]
                                             for c, a in cols.items()}})
    got = gfs.export_agent_finance_series(None, "s", "o", 2030, fast, dev_engine=engine)
    ref = gfs.export_agent_finance_series(None, "s", "o", 2030, slow, dev_engine=engine)
    assert len(got) == 2 * n == len(ref)
    assert got[["agent_id", "year", "scenario_case"]].equals(ref[["agent_id", "year", "scenario_case"]])
    for k in gfs.SERIES:
        assert all(np.array_equal(np.asarray(a), np.asarray(b)) for a, b in zip(got[k], ref[k])), k
