"""Oracle restatement of the finance-series export (oracle/finance_series.py)
against the reference's own records (tests/golden/finance_series.json):
bit-exact (values are copies, non-finite -> 0)."""
import numpy as np
import pytest

from oracle import finance_series as ofs
from tests.helpers import golden_finance


@pytest.mark.parametrize("case", ["columns", "index_agent_id", "no_columns"])
def test_records_match_reference(case):
    meta = golden_finance()
    c = next(c for c in meta["cases"] if c["name"] == case)
    rows = c["rows"]
    if case == "no_columns":
        rows = [{"agent_id": r["agent_id"]} for r in rows]
        assert ofs.records([{} for _ in rows], meta["year"]) is None
        assert c["records"] is None
        return
    got = ofs.records(rows, meta["year"])
    assert len(got) == len(c["records"])
    for a, b in zip(got, c["records"]):
        assert (a["agent_id"], a["year"], a["scenario_case"]) == (b["agent_id"], b["year"], b["scenario_case"])
        for k in ("cf_energy_value", "utility_bill_w_sys", "utility_bill_wo_sys"):
            assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k


def test_golden_covers_edges():
    meta = golden_finance()
    c = meta["cases"][0]
    lens = {len(r["cf_energy_value_pv_batt"]) for r in c["rows"] if isinstance(r["cf_energy_value_pv_batt"], list)}
    assert {10, 21, 26, 31, 51} <= lens                      # short, 26-long, long lists
    assert any(isinstance(r["cf_energy_value_pv_only"], np.ndarray) for r in c["rows"])
    assert any(not np.all(np.isfinite(r["utility_bill_w_sys_pv_batt"])) for r in c["rows"]
               if isinstance(r["utility_bill_w_sys_pv_batt"], list))


def test_row_column_staging_matches_cell_staging():
    """finance_series._stage_rows (a yearly RowColumn staged whole) equals the
    cell-by-cell staging of the same lists: first 51 entries, zero past each
    list's end."""
    from dgen_amd import finance_series as gfs
    from dgen_amd.hourly_column import yearly_column
    rng = np.random.default_rng(3)
    n = 200
    a = rng.normal(size=(n, 60))
    lens = rng.integers(0, 61, n)
    col = yearly_column(a, lens)[::-1]
    got = np.full((n, gfs.STRIDE), 7.0)
    gfs._stage_rows(col, got)
    ref = np.zeros((n, gfs.STRIDE))
    for r, v in enumerate(col):
        k = min(len(v), gfs.STRIDE)
        ref[r, :k] = v[:k]
    assert np.array_equal(got, ref)
    assert col.cells_are_lists()
