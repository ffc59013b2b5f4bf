"""Oracle restatement of the battery-attachment allocation and the per-state
hourly export (oracle/attach.py) against the reference's own outputs
(tests/golden/attach.json, make_golden_attach.py): bit-exact."""
import numpy as np
import pytest

from oracle import attach as oa
from tests.helpers import golden_attach

CASES = [c["name"] for c in golden_attach()[0]["cases"]]


def _case(name):
    meta, hourly = golden_attach()
    c = next(c for c in meta["cases"] if c["name"] == name)
    return c, hourly[name]


@pytest.mark.parametrize("name", CASES)
def test_allocation_matches_reference(name):
    c, _ = _case(name)
    i = c["inputs"]
    got = oa.allocate(i["state_abbr"], i["sector_abbr"], i["agent_id"], i["new_adopters"],
                      i["storage_attachment_rate"], i["batt_kw"], i["batt_kwh"],
                      i["batt_kw_cum_last_year"], i["batt_kwh_cum_last_year"])
    for k, v in c["alloc"].items():
        assert np.array_equal(np.asarray(got[k]), np.asarray(v)), k


@pytest.mark.parametrize("name", CASES)
def test_state_export_matches_reference(name):
    c, (base, pvo, wbt) = _case(name)
    i = c["inputs"]
    w = oa.weights(i["customers_in_bin"], i["number_of_adopters"], i["batt_kw_cum_last_year"],
                   i["batt_kw"], c["alloc"]["batt_adopters_added_this_year"])
    got = oa.export(i["state_abbr"], base, pvo, wbt, w)
    assert got["state_abbr"] == c["export"]["state_abbr"]
    for a, b in zip(got["net_sum"], c["export"]["net_sum"]):
        assert np.array_equal(a, np.asarray(b))


def test_golden_covers_edges():
    meta, _ = golden_attach()
    names = {c["name"]: c for c in meta["cases"]}
    # the tie case exercises the agent_id tie-break; str_ids: string order != numeric
    assert sum(names["ties"]["alloc"]["batt_adopters_added_this_year"]) > 0
    assert sum(names["str_ids"]["alloc"]["batt_adopters_added_this_year"]) > 0


def test_host_grouping_matches_pandas():
    """dgen_amd.attachment's host grouping == pandas groupby(sort=False)
    (first-appearance groups, row order inside, NaN keys dropped) and the
    agent_id tie-break ranks == Python string order."""
    import pandas as pd
    from dgen_amd.attachment import group_segments, string_ranks
    rng = np.random.default_rng(1)
    st = list(rng.choice(["CA", "DE", "NY", None], 300))
    st = [float("nan") if s is None else s for s in st]
    sec = list(rng.choice(["res", "com"], 300))
    idx, off, keys = group_segments(list(zip(st, sec)))
    df = pd.DataFrame({"s": st, "c": sec})
    groups = [(k, g.index.to_numpy()) for k, g in df.groupby(["s", "c"], sort=False)]
    assert [k for k, _ in groups] == keys
    for g, (_, rows) in enumerate(groups):
        assert np.array_equal(idx[off[g]:off[g + 1]], rows)
    ids = [9, 10, 100, 1, 1000, 99, 2]
    r = string_ranks(ids)
    assert [ids[i] for i in np.argsort(r)] == sorted(ids, key=str)
