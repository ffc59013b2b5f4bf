"""Host tariff compiler vs the reference's normalize_tariff / process_tariff
outputs captured in tests/golden/tariffs.json (bit-exact, incl. float32
rounding) and the SURVEY Appendix C known answers."""
import json
import math

import numpy as np
import pytest

from dgen_amd import tariff as T
from tests import helpers


def _eq(a, b):
    """Exact structural equality with NaN == NaN."""
    if isinstance(a, float) and isinstance(b, float):
        return (a == b) or (math.isnan(a) and math.isnan(b))
    if isinstance(a, (list, tuple)) and isinstance(b, (list, tuple)):
        return len(a) == len(b) and all(_eq(x, y) for x, y in zip(a, b))
    if isinstance(a, dict) and isinstance(b, dict):
        return a.keys() == b.keys() and all(_eq(a[k], b[k]) for k in a)
    if isinstance(a, bool) or isinstance(b, bool):
        return a == b and type(a) == type(b)
    if isinstance(a, (int, float)) and isinstance(b, (int, float)):
        return a == b
    return a == b


def _roundtrip(obj):
    return json.loads(json.dumps(obj))


@pytest.mark.parametrize("case", helpers.golden_tariffs(), ids=lambda c: c["name"])
def test_normalize_matches_reference(case):
    got = _roundtrip(T.normalize_tariff(case["raw"], net_sell_rate_scalar=0.0))
    assert _eq(got, case["normalized"]), case["name"]


@pytest.mark.parametrize("case", helpers.golden_tariffs(), ids=lambda c: c["name"])
def test_process_matches_reference(case):
    _, arr = helpers.golden_agents()
    ws = arr["wholesale"][0] * 1.1
    td = T.normalize_tariff(case["raw"], 0.0)
    for variant, ts in (("ts_none", None), ("ts_8760", ws)):
        got = _roundtrip(T.rate_fields(td, 0.0, ts_sell_rate=ts))
        assert _eq(got, case["process"][variant]), (case["name"], variant)


def test_appendix_c_known_answers():
    g = {c["name"]: c for c in helpers.golden_tariffs()}
    k1 = g["K1"]["normalized"]["ur_ec_tou_mat"]
    assert k1 == [[1, 1, 9.999999680285692e+37, 0, 0.11999999731779099, 0],
                  [2, 1, 9.999999680285692e+37, 0, 0.2800000011920929, 0]]
    k2 = g["K2"]["normalized"]["ur_ec_tou_mat"]
    assert k2[2][2] == 500.0           # period-2 tier-1 cap harmonised to 500
    k3 = g["K3"]["normalized"]
    assert all(v == 1 for row in k3["ur_ec_sched_weekday"] for v in row)   # ids > P clamp to 1
    assert g["K5"]["normalized"]["ur_dc_enable"] == 1
    assert g["K5"]["process"]["ts_none"]["ur_dc_enable"] == 0


def test_record_packing_k3():
    raw = next(c["raw"] for c in helpers.golden_tariffs() if c["name"] == "K3")
    ct = T.compile_tariff(raw, is_ca=False)
    r = ct.record
    assert int(r["P"]) == 2 and int(r["T"]) == 2
    assert (r["wkday"] == 0).all()                   # everything billed at period 1
    assert r["cap"][0] == 300.0
    assert r["buy"][1, 0] == np.float32(0.31)


def test_ca_override_sell_quarter_buy():
    raw = next(c["raw"] for c in helpers.golden_tariffs() if c["name"] == "K1")
    ct = T.compile_tariff(raw, is_ca=True)
    r = ct.record
    assert int(r["mo"]) == 2
    P, Tn = int(r["P"]), int(r["T"])
    assert np.array_equal(r["sell"][:P, :Tn], (r["buy"][:P, :Tn] * 0.25).astype(np.float32).astype(float))


def test_table_dedup_and_keys():
    tt = T.TariffTable()
    a = tt.add({"e_prices": [[0.1]]}, False)
    b = tt.add({"e_prices": [[0.1]]}, False)
    c = tt.add({"e_prices": [[0.1]]}, True)
    d = tt.add({"e_prices": [[0.1]]}, False, key="switch-row:3")
    assert a == b and c != a and d not in (a, c)
    assert tt.array().dtype == T.TARIFF_DTYPE and len(tt) == 3


def test_empty_tariff_flags():
    ct = T.compile_tariff({}, is_ca=False)
    assert int(ct.record["flags"]) & T.ST_EMPTY_EC


def test_too_many_periods_rejected():
    raw = {"e_prices": [[0.1] * 13], "e_wkday_12by24": [[0] * 24] * 12}
    with pytest.raises(T.TariffError):
        T.compile_tariff(raw, is_ca=False)


# ---------------------------------------------------------------------------
# demand charges (extension mode): the reference's process_tariff demand branch
# (ff:604-615) captured with SKIP_DEMAND_CHARGES flipped -> tariffs_dc.json
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("case", helpers.golden_tariffs_dc(), ids=lambda c: c["name"])
def test_demand_compile_matches_reference(case):
    td = T.normalize_tariff(case["raw"], 0.0)
    assert _eq(_roundtrip(td), case["normalized"]), case["name"]
    got = _roundtrip(T.rate_fields(td, 0.0, ts_sell_rate=None, skip_demand_charges=False))
    assert _eq(got, case["process"]), case["name"]
    # the reference's own switch value keeps demand charges off
    off = T.rate_fields(td, 0.0, ts_sell_rate=None)
    assert off["ur_dc_enable"] == 0 and "ur_dc_tou_mat" not in off


def _dc(name):
    case = next(c for c in helpers.golden_tariffs_dc() if c["name"] == name)
    return T.compile_tariff(case["raw"], is_ca=False, skip_demand_charges=False)


def test_demand_record_packing():
    ct = _dc("dc_tou_ur")
    d = ct.demand
    assert d is not None and int(d["flags"]) == 0
    assert list(d["tou_nt"][:3]) == [2, 2, 0] and list(d["flat_nt"]) == [0] * 12
    assert d["tou_cap"][0, 0] == 50.0 and d["tou_price"][1, 1] == np.float32(14.25)
    assert int(d["wkday"][0, 12]) == 1 and int(d["wkday"][0, 11]) == 0 and int(d["wkend"][5, 15]) == 0
    both = _dc("dc_both_ur").demand
    assert list(both["flat_nt"]) == [2] * 12 and both["flat_price"][7, 1] == 7.0
    assert list(both["tou_nt"][:4]) == [1, 1, 1, 0]


def test_demand_flags_outside_ssc_limits():
    # the legacy flat builder numbers months 1..12 (ff:805-806); SSC's month
    # column is 0-based, so month 12 is rejected
    assert int(_dc("dc_legacy_flat_12").record["flags"]) & T.ST_DEMAND
    assert int(_dc("dc_tier_gap").record["flags"]) & T.ST_DEMAND
    assert int(_dc("dc_period9").record["flags"]) & T.ST_DEMAND
    assert int(_dc("dc_ragged_sched").record["flags"]) & T.ST_DEMAND      # zero-padded schedule
    assert _dc("dc_flag_only").demand is None and _dc("dc_nonfinite").demand is None
    assert int(_dc("dc_legacy_tou").record["flags"]) == 0


def test_demand_table_indices():
    tt = T.TariffTable(skip_demand_charges=False)
    a = tt.add(next(c["raw"] for c in helpers.golden_tariffs_dc() if c["name"] == "dc_tou_ur"), False)
    b = tt.add({"e_prices": [[0.1]]}, False)
    c = tt.add(next(c["raw"] for c in helpers.golden_tariffs_dc() if c["name"] == "dc_flat_ur"), False)
    arr = tt.array()
    assert [int(arr[k]["dc"]) for k in (a, b, c)] == [1, 0, 2]
    assert tt.demand_array().shape == (2,)
    assert T.TariffTable().add(next(c["raw"] for c in helpers.golden_tariffs_dc()), False) == 0
