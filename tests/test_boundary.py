"""Host side of the drop-in boundary (no GPU): profile sources, columnarisation
of reference-style agent rows, rate-switch candidate expansion, error mapping."""
import sqlite3
import json

import numpy as np
import pandas as pd
import pytest

from dgen_amd import _lib
from dgen_amd import financial_functions as ff
from dgen_amd.profiles import ProfileStore, SqlProfileSource
from tests import helpers


def test_columnarize_golden_rows_matches_builder():
    rows, store, table = helpers.golden_rows()
    b = ff._columnarize(rows, store, table)
    cols = b.columns()
    b2, cols2, shapes, cfs, _ = helpers.golden_population()
    for k in cols:
        if k in ("load_row", "cf_row"):
            continue
        assert np.array_equal(cols[k], cols2[k]), k
    assert np.array_equal(store.shapes[cols["load_row"]], shapes[cols2["load_row"]])
    assert np.array_equal(store.cfs[cols["cf_row"]], cfs[cols2["cf_row"]])
    assert np.array_equal(b.tariffs.array(), b2.tariffs.array())
    assert np.array_equal(b.switches.array(), b2.switches.array())


def test_switch_candidates_follow_reference_filter():
    rows, store, table = helpers.golden_rows()
    b = ff._columnarize(rows, store, table)
    cols = b.columns()
    sw = b.switches.array()
    for i, r in enumerate(rows):
        for tech in ("solar", "storage"):
            ref = table[(table["tech"] == tech) & (table["eia_id"] == r["eia_id"]) &
                        (table["res_com"] == str(r["sector_abbr"]).upper()[0])]
            off, cnt = cols[f"sw_{tech}_off"][i], cols[f"sw_{tech}_cnt"][i]
            assert cnt == len(ref)
            got = sw[off:off + cnt]
            assert np.array_equal(got["min_kw"], ref["min_kw_limit"].to_numpy(float))
            assert np.array_equal(got["max_kw"], ref["max_kw_limit"].to_numpy(float))
            assert np.array_equal(got["one_time_charge"], ref["one_time_charge"].to_numpy(float))


def test_wholesale_nonfinite_disables_ts():
    rows, store, table = helpers.golden_rows()
    b = ff._columnarize(rows, store, table)
    cols = b.columns()
    tags = [a["tag"] for a in helpers.golden_agents()[0]["agents"]]
    assert cols["wholesale_row"][tags.index("res_mo2_nan_ts")] == -1
    assert cols["wholesale_row"][tags.index("res_CA")] == -1        # CA: ts_sell None
    assert cols["wholesale_row"][tags.index("res_mo2_ts")] >= 0


def test_scratch_slots_for_net_billing_agents():
    rows, store, table = helpers.golden_rows()
    b = ff._columnarize(rows, store, table)
    cols = b.columns()
    tr = b.tariffs.array()
    for i in range(len(rows)):
        if tr["mo"][cols["tariff0"][i]] == 2:
            assert cols["scratch_slot"][i] >= 0


def test_rate_switch_table_required_like_reference():
    rows, store, _ = helpers.golden_rows()
    with pytest.raises(AttributeError):
        ff.size_rows(rows[:1], store, None)


def test_status_mapping():
    ids = ["a", "b"]
    with pytest.raises(ZeroDivisionError):
        ff._raise_for_status(np.array([0, _lib.ST_ZERO_LOAD], np.int32), ids)
    with pytest.raises(ValueError):
        ff._raise_for_status(np.array([_lib.ST_BOUNDS, 0], np.int32), ids)
    with pytest.raises(_lib.DgenError):
        ff._raise_for_status(np.array([_lib.ST_TARIFF, 0], np.int32), ids)
    ff._raise_for_status(np.array([0, 0], np.int32), ids)


def test_profile_store_keys_and_validation():
    st = ProfileStore()
    k = st.add_load((1, "res", "DE"), np.ones(8760))
    assert st.add_load((np.int64(1), "res", "DE"), np.ones(8760)) == k
    with pytest.raises(ValueError):
        st.add_load((2, "res", "DE"), np.ones(10))
    with pytest.raises(ValueError):
        st.add_solar((1, 20, 180), np.full(8760, 0.5))
    with pytest.raises(KeyError):
        st.load_row({"bldg_id": 9, "sector_abbr": "res", "state_abbr": "DE"})


def _sqlite_con(shapes, cfs):
    con = sqlite3.connect(":memory:")
    con.execute("ATTACH DATABASE ':memory:' AS diffusion_load_profiles")
    con.execute("ATTACH DATABASE ':memory:' AS diffusion_resource_solar")
    con.execute("CREATE TABLE diffusion_load_profiles.resstock_load_profiles "
                "(bldg_id INTEGER, sector_abbr TEXT, state_abbr TEXT, kwh_load_profile TEXT)")
    con.execute("CREATE TABLE diffusion_resource_solar.solar_resource_hourly "
                "(solar_re_9809_gid TEXT, tilt TEXT, azimuth TEXT, cf TEXT)")
    for k, row in enumerate(shapes):
        con.execute("INSERT INTO diffusion_load_profiles.resstock_load_profiles VALUES (?,?,?,?)",
                    (1000 + k, "res", "DE", json.dumps(row.astype(float).tolist())))
    for k, row in enumerate(cfs):
        con.execute("INSERT INTO diffusion_resource_solar.solar_resource_hourly VALUES (?,?,?,?)",
                    (str(5000 + k), "20", "180", json.dumps(row.tolist())))
    return con


def test_sql_source_runs_reference_queries():
    _, arr = helpers.golden_agents()
    con = _sqlite_con(arr["shapes"][:2], arr["cfs"][:2])
    src = SqlProfileSource(con)
    agents = [{"bldg_id": 1001, "sector_abbr": "res", "state_abbr": "DE",
               "solar_re_9809_gid": 5000, "tilt": 20, "azimuth": 180}]
    src.ensure(agents)
    assert np.array_equal(src.shapes[src.load_row(agents[0])], arr["shapes"][1])
    assert np.array_equal(src.cfs[src.solar_row(agents[0])], arr["cfs"][0])


def _frame_vs_rows(df, store, table):
    from dgen_amd.columnar import columnize_frame
    rows = []
    for aid, row in df.iterrows():
        r = row.copy()
        r.name = aid
        rows.append(r)
    b1 = ff._columnarize(rows, store, table)
    c1 = b1.columns()
    b2 = columnize_frame(df, store, table)
    c2 = b2.frame_columns
    for k in c1:
        assert np.array_equal(c1[k], c2[k], equal_nan=True), k
        assert c1[k].dtype == c2[k].dtype, k
    assert np.array_equal(b1.tariffs.array(), b2.tariffs.array())
    assert np.array_equal(b1.switches.array(), b2.switches.array())
    w1, w2 = b1.wholesale.array(), b2.wholesale.array()
    assert (w1 is None and w2 is None) or np.array_equal(w1, w2)


def test_columnize_frame_matches_row_builder_golden():
    rows, store, table = helpers.golden_rows()
    _frame_vs_rows(pd.DataFrame(rows), store, table)


def test_columnize_frame_matches_row_builder_synthetic():
    """Shared tariff dicts / wholesale arrays (as merges leave them), CA rows,
    rate-switch candidates, and wholesale arrays that only some multipliers
    make non-finite in float32 (the row enters the table at its first valid
    use, as in the row builder)."""
    from dgen_amd.synth import reference_frame
    df, store, table = reference_frame(3000, seed=11)
    # the same county array with a multiplier that overflows float32 first
    big = np.full(8760, 1e36)
    idx = df.index[df["state_abbr"] != "CA"][:6]
    df.loc[idx[:3], "wholesale_prices"] = pd.Series([big, big, big], index=idx[:3])
    df.loc[idx[0], "elec_price_multiplier"] = 1e3          # 1e39 -> inf in f32: no TS row
    df.loc[idx[1], "elec_price_multiplier"] = 1.0
    nan_arr = np.full(8760, 0.03)
    nan_arr[5] = np.nan
    df.loc[idx[3:5], "wholesale_prices"] = pd.Series([nan_arr, nan_arr], index=idx[3:5])
    df.loc[idx[5], "wholesale_prices"] = None
    _frame_vs_rows(df, store, table)
