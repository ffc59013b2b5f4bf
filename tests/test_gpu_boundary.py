"""Drop-in boundary on the GPU: calc_system_size_and_performance / size_chunk
with reference-style agent rows vs the golden captures of the reference's own
function (same fields, same values within the stated tolerances)."""
import numpy as np
import pandas as pd
import pytest

from dgen_amd import financial_functions as ff
from tests import helpers

pytestmark = pytest.mark.gpu

SCALARS = ["system_kw", "annual_energy_production_kwh", "naep", "capacity_factor", "price_per_kwh",
           "npv", "batt_kw", "batt_kwh"]
ARRAYS = ["cash_flow", "cf_energy_value_pv_only", "utility_bill_w_sys_pv_only",
          "utility_bill_wo_sys_pv_only", "cf_energy_value_pv_batt", "utility_bill_w_sys_pv_batt",
          "utility_bill_wo_sys_pv_batt"]


def _check_row(out, g, i, arr, hourly=True):
    for k in SCALARS:
        assert np.isclose(out[k], g[k], rtol=1e-6, atol=1e-6), (g["tag"], k, out[k], g[k])
    assert out["payback_period"] == g["payback_period"], g["tag"]
    for k in ARRAYS:
        assert np.allclose(out[k], g[k], rtol=1e-6, atol=1e-5), (g["tag"], k)
    assert out["tariff_id"] == g["final_tariff_id"], g["tag"]
    assert out["nem_system_kw_limit"] == g["nem_system_kw_limit"], g["tag"]
    if hourly:
        for k in ("baseline_net_hourly", "adopter_net_hourly_pvonly", "adopter_net_hourly_with_batt"):
            ref = arr[f"{i}__{k}"]
            assert len(out[k]) == 8760
            # the drop-in path computes the planes in fp64 (dgen_outputs.hourly_f64),
            # like the reference's lists: only the generation term's association
            # (cf x (kW x 0.96 / 1e6) vs ((cf / 1e6) x kW ...)) differs in the last bits
            assert isinstance(out[k][0], float)
            assert np.allclose(out[k], ref, rtol=1e-12, atol=1e-12 * max(1.0, np.abs(ref).max())), (g["tag"], k)


def test_calc_system_size_and_performance_single_rows():
    rows, store, table = helpers.golden_rows()
    meta, arr = helpers.golden_agents()
    for i in (0, 4, 6, 9, 12):          # K1, sticky switch, storage switch, CA, 5 GWh commercial
        out = ff.calc_system_size_and_performance(store, rows[i], None, table)
        assert isinstance(out, pd.Series)
        _check_row(out, meta["agents"][i], i, arr)
        assert out["pv_per_kw_hourly"] == (np.asarray(arr["cfs"][meta["agents"][i]["inputs"]["cf_row"]],
                                                      float) / 1e6).tolist()


def test_size_chunk_matches_golden_and_aggregates():
    rows, store, table = helpers.golden_rows()
    meta, arr = helpers.golden_agents()
    df = pd.DataFrame(rows)
    ff._worker_conn = store
    out, agg = ff.size_chunk(df, None, table, "simple")
    assert list(out.index) == list(df.index)
    assert "pv_per_kw_hourly" not in out.columns
    for i, (aid, r) in enumerate(out.iterrows()):
        _check_row(r, meta["agents"][i], i, arr)
    base = sum(arr[f"{i}__baseline_net_hourly"] * 10.0 for i in range(len(rows)))
    assert agg["n_hours"] == 8760
    assert np.allclose(agg["net_sum_kw"], base, rtol=1e-5)


def test_empty_and_repeated_rows():
    """An empty chunk returns what the reference's loop returns for no rows
    (ff:1209-1218: an empty frame, n_hours 0, no sums); the same agent twice in
    one chunk gives two identical rows, the golden ones."""
    rows, store, table = helpers.golden_rows()
    meta, arr = helpers.golden_agents()
    ff._worker_conn = store
    out, agg = ff.size_chunk(pd.DataFrame(rows).iloc[:0], None, table, "simple")
    assert len(out) == 0 and agg == {"mode": "simple", "n_hours": 0, "net_sum_kw": []}
    r1 = rows[4].copy()
    r1.name = 99
    out, agg = ff.size_chunk(pd.DataFrame([rows[4], r1]), None, table, "simple")
    assert list(out.index) == [rows[4].name, 99]
    for _, r in out.iterrows():
        _check_row(r, meta["agents"][4], 4, arr)
    a, b = out.iloc[0], out.iloc[1]
    for k in SCALARS + ["payback_period"]:
        assert a[k] == b[k], k
    assert np.array_equal(np.asarray(a["adopter_net_hourly_with_batt"]), np.asarray(b["adopter_net_hourly_with_batt"]))


def test_zero_load_raises_like_reference():
    rows, store, table = helpers.golden_rows()
    r = rows[0].copy()
    r["load_kwh_per_customer_in_bin"] = 0.0
    with pytest.raises(ZeroDivisionError):
        ff.calc_system_size_and_performance(store, r, None, table)


def test_kwh_per_kw_units_are_sized_like_the_oracle():
    """kWh/kW tier units (codes 1 and 3: SSC scales the caps by the month's
    peak import) are billed: the agents are sized, no warning, and every
    agent of the chunk matches the oracle's restatement (oracle/orc.c
    month_energy_charge with the month peaks of the billed case)."""
    import warnings
    from dgen_amd.columnar import columnize_frame
    from oracle import oracle as orc
    rows, store, table = helpers.golden_rows()
    df = pd.DataFrame(rows[:6]).copy()
    ones = [[1] * 24 for _ in range(12)]
    df.at[df.index[2], "tariff_dict"] = {"ur_ec_tou_mat": [[1, 1, 150.0, 1, 0.2, 0.0], [1, 2, 1e38, 1, 0.25, 0.0]],
                                         "ur_ec_sched_weekday": ones, "ur_ec_sched_weekend": ones,
                                         "ur_metering_option": 0}
    df.at[df.index[4], "tariff_dict"] = {"e_prices": [[0.12, 0.2], [0.18, 0.3]], "e_levels": [[6.0, 6.0], [1e9, 1e9]],
                                         "energy_rate_unit": "kWh/kW daily",
                                         "e_wkday_12by24": [[1 if 15 <= h < 20 else 0 for h in range(24)]] * 12,
                                         "e_wkend_12by24": [[0] * 24] * 12}
    ff._worker_conn = store
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        out, agg = ff.size_chunk(df, None, table, "simple", hourly="array")
    assert np.isfinite(out["system_kw"].to_numpy(float)).all() and np.isfinite(agg["net_sum_kw"]).all()
    b = columnize_frame(df, store, table)
    cols = b.frame_columns
    recs = b.tariffs.array()
    assert set(recs["unit"][cols["tariff0"][[2, 4]]]) == {1, 3}
    opop = helpers.oracle_population(cols, recs, b.switches.array(), store.shapes, store.cfs, b.wholesale.array())
    ref = opop.run(orc.make_cfg())
    for i, r in enumerate(ref):
        row = out.iloc[i]
        assert abs(row["system_kw"] - r["system_kw"]) <= 1e-9 * max(1.0, r["system_kw"]), i
        for k in ("npv", "batt_kwh"):
            assert np.isclose(row[k], r[k], rtol=1e-6, atol=1e-6), (i, k, row[k], r[k])
        assert row["payback_period"] == r["payback_period"], i
        n1 = int(df["economic_lifetime_yrs"].iloc[i]) + 1
        assert np.allclose(np.asarray(row["utility_bill_w_sys_pv_only"], float), r["bill_w_pv_only"][:n1],
                           rtol=1e-6, atol=1e-5), i
        assert np.allclose(np.asarray(row["utility_bill_w_sys_pv_batt"], float), r["bill_w_pv_batt"][:n1],
                           rtol=1e-6, atol=1e-5), i


def test_size_chunk_array_mode_equals_list_mode():
    """hourly="array" (ndarray row views for every list-valued column) carries
    exactly the values of the reference's list form."""
    rows, store, table = helpers.golden_rows()
    df = pd.DataFrame(rows)
    ff._worker_conn = store
    lst, agg_l = ff.size_chunk(df, None, table, "simple", hourly="list")
    arr, agg_a = ff.size_chunk(df, None, table, "simple", hourly="array")
    assert list(arr.columns) == list(lst.columns)
    assert agg_a["net_sum_kw"] == agg_l["net_sum_kw"]
    for k in ARRAYS + ["baseline_net_hourly", "adopter_net_hourly_pvonly", "adopter_net_hourly_with_batt",
                       "adopter_net_hourly"]:
        for a, l in zip(arr[k], lst[k]):
            assert isinstance(a, np.ndarray) and a.dtype == np.float64, k
            assert np.array_equal(a, np.asarray(l, np.float64)), k


def test_size_chunk_lazy_mode_equals_array_mode():
    """hourly="lazy" (the default): the hourly cells are rows of a plane that
    downloads in the background; np.asarray(cell), len, indexing and pickling
    give the array mode's values exactly."""
    import pickle
    rows, store, table = helpers.golden_rows()
    df = pd.DataFrame(rows)
    ff._worker_conn = store
    arr, agg_a = ff.size_chunk(df, None, table, "simple", hourly="array")
    lz, agg_l = ff.size_chunk(df, None, table, "simple", hourly="lazy")
    assert agg_a["net_sum_kw"] == agg_l["net_sum_kw"]
    for k in ("baseline_net_hourly", "adopter_net_hourly_pvonly", "adopter_net_hourly_with_batt",
              "adopter_net_hourly"):
        for a, c in zip(arr[k], lz[k]):
            assert len(c) == 8760 and c[17] == a[17]
            assert np.array_equal(np.asarray(c, dtype=float), a), k
            assert np.array_equal(pickle.loads(pickle.dumps(c)), a), k
    for k in SCALARS + ["payback_period"]:
        assert np.array_equal(arr[k].to_numpy(float), lz[k].to_numpy(float)), k
    # yearly cells: Python lists, as the reference's finance export requires
    # (finance_series_export.py:51-64), with the array mode's values
    for k in ARRAYS:
        for a, c in zip(arr[k], lz[k]):
            assert isinstance(c, list) and c == a.tolist(), k


def test_device_mode_export_reduces_planes_in_place():
    """size_chunk(hourly="device"): the hourly planes stay in HBM; the per-state
    export (attachment.export_state_hourly_with_storage_mix) sums them there,
    bit-identical to the export of the array mode's host cells, and the planes
    never cross PCIe (until a cell is read: then they match the array mode)."""
    from dgen_amd import attachment as ga
    from dgen_amd.synth import reference_frame
    df, store, table = reference_frame(3000)
    ff._worker_conn = store
    arr, _ = ff.size_chunk(df, None, table, "simple", hourly="array")
    dv, _ = ff.size_chunk(df, None, table, "simple", hourly="device")
    rng = np.random.default_rng(4)
    extra = {"customers_in_bin": rng.uniform(10, 400, len(df)), "number_of_adopters": rng.uniform(0, 20, len(df)),
             "batt_kw_cum_last_year": rng.uniform(0, 30, len(df)),
             "batt_adopters_added_this_year": rng.integers(0, 3, len(df))}
    recs = []
    for frame in (arr, dv):
        f = frame.copy()
        for k, v in extra.items():
            f[k] = v
        f = f.iloc[::-1]                 # a reordered frame: rows map to their own device columns
        recs.append(ga.export_state_hourly_with_storage_mix("eng", "s", "o", 2027, f))
    planes = [dv[k].array._plane for k in ("baseline_net_hourly", "adopter_net_hourly_pvonly",
                                           "adopter_net_hourly_with_batt")]
    assert not any(p.done() for p in planes)                    # nothing downloaded
    a, d = recs
    assert a["state_abbr"].tolist() == d["state_abbr"].tolist()
    assert a["n_hours"].tolist() == d["n_hours"].tolist()
    for x, y in zip(a["net_sum"], d["net_sum"]):
        assert np.array_equal(np.asarray(x), np.asarray(y))
    j = len(df) // 2
    assert np.array_equal(np.asarray(dv["adopter_net_hourly_with_batt"].iloc[j]),
                          np.asarray(arr["adopter_net_hourly_with_batt"].iloc[j]))


def test_sub_batched_frame_equals_one_call():
    """A frame larger than the device budget (forced: 50k rows) is sized in
    consecutive sub-batches (financial_functions._run_device): every output --
    scalars, yearly lists, the three fp64 hourly planes, the rewritten tariff
    columns -- bit-identical to one call over the whole frame; size_chunk's
    net_sum_kw (a sum over the sub-batches' sums) within 1e-12 relative."""
    from dgen_amd.synth import reference_frame
    df, store, table = reference_frame(200_000)
    ff._worker_conn = store
    tm1, tm4 = {}, {}
    one, agg1 = ff.size_chunk(df, None, table, "simple", timing=tm1, max_rows=len(df))
    sub, agg4 = ff.size_chunk(df, None, table, "simple", timing=tm4, max_rows=50_000)
    assert "sub_batches" not in tm1 and tm4["sub_batches"] == 4
    assert list(sub.index) == list(df.index) and list(sub.columns) == list(one.columns)
    for k in SCALARS + ["payback_period", "tariff_id", "nem_system_kw_limit"]:
        assert one[k].equals(sub[k]), k              # NaN == NaN (no switch: the limit stays NaN)
    for k in ARRAYS:
        assert np.array_equal(one[k].array.to_2d(), sub[k].array.to_2d()), k
    for k in ("baseline_net_hourly", "adopter_net_hourly_pvonly", "adopter_net_hourly_with_batt"):
        a = one[k].array.to_2d()
        seg = sub[k].array._plane
        assert len(seg.parts) == 4
        for (p, idx, _), lo in zip(seg.parts, seg.off[:-1]):
            assert np.array_equal(p.result()[idx], a[lo:lo + idx.shape[0]]), k
        del a
    n1, n4 = np.asarray(agg1["net_sum_kw"]), np.asarray(agg4["net_sum_kw"])
    assert np.allclose(n1, n4, rtol=1e-12, atol=0.0)
    # the per-row form reads the same cells
    j = 123_457
    assert np.array_equal(np.asarray(sub["adopter_net_hourly_with_batt"].iloc[j]),
                          np.asarray(one["adopter_net_hourly_with_batt"].iloc[j]))


def test_device_mode_export_with_repeated_rows_uses_host_sums():
    """A frame whose rows repeat a plane column (pd.concat([df, df])): the
    device export cannot scatter two rows' weights into one column, so it
    takes the host path -- the same records as the array mode's frame."""
    from dgen_amd import attachment as ga
    from dgen_amd.synth import reference_frame
    df, store, table = reference_frame(600)
    ff._worker_conn = store
    arr, _ = ff.size_chunk(df, None, table, "simple", hourly="array")
    dv, _ = ff.size_chunk(df, None, table, "simple", hourly="device")
    rng = np.random.default_rng(5)
    recs = []
    w = {"customers_in_bin": rng.uniform(10, 400, 2 * len(df)),
         "number_of_adopters": rng.uniform(0, 20, 2 * len(df)),
         "batt_kw_cum_last_year": rng.uniform(0, 30, 2 * len(df)),
         "batt_adopters_added_this_year": rng.integers(0, 3, 2 * len(df))}
    for frame in (arr, dv):
        f = pd.concat([frame, frame])
        for k, v in w.items():
            f[k] = v
        recs.append(ga.export_state_hourly_with_storage_mix("eng", "s", "o", 2027, f))
    a, d = recs
    assert a["state_abbr"].tolist() == d["state_abbr"].tolist()
    for x, y in zip(a["net_sum"], d["net_sum"]):
        assert np.array_equal(np.asarray(x), np.asarray(y))
