"""GPU parity: the HIP path (through the C-ABI) vs the golden boundary captures
(reference driver + oracle SSC primitives) and vs the CPU oracle.

Tolerances: integer / index work bit-exact (Brent evaluation count, rate-switch
state, tariff-period assignment via slot sums, numpy-order row sums);
floating point within the north star's 1e-6 relative on bills / NPV / payback,
and the chosen kW within scipy's xatol (in practice the Brent path is
identical and kW agrees to ~1e-15).
"""
import numpy as np
import pytest

from tests import helpers

pytestmark = pytest.mark.gpu

RTOL = 1e-6


def _close(a, b, rtol=RTOL, atol=1e-6):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    return np.allclose(a, b, rtol=rtol, atol=atol, equal_nan=True)


@pytest.fixture(scope="module")
def golden_gpu(engine):
    from dgen_amd.engine import outputs_to_host
    b, cols, shapes, cfs, ws = helpers.golden_population()
    engine.load_profiles(shapes, cfs, ws)
    engine.set_tariffs(b.tariffs.array())
    engine.set_switches(b.switches.array())
    batch = engine.upload_agents(cols)
    out = engine.alloc_outputs(batch.n, hourly=True)
    engine.size(batch, out)
    import torch
    torch.cuda.synchronize()
    return b, cols, outputs_to_host(out)


def test_prep_row_sums_bit_exact(engine):
    _, arr = helpers.golden_agents()
    engine.load_profiles(arr["shapes"], arr["cfs"], arr["wholesale"])
    s, naep = engine.profile_sums()
    for k, row in enumerate(arr["shapes"]):
        assert s[k] == row.astype(np.float64).sum()
    for k, row in enumerate(arr["cfs"]):
        assert naep[k] == (np.asarray(row, dtype=float) / 1e6).sum()


def test_brent_selftest_matches_scipy(engine):
    cases = helpers.golden_brent()
    xs, xo, nf = engine.brent_selftest([c["low"] for c in cases], [c["high"] for c in cases],
                                       [c["xatol"] for c in cases], [c["c2"] for c in cases],
                                       [c["x0"] for c in cases], [c["c1"] for c in cases], maxn=64)
    for k, c in enumerate(cases):
        assert nf[k] == c["nfev"], c
        assert xs[k, : c["nfev"]].tolist() == c["xs"], c
        assert xo[k] == c["x"], c


def test_golden_agents_scalars(golden_gpu):
    b, cols, o = golden_gpu
    meta, _ = helpers.golden_agents()
    for i, g in enumerate(meta["agents"]):
        tag = g["tag"]
        assert o["status"][i] == 0, (tag, o["status"][i])
        assert o["nfev"][i] == len(g["evals_pv"]), tag
        assert abs(o["system_kw"][i] - g["system_kw"]) <= 1e-9 * max(1.0, g["system_kw"]), tag
        assert abs(o["x_last"][i] - g["evals_pv"][-1]) <= 1e-9 * max(1.0, g["system_kw"]), tag
        for k_o, k_g in (("annual_kwh", "annual_energy_production_kwh"), ("naep", "naep"),
                         ("capacity_factor", "capacity_factor"), ("price_per_kwh", "price_per_kwh"),
                         ("npv", "npv"), ("batt_kw", "batt_kw"), ("batt_kwh", "batt_kwh")):
            assert _close(o[k_o][i], g[k_g]), (tag, k_o, o[k_o][i], g[k_g])
        assert o["payback_period"][i] == g["payback_period"], (tag, o["payback_period"][i])
        tid = helpers.final_tariff_id(b, 900 + i, o["tariff_final"][i], o["switched"][i])
        assert tid == g["final_tariff_id"], tag
        assert (1e6 if o["switched"][i] else 100.0) == g["nem_system_kw_limit"], tag


def test_golden_agents_arrays(golden_gpu):
    b, cols, o = golden_gpu
    meta, _ = helpers.golden_agents()
    pairs = (("cash_flow", "cash_flow"), ("cfev_pv", "cf_energy_value_pv_only"),
             ("bill_w_pv", "utility_bill_w_sys_pv_only"), ("bill_wo_pv", "utility_bill_wo_sys_pv_only"),
             ("cfev_batt", "cf_energy_value_pv_batt"), ("bill_w_batt", "utility_bill_w_sys_pv_batt"),
             ("bill_wo_batt", "utility_bill_wo_sys_pv_batt"))
    for i, g in enumerate(meta["agents"]):
        n1 = len(g["cash_flow"])
        for k_o, k_g in pairs:
            assert _close(o[k_o][i, :n1], g[k_g], atol=1e-5), (g["tag"], k_o)


def test_golden_agents_hourly(golden_gpu):
    b, cols, o = golden_gpu
    meta, arr = helpers.golden_agents()
    for i, g in enumerate(meta["agents"]):
        for k_o, k_g in (("baseline", "baseline_net_hourly"), ("net_pvonly", "adopter_net_hourly_pvonly"),
                         ("net_with_batt", "adopter_net_hourly_with_batt")):
            ref = arr[f"{i}__{k_g}"]
            got = o[k_o][i].astype(np.float64)
            # fp32 hourly planes: 1 ulp of fp32 plus the dispatch's fp64 noise
            assert np.allclose(got, ref, rtol=2e-6, atol=2e-6 * max(1.0, float(np.abs(ref).max()))), \
                (g["tag"], k_o, float(np.abs(got - ref).max()))
