"""Demand charges (extension mode; the reference keeps them off, ff:35): GPU vs
the CPU oracle's restatement on seeded commercial populations whose tariffs
carry monthly flat and TOU demand charges (dgen_amd.synth 'com_dc_batt'), NEM
and net billing, with the battery run.  The compile of the demand mats is
pinned to the reference (tests/test_tariff.py, tariffs_dc.json); the SSC
demand arithmetic is parity unpinned, so this checks GPU == restatement."""
import numpy as np
import pytest
import torch

from dgen_amd.columnar import assign_scratch
from dgen_amd.engine import outputs_to_host
from dgen_amd.synth import make_population
from oracle import oracle as orc
from tests import helpers

pytestmark = pytest.mark.gpu


def _pop(n, net_billing=False, seed=7, long_life=False):
    pop = make_population("com_dc_batt", n, seed=20260000 + seed, n_res_shapes=16, n_com_shapes=32,
                          n_cf=32, n_counties=16, n_tariffs=24)
    if long_life:            # 33..50-year lives: one agent per wave (64 year lanes)
        life = pop.cols["econ_life"].copy()
        life[::3] = 33 + (np.arange(life[::3].size) % 18)
        pop.cols["econ_life"] = life
    if net_billing:          # every other tariff bills net (mo 2): hourly imports + demand
        t = pop.tariffs.copy()
        t["mo"][1::2] = 2
        pop.tariffs = t
        pop.n_scratch = assign_scratch(pop.cols, pop.tariffs, pop.switches)
    return pop


def _run(eng, pop, demand):
    eng.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
    eng.set_tariffs(pop.tariffs, demand)
    eng.set_switches(pop.switches)
    batch = eng.upload_agents(pop.cols, pop.n_scratch)
    out = eng.alloc_outputs(batch.n, hourly=True)
    eng.size(batch, out)
    torch.cuda.synchronize()
    return outputs_to_host(out)


def _check(o, ref, life, pop, opop):
    """Every agent against the oracle, on the oracle's Brent path (the
    certified paths re-run the agents a device / oracle difference bound does
    not settle in the oracle's arithmetic)."""
    for i, r in enumerate(ref):
        assert o["status"][i] == 0 and r["status"] == 0, i
        assert helpers.same_path(o, i, r), (i, o["nfev"][i], r["nfev"], o["system_kw"][i], r["system_kw"])
        assert o["tariff_final"][i] == r["tariff_final"], i
        assert abs(o["system_kw"][i] - r["system_kw"]) <= 1e-9 * max(1.0, r["system_kw"]), i
        for k in ("npv", "first_with", "first_without", "batt_kwh", "npv_pv_batt"):
            assert np.isclose(o[k][i], r[k], rtol=1e-6, atol=1e-6), (i, k, o[k][i], r[k])
        assert o["payback_period"][i] == r["payback_period"], i
        N1 = int(life[i]) + 1
        for k_o, k_r in (("bill_w_pv", "bill_w_pv_only"), ("bill_wo_pv", "bill_wo_pv_only"),
                         ("bill_w_batt", "bill_w_pv_batt"), ("bill_wo_batt", "bill_wo_pv_batt"),
                         ("cash_flow", "cash_flow")):
            assert np.allclose(o[k_o][i, :N1], r[k_r], rtol=1e-6, atol=1e-5), (i, k_o)


@pytest.mark.parametrize("net_billing,long_life", [(False, False), (True, False), (True, True)])
def test_demand_charges_match_oracle(engine_dc, net_billing, long_life):
    pop = _pop(160, net_billing, long_life=long_life)
    assert pop.demand.size and (pop.tariffs["dc"] > 0).all()
    o = _run(engine_dc, pop, pop.demand)
    opop = helpers.oracle_population(pop.cols, pop.tariffs, pop.switches, pop.shapes, pop.cfs,
                                     pop.wholesale, demand=pop.demand)
    _check(o, opop.run(orc.make_cfg()), pop.cols["econ_life"], pop, opop)


def test_reference_mode_ignores_demand_records(engine, engine_dc):
    """skip_demand_charges = 1 (the reference) bills exactly as if the tariffs
    had no demand records; billing them raises every no-system bill."""
    pop = _pop(96, seed=9)
    o_ref = _run(engine, pop, pop.demand)
    stripped = pop.tariffs.copy()
    stripped["dc"] = 0
    o_plain = _run(engine, type(pop)(**{**pop.__dict__, "tariffs": stripped}), None)
    for k in ("system_kw", "npv", "first_without", "npv_pv_batt"):
        assert np.array_equal(o_ref[k], o_plain[k]), k
    o_dc = _run(engine_dc, pop, pop.demand)
    assert (o_dc["first_without"] > o_ref["first_without"]).all()


def _run_records(eng, pop, demand, cap):
    eng.set_dc_records(cap)
    try:
        return _run(eng, pop, demand)
    finally:
        eng.set_dc_records(True)


@pytest.mark.parametrize("net_billing,long_life", [(False, False), (True, False), (True, True)])
def test_demand_records_bit_identical(engine_dc, net_billing, long_life):
    """The battery-case demand pass over the scan's records (default), over the
    system-output plane (records off) and with records that overflow a small
    capacity (those agents fall back to the plane) give bit-identical outputs:
    the peaks are maxima of the same imports."""
    pop = _pop(160, net_billing, seed=11, long_life=long_life)
    on = _run_records(engine_dc, pop, pop.demand, True)
    off = _run_records(engine_dc, pop, pop.demand, False)
    small = _run_records(engine_dc, pop, pop.demand, 24)
    for k in ("system_kw", "npv", "npv_pv_batt", "first_without", "bill_w_batt", "bill_wo_batt",
              "cfev_batt", "batt_kwh", "net_with_batt"):
        assert np.array_equal(on[k], off[k], equal_nan=True), k
        assert np.array_equal(small[k], off[k], equal_nan=True), k


def test_kwh_per_kw_records_bit_identical(engine):
    """kWh/kW tier peaks (reference mode, the PK kernels) from the records equal
    the staged pass over the plane, bit for bit."""
    pop = make_population("com_kwkw", 192, seed=20260000 + 21, n_res_shapes=16, n_com_shapes=32,
                          n_cf=32, n_counties=16, n_tariffs=24)
    on = _run_records(engine, pop, pop.demand, True)
    off = _run_records(engine, pop, pop.demand, False)
    for k in ("system_kw", "npv", "npv_pv_batt", "bill_w_batt", "bill_wo_batt", "status"):
        assert np.array_equal(on[k], off[k], equal_nan=True), k


def test_short_demand_period_table_is_flagged(engine_dc):
    """A C-ABI caller whose dgen_tables.max_dc_periods is smaller than the
    periods its demand schedules use (Engine.set_tariffs fills it correctly):
    the battery-case scan sizes its per-period LDS maxima from that field, so an
    hour of a later period flags DGEN_ST_DEMAND on the agent instead of being
    written past the region; the same engine with the right field then gives the
    untouched result again, bit for bit."""
    from dgen_amd import _lib
    pop = _pop(96, seed=13)
    assert int(max(pop.demand["wkday"].max(), pop.demand["wkend"].max())) >= 1
    good = _run(engine_dc, pop, pop.demand)
    assert (good["status"] == 0).all()
    engine_dc.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
    engine_dc.set_tariffs(pop.tariffs, pop.demand)
    engine_dc.set_switches(pop.switches)
    engine_dc.tables.max_dc_periods = 1          # malformed: the schedules use more
    batch = engine_dc.upload_agents(pop.cols, pop.n_scratch)
    out = engine_dc.alloc_outputs(batch.n, hourly=True)
    engine_dc.size(batch, out)
    torch.cuda.synchronize()
    bad = outputs_to_host(out)
    flagged = (bad["status"] & _lib.ST_DEMAND) != 0
    assert flagged.any()
    again = _run(engine_dc, pop, pop.demand)
    for k in ("status", "system_kw", "npv", "npv_pv_batt", "batt_kwh", "first_without"):
        assert np.array_equal(again[k], good[k], equal_nan=True), k


def _run_prebuild(eng, pop, demand, on):
    eng.set_dc_prebuild(on)
    try:
        o = _run(eng, pop, demand)
        assert eng.last_paths()["dc_prebuild"] == int(on)
        return o
    finally:
        eng.set_dc_prebuild(True)


@pytest.mark.parametrize("net_billing,long_life", [(False, False), (True, False), (True, True)])
def test_prebuilt_envelopes_bit_identical(engine_dc, net_billing, long_life):
    """The PV-only search's demand envelopes prebuilt by k_dc_env (day lanes,
    default) or built inside k_size (hour lanes): the same kept lines, so
    every output -- Brent path, bills, NPV, planes -- is bit-identical."""
    pop = _pop(160, net_billing, seed=13, long_life=long_life)
    on = _run_prebuild(engine_dc, pop, pop.demand, True)
    off = _run_prebuild(engine_dc, pop, pop.demand, False)
    for k in on:
        if on[k] is not None:
            assert np.array_equal(on[k], off[k], equal_nan=True), k


def test_prebuilt_envelopes_kwh_per_kw_bit_identical(engine):
    """The same for kWh/kW tier peaks (reference mode, PK kernels)."""
    pop = make_population("com_kwkw", 192, seed=20260000 + 23, n_res_shapes=16, n_com_shapes=32,
                          n_cf=32, n_counties=16, n_tariffs=24)
    on = _run_prebuild(engine, pop, pop.demand, True)
    off = _run_prebuild(engine, pop, pop.demand, False)
    for k in on:
        if on[k] is not None:
            assert np.array_equal(on[k], off[k], equal_nan=True), k


@pytest.mark.parametrize("long_life", [False, True])
def test_no_net_kernels_bit_identical(engine_dc, long_life):
    """A demand-charge batch none of whose agents can bill net runs the
    NET = false instantiations of k_size / k_batt_finance (dgen_tables.no_net,
    set per batch); forcing the NET = true ones gives every output bit for bit
    (the net-billing paths are unreachable for these agents)."""
    pop = _pop(160, False, seed=17, long_life=long_life)
    eng = engine_dc
    eng.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
    eng.set_tariffs(pop.tariffs, pop.demand)
    eng.set_switches(pop.switches)
    res = []
    for no_net in (True, False):
        batch = eng.upload_agents(pop.cols, pop.n_scratch)
        assert batch.no_net                 # C4's table holds net variants no agent reaches
        batch.no_net = no_net
        out = eng.alloc_outputs(batch.n, hourly=True)
        eng.size(batch, out)
        torch.cuda.synchronize()
        res.append(outputs_to_host(out))
    a, b = res
    for k in a:
        if a[k] is not None:
            assert np.array_equal(a[k], b[k], equal_nan=True), k
