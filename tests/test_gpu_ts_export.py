"""Round-4 device paths against the forms they replace:

* the TS sell-rate agents' battery-case net-billing split built in a scan of
  their own (k_hourly_batt<TS>, batches with hourly planes) against the plane
  pass it replaces (DGEN_TS_SCAN=0: k_batt_finance's yl_nb_build<true>) and
  against the oracle, and its independence of the batch an agent is sized in;
* the per-state export through one combined plane (dgen_export_plane +
  dgen_state_hourly planes_f32 = 3) against the three-plane form, bit for bit.
"""
import os

import numpy as np
import pytest
import torch

from dgen_amd.engine import Engine, outputs_to_host, path_class, profile_order
from dgen_amd.synth import make_population
from oracle import oracle as orc
from tests import helpers

pytestmark = pytest.mark.gpu

BATT = ("npv_pv_batt", "bill_w_batt", "bill_wo_batt", "cfev_batt")


def _pop(n, seed=20260417):
    return make_population("national_mixed", n, seed=seed, n_res_shapes=64, n_com_shapes=32, n_cf=32,
                           n_counties=16, n_tariffs=48)


def _size(eng, pop, cols=None, hourly=True):
    cols = pop.cols if cols is None else cols
    eng.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
    eng.set_tariffs(pop.tariffs)
    eng.set_switches(pop.switches)
    batch = eng.upload_agents(cols, order=profile_order(cols))
    out = eng.alloc_outputs(batch.n, hourly=hourly)
    eng.size(batch, out)
    torch.cuda.synchronize()
    return outputs_to_host(out, batch.perm), batch, out


def test_ts_scan_matches_plane_pass_and_oracle(engine):
    """The TS agents' scan-built split bills what the plane pass bills (the
    split's sums re-associate: 1e-9 relative) and what the oracle bills
    (1e-6); every other output is bit-identical."""
    pop = _pop(600)
    ts = path_class(pop.cols) == 2
    assert ts.sum() >= 40
    on, _, _ = _size(engine, pop)
    old = os.environ.get("DGEN_TS_SCAN")
    os.environ["DGEN_TS_SCAN"] = "0"                 # read by dgen_open
    try:
        eng_off = Engine(0, engine.cfg)
        off, _, _ = _size(eng_off, pop)
        eng_off.close()
    finally:
        if old is None:
            os.environ.pop("DGEN_TS_SCAN")
        else:
            os.environ["DGEN_TS_SCAN"] = old
    for k in ("system_kw", "npv", "nfev", "batt_kwh", "batt_kw", "annual_kwh", "net_with_batt"):
        assert np.array_equal(on[k], off[k], equal_nan=True), k
    for k in BATT:
        a, b = np.asarray(on[k], np.float64), np.asarray(off[k], np.float64)
        assert np.allclose(a, b, rtol=1e-9, atol=1e-9, equal_nan=True), k
    opop = helpers.oracle_population(pop.cols, pop.tariffs, pop.switches, pop.shapes, pop.cfs, pop.wholesale)
    ref = opop.run(orc.make_cfg(), hourly=False)
    for i in np.flatnonzero(ts):
        assert np.isclose(on["npv_pv_batt"][i], ref[i]["npv_pv_batt"], rtol=1e-6, atol=1e-6), i


def test_ts_agent_independent_of_batch(engine):
    """With hourly planes a TS agent's battery outputs are the same bits in
    the national batch, in a batch of the TS agents alone and alone."""
    pop = _pop(900, seed=20260418)
    ts = np.flatnonzero(path_class(pop.cols) == 2)
    full, _, _ = _size(engine, pop)
    part, _, _ = _size(engine, pop, {k: np.asarray(v)[ts] for k, v in pop.cols.items()})
    for k in BATT:
        assert np.array_equal(full[k][ts], part[k], equal_nan=True), k
    j = int(ts[0])
    one, _, _ = _size(engine, pop, {k: np.asarray(v)[[j]] for k, v in pop.cols.items()})
    for k in BATT:
        assert np.array_equal(full[k][j], one[k][0], equal_nan=True), k


def test_ts_agent_outputs_with_and_without_planes(engine):
    """The one dependence on the hourly flag: a TS sell-rate
    agent's battery-case split is built by its own scan when planes are
    requested and by k_batt_finance's plane pass otherwise, so the four
    battery-case money outputs of those agents differ between the two calls by
    the re-association of the split's sums (pinned here at 1e-9 relative);
    the search, the sizing and every discrete decision are bit-identical, and
    every other agent's outputs are the same bits."""
    pop = _pop(800, seed=20260421)
    ts = path_class(pop.cols) == 2
    assert ts.sum() >= 40
    on, _, _ = _size(engine, pop, hourly=True)
    off, _, _ = _size(engine, pop, hourly=False)
    for k in ("system_kw", "npv", "nfev", "tariff_final", "switched", "batt_kwh", "batt_kw", "payback_period",
              "first_with", "first_without", "cash_flow", "status"):
        assert np.array_equal(on[k], off[k], equal_nan=True), k
    for k in BATT:
        a, b = np.asarray(on[k], np.float64), np.asarray(off[k], np.float64)
        assert np.array_equal(a[~ts], b[~ts], equal_nan=True), k
        assert np.allclose(a[ts], b[ts], rtol=1e-9, atol=1e-9, equal_nan=True), k


def test_combined_export_plane_bit_identical(engine):
    """dgen_export_plane's combined plane summed by dgen_state_hourly
    (planes_f32 = 3) gives the three-plane form's per-state rows bit for bit."""
    from dgen_amd import _lib
    from dgen_amd.attachment import state_hourly, state_hourly_combined
    pop = _pop(700, seed=20260419)
    _, batch, out = _size(engine, pop)
    n = batch.n
    rng = np.random.default_rng(5)
    w = tuple(torch.from_numpy(rng.random(n) * 40.0).to(engine.dev) for _ in range(3))
    st = rng.integers(0, 7, n)                       # a state per device row
    idx = np.argsort(st, kind="stable").astype(np.int64)
    so = np.concatenate([[0], np.cumsum(np.bincount(st))]).astype(np.int64)
    planes = (out["baseline"], out["net_pvonly"], out["net_with_batt"])
    ref = state_hourly(engine, planes, w, idx, so)
    plane = torch.empty((_lib.NH // 4, n, 4), dtype=torch.float64, device=engine.dev)
    rest = {k: v for k, v in out.items() if k not in _lib.OUTPUT_HOURLY}
    assert engine.export_plane(batch, engine.c_outputs(rest), w, plane)
    got = state_hourly_combined(engine, plane, idx, so)
    assert torch.equal(ref, got)
