"""Device battery attachment (k_batt_attach) and per-state hourly export
(k_export_weights + k_state_hourly) through the drop-in functions, against the
reference's own outputs (tests/golden/attach.json) and, at larger sizes,
against the oracle restatement (oracle/attach.py).

Tolerances: integer allocation bit-exact; capacities (a * kW products)
bit-exact; the hourly state sums within 1e-12 relative (the reference adds
agents sequentially in iterrows order, the device in a fixed tree)."""
import numpy as np
import pandas as pd
import pytest
import torch

from dgen_amd import attachment as ga
from dgen_amd.engine import tile_hourly
from oracle import attach as oa
from tests.helpers import golden_attach

pytestmark = pytest.mark.gpu

CASES = [c["name"] for c in golden_attach()[0]["cases"]]


def _frame(c, hourly=None):
    df = pd.DataFrame(c["inputs"])
    df = df.set_index("agent_id", drop=False)
    if hourly is not None:
        base, pvo, wbt = hourly
        df["baseline_net_hourly"] = list(base)
        df["adopter_net_hourly_pvonly"] = list(pvo)
        df["adopter_net_hourly_with_batt"] = list(wbt)
    return df


@pytest.mark.parametrize("name", CASES)
def test_allocation_device_matches_reference(engine, name):
    meta, _ = golden_attach()
    c = next(c for c in meta["cases"] if c["name"] == name)
    out = ga._allocate_battery_adopters_integer(_frame(c), 2027, engine=engine)
    for k, v in c["alloc"].items():
        assert np.array_equal(out[k].to_numpy(), np.asarray(v)), k
    assert out["batt_adopters_added_this_year"].dtype.kind == "i"


@pytest.mark.parametrize("name", CASES)
def test_state_export_device_matches_reference(engine, name):
    meta, hourly = golden_attach()
    c = next(c for c in meta["cases"] if c["name"] == name)
    df = _frame(c, hourly[name])
    df = ga._allocate_battery_adopters_integer(df, 2027, engine=engine)
    seen = []
    rec = ga.export_state_hourly_with_storage_mix("eng", "s", "o", 2027, df,
                                                  writer=lambda r, *a, **k: seen.append((r, a, k)),
                                                  dev_engine=engine)
    assert rec["state_abbr"].tolist() == c["export"]["state_abbr"]
    assert rec["n_hours"].tolist() == c["export"]["n_hours"]
    for a, b in zip(rec["net_sum"], c["export"]["net_sum"]):
        assert np.allclose(np.asarray(a), np.asarray(b), rtol=1e-12, atol=1e-12)
    assert seen and seen[0][1][3] == "state_hourly_agg" and seen[0][2]["if_exists"] == "append"


def _population(rng, n, n_states=9, n_sec=3, ties=False):
    st = rng.integers(0, n_states, n)
    sec = rng.integers(0, n_sec, n)
    new = rng.uniform(0, 4, n) * (rng.random(n) < 0.8)
    if ties:
        new[::3] = 2.5
    ids = rng.permutation(n * 3)[:n]
    rate = rng.uniform(0, 0.7, n_states)
    rate[0] = 0.0
    bkw = np.where(rng.random(n) < 0.1, 0.0, rng.uniform(2, 40, n))
    prev = np.maximum(np.round(rng.uniform(0, 6, n)) * bkw + rng.uniform(-0.3, 0.3, n) * (bkw > 0), 0)
    return dict(state=[f"S{s}" for s in st], sector=[f"c{s}" for s in sec], agent_id=ids,
                new_adopters=new, rate=rate[st], batt_kw=bkw, batt_kwh=bkw * 2.0,
                batt_kw_cum_last_year=prev, batt_kwh_cum_last_year=prev * 2.0,
                customers=new + rng.uniform(0, 300, n), adopters=new + rng.uniform(0, 40, n))


@pytest.mark.parametrize("n,ties", [(20000, False), (60000, True)])
def test_allocation_large_vs_oracle(engine, n, ties):
    p = _population(np.random.default_rng(n), n, ties=ties)
    args = (p["state"], p["sector"], p["agent_id"], p["new_adopters"], p["rate"], p["batt_kw"],
            p["batt_kwh"], p["batt_kw_cum_last_year"], p["batt_kwh_cum_last_year"])
    got = ga.allocate_arrays(engine, *args)
    ref = oa.allocate(*args)
    assert np.array_equal(got["added"], ref["batt_adopters_added_this_year"])
    for k in ("new_batt_kw", "new_batt_kwh", "batt_kw_cum", "batt_kwh_cum"):
        assert np.array_equal(got[k], ref[k]), k
    # property: each group's total is round(r * sum(new)) when r > 0 and sum > 0
    assert got["added"].sum() > 0


def test_allocation_edges(engine):
    # empty frame, a single agent, all-zero adopters, rate > 1 clamps, NaN state dropped
    e = ga.allocate_arrays(engine, [], [], [], [], [], [], [], [], [])
    assert all(len(v) == 0 for v in e.values())
    one = ga.allocate_arrays(engine, ["A"], ["res"], [7], [2.6], [1.5], [5.0], [10.0], [1.0], [2.0])
    assert one["added"].tolist() == [3] and one["batt_kw_cum"].tolist() == [16.0]
    z = ga.allocate_arrays(engine, ["A", "A"], ["r", "r"], [1, 2], [0.0, 0.0], [0.5, 0.5],
                           [1.0, 1.0], [2.0, 2.0], [0.0, 0.0], [0.0, 0.0])
    assert z["added"].tolist() == [0, 0]
    nan_st = ga.allocate_arrays(engine, [float("nan"), "B"], ["r", "r"], [1, 2], [3.0, 3.0],
                                [1.0, 1.0], [1.0, 1.0], [2.0, 2.0], [0.0, 0.0], [0.0, 0.0])
    assert nan_st["added"].tolist() == [0, 3]


def test_state_hourly_from_sizing_planes(engine):
    """Export straight from the sizing kernels' device planes (device order)
    vs the oracle export on the host copies of the same planes."""
    from tests import helpers
    from dgen_amd.engine import outputs_to_host, profile_order
    b, cols, shapes, cfs, ws = helpers.golden_population()
    engine.load_profiles(shapes, cfs, ws)
    engine.set_tariffs(b.tariffs.array())
    engine.set_switches(b.switches.array())
    batch = engine.upload_agents(cols, order=profile_order(cols))
    out = engine.alloc_outputs(batch.n, hourly=True)
    engine.size(batch, out)
    torch.cuda.synchronize()
    h = outputs_to_host(out, batch.perm)
    n = batch.n
    meta, _ = helpers.golden_agents()
    states = [a["inputs"]["state_abbr"] for a in meta["agents"]]
    rng = np.random.default_rng(5)
    cust = rng.uniform(5, 50, n)
    adopt = rng.uniform(0, 5, n)
    added = rng.integers(0, 3, n)
    bkw_ly = np.round(rng.uniform(0, 4, n)) * h["batt_kw"]
    got, keys = ga.state_hourly_from_outputs(engine, out, batch.perm, states, cust, adopt, bkw_ly,
                                             h["batt_kw"], added)
    got = got.cpu().numpy()
    w = oa.weights(cust, adopt, bkw_ly, h["batt_kw"], added)
    ref = oa.export(states, h["baseline"].astype(np.float64), h["net_pvonly"].astype(np.float64),
                    h["net_with_batt"].astype(np.float64), w)
    assert keys == ref["state_abbr"]
    for s in range(len(keys)):
        assert np.allclose(got[s], ref["net_sum"][s], rtol=1e-12, atol=1e-12), keys[s]
    again, _ = ga.state_hourly_from_outputs(engine, out, batch.perm, states, cust, adopt, bkw_ly,
                                            h["batt_kw"], added)
    assert np.array_equal(got, again.cpu().numpy())


def test_state_hourly_full_size(engine):
    """8760-h planes, 40k agents over 51 states: device vs float64 numpy."""
    rng = np.random.default_rng(11)
    n, nh, S = 40000, 8760, 51
    st = np.sort(rng.integers(0, S, n))
    so = np.searchsorted(st, np.arange(S + 1)).astype(np.int64)
    planes = [torch.rand((nh, n), dtype=torch.float32, device=engine.dev) for _ in range(3)]
    wts = [torch.as_tensor(rng.integers(0, 20, n).astype(np.float64), device=engine.dev)
           for _ in range(2)] + [torch.as_tensor(rng.uniform(0, 100, n), device=engine.dev)]
    # f32 planes are read in the sizing outputs' hour-quad tiles
    got = ga.state_hourly(engine, [tile_hourly(p) for p in planes], wts, None, so)
    P = [p.double() for p in planes]
    contrib = P[1] * wts[0] + P[2] * wts[1] + P[0] * wts[2]              # [nh, n]
    ref = torch.stack([contrib[:, so[s]:so[s + 1]].sum(dim=1) for s in range(S)]) / 1000.0
    assert torch.allclose(got, ref, rtol=1e-11, atol=1e-9)
