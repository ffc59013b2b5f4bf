"""Device segmented sums (per-(state, sector) totals, per-state hourly nets)
vs numpy, and run-to-run determinism."""
import numpy as np
import pytest
import torch

from dgen_amd.dist import global_totals, group_order
from dgen_amd.engine import hourly_plane

pytestmark = pytest.mark.gpu


def test_segment_sums_f64_f32_weighted(engine):
    rng = np.random.default_rng(3)
    n, k = 5000, 7
    v1 = rng.standard_normal((k, n))
    v2 = rng.standard_normal((k, n)).astype(np.float32)
    w1 = rng.uniform(0, 3, n)
    w2 = rng.uniform(0, 3, n)
    off = np.array([0, 0, 17, 1000, 4321, 5000], dtype=np.int64)
    d = lambda a: torch.as_tensor(a, device=engine.dev)
    got = engine.segment_sums(d(v1), off).cpu().numpy()
    for s in range(len(off) - 1):
        ref = v1[:, off[s]:off[s + 1]].sum(axis=1)
        assert np.allclose(got[s], ref, rtol=1e-12, atol=1e-9)
    got2 = engine.segment_sums(d(v2), off, w1=w1, v2=d(v2), w2=w2).cpu().numpy()
    ref2 = np.stack([(v2.astype(float) * (w1 + w2))[:, off[s]:off[s + 1]].sum(axis=1)
                     for s in range(len(off) - 1)])
    assert np.allclose(got2, ref2, rtol=1e-9, atol=1e-6)
    again = engine.segment_sums(d(v1), off).cpu().numpy()
    assert np.array_equal(got, again)


def test_state_hourly_net_sums_from_sizing(engine):
    from tests import helpers
    from dgen_amd.engine import outputs_to_host
    b, cols, shapes, cfs, ws = helpers.golden_population()
    engine.load_profiles(shapes, cfs, ws)
    engine.set_tariffs(b.tariffs.array())
    engine.set_switches(b.switches.array())
    batch = engine.upload_agents(cols)
    out = engine.alloc_outputs(batch.n, hourly=True)
    engine.size(batch, out)
    torch.cuda.synchronize()
    meta, _ = helpers.golden_agents()
    states = [a["inputs"]["state_abbr"] for a in meta["agents"]]
    perm, off, uniq = group_order(states)
    n_adopt = np.linspace(0.0, 3.0, batch.n)
    n_non = 10.0 - n_adopt
    p = torch.as_tensor(perm, device=engine.dev)
    adop = hourly_plane(out["net_pvonly"]).index_select(1, p)
    base = hourly_plane(out["baseline"]).index_select(1, p)
    got = engine.segment_sums(adop, off, w1=n_adopt[perm], v2=base, w2=n_non[perm]).cpu().numpy()
    h = outputs_to_host(out)
    for s, st in enumerate(uniq):
        idx = [i for i in range(batch.n) if states[i] == st]
        ref = sum(h["net_pvonly"][i].astype(float) * n_adopt[i] + h["baseline"][i].astype(float) * n_non[i]
                  for i in idx)
        assert np.allclose(got[s], ref, rtol=1e-9, atol=1e-6), st
    tot = global_totals(engine, out, [(a["inputs"]["state_abbr"], a["inputs"]["sector_abbr"])
                                      for a in meta["agents"]],
                        sorted({(a["inputs"]["state_abbr"], a["inputs"]["sector_abbr"])
                                for a in meta["agents"]})).cpu().numpy()
    assert np.isclose(tot[:, 0].sum(), h["system_kw"].sum(), rtol=1e-12)
    assert tot[:, 3].sum() == batch.n
