#!/usr/bin/env python3
"""Diagnostic: GPU vs oracle per agent on one small synthetic population,
printing the agents whose outputs differ beyond the parity tolerance and,
for the worst, the per-year bill / cash-flow differences.
usage: diag_pop.py CONFIG N [replan_hours]"""
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from dgen_amd.config import EngineConfig  # noqa: E402
from dgen_amd.engine import Engine, outputs_to_host  # noqa: E402
from dgen_amd.synth import make_population  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from tests import helpers  # noqa: E402

cfg_name, n = sys.argv[1], int(sys.argv[2])
rh = int(sys.argv[3]) if len(sys.argv) > 3 else 24
pop = make_population(cfg_name, n, n_res_shapes=64, n_com_shapes=32, n_cf=32, n_counties=16, n_tariffs=48)
eng = Engine(0, EngineConfig(batt_update_hours=rh))
eng.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
eng.set_tariffs(pop.tariffs)
eng.set_switches(pop.switches)
for order in (None,):
    batch = eng.upload_agents(pop.cols, pop.n_scratch, order=order)
    out = eng.alloc_outputs(batch.n, hourly=False)
    eng.size(batch, out)
    torch.cuda.synchronize()
    o = outputs_to_host(out, batch.perm)
opop = helpers.oracle_population(pop.cols, pop.tariffs, pop.switches, pop.shapes, pop.cfs, pop.wholesale)
ref = opop.run(orc.make_cfg(batt_update_hours=rh))
bad = []
for i, r in enumerate(ref):
    d = abs(o["npv"][i] - r["npv"]) / max(1.0, abs(r["npv"]))
    if d > 1e-7 or o["nfev"][i] != r["nfev"]:
        bad.append((d, i))
bad.sort(reverse=True)
print(f"{cfg_name} n={n} replan={rh}: {len(bad)} agents with npv rel diff > 1e-7")
for d, i in bad[:8]:
    r = ref[i]
    print(f"  agent {i}: npv rel {d:.2e} gpu {o['npv'][i]!r} orc {r['npv']!r} nfev {o['nfev'][i]}/{r['nfev']} "
          f"kw {o['system_kw'][i]!r}/{r['system_kw']!r} xlast {o['x_last'][i]!r} "
          f"w1 {o['first_with'][i]!r}/{r['first_with']!r} wo1 {o['first_without'][i]!r}/{r['first_without']!r}")
if bad:
    i = bad[0][1]
    r = ref[i]
    N1 = int(pop.cols["econ_life"][i]) + 1
    for k_o, k_r in (("bill_w_pv", "bill_w_pv_only"), ("bill_wo_pv", "bill_wo_pv_only"), ("cash_flow", "cash_flow"),
                     ("cfev_pv", "cf_energy_value_pv_only")):
        dd = o[k_o][i, :N1] - np.asarray(r[k_r])
        print(f"  {k_o}: max abs diff {np.abs(dd).max():.3e} at year {int(np.abs(dd).argmax())}; first years {dd[:4]}")
