#!/usr/bin/env python3
"""Diagnostic (not product): size the demand-charge parity population with the
dc_dbg variant (scripts/make_ablations.py), read back its per-evaluation
capture of agents 0-3 (kW', degradation factor, demand charge and energy bill
of every year lane) and compare each lane with the oracle's Utilityrate5
restatement at the same kW' -- energy bill and demand charge separately.
Usage: DGEN_LIB=ablate/libdgen_dc_dbg.so dbg_dc_eval.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgen_amd import _lib  # noqa: E402
from dgen_amd.config import EngineConfig  # noqa: E402
from dgen_amd.engine import Engine, outputs_to_host  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from tests.helpers import oracle_tariffs  # noqa: E402
from tests.test_gpu_demand import _pop  # noqa: E402


def main():
    pop = _pop(160, net_billing=False)
    eng = Engine(0, EngineConfig(skip_demand_charges=0))
    eng.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
    eng.set_tariffs(pop.tariffs, pop.demand)
    eng.set_switches(pop.switches)
    batch = eng.upload_agents(pop.cols, pop.n_scratch)
    out = eng.alloc_outputs(batch.n, hourly=False)
    eng.size(batch, out)
    torch.cuda.synchronize()
    o = outputs_to_host(out)
    cap = np.zeros((4, 24, 64, 6))
    L = _lib.load()
    L.dgen_debug_dcdbg.restype = ctypes.c_int32
    L.dgen_debug_dcdbg.argtypes = [ctypes.c_void_p]
    print("copy rc", L.dgen_debug_dcdbg(cap.ctypes.data), flush=True)
    np.save("gpurun_out/dc_dbg_capture.npy", cap)
    ts_dc = oracle_tariffs(pop.tariffs, pop.demand)
    t_plain = pop.tariffs.copy()
    t_plain["dc"] = 0
    ts_plain = oracle_tariffs(t_plain)
    cfg = orc.make_cfg()
    c = pop.cols
    for i in range(4):
        lr, cr, tix = int(c["load_row"][i]), int(c["cf_row"][i]), int(c["tariff0"][i])
        load = pop.shapes[lr].astype(np.float64) * (c["load_kwh"][i] / orc.np_sum(pop.shapes[lr]))
        cfk = pop.cfs[cr].astype(np.float64) / 1e6
        N = int(c["econ_life"][i])
        seg = (i % 2) * 32
        print(f"agent {i}: system_kw {o['system_kw'][i]:.6f} nfev {o['nfev'][i]} tariff {o['tariff_final'][i]} "
              f"(t0 {tix}) lanes {seg}..{seg + N - 1}")
        for e in range(24):
            r = cap[i, e, seg:seg + N]
            if not r[:, 0].any():
                break
            kws = r[0, 0]
            gen = cfk * kws
            a = orc.ur5(ts_dc[tix], cfg, gen, load, None, N, c["inflation"][i] * 100,
                        c["escalator"][i] * 100, c["pv_deg"][i] * 100)
            b = orc.ur5(ts_plain[tix], cfg, gen, load, None, N, c["inflation"][i] * 100,
                        c["escalator"][i] * 100, c["pv_deg"][i] * 100)
            rr = r[:, 5]
            o_e = b["bill_w"][1:N + 1] / rr
            o_dc = (a["bill_w"][1:N + 1] - b["bill_w"][1:N + 1]) / rr
            de = np.abs(r[:, 3] - o_e) / np.maximum(1.0, np.abs(o_e))
            dd = np.abs(r[:, 2] - o_dc) / np.maximum(1.0, np.abs(o_dc))
            print(f"  eval {e}: kw' {kws:.6f} env_ok {r[0, 4]:.0f} uniform_kws {np.ptp(r[:, 0]) == 0} "
                  f"energy max rel {de.max():.2e} dc max rel {dd.max():.2e} "
                  f"dc dev/oracle lane0 {r[0, 2]:.4f}/{o_dc[0]:.4f} lane{N - 1} {r[N - 1, 2]:.4f}/{o_dc[N - 1]:.4f}")
            if dd.max() > 1e-9:
                bad = np.nonzero(dd > 1e-9)[0]
                print("     dc mismatch lanes", bad.tolist()[:12], "s", r[bad[:4], 1].tolist())


if __name__ == "__main__":
    main()
