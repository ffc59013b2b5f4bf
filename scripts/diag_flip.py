#!/usr/bin/env python3
"""Diagnostic (not product): the Brent path of chosen agents of a demand-charge
population on the device (DGEN_LIB=ablate/libdgen_btrace.so, the k_size
evaluation trace) against the oracle's (oracle.brent_trace), evaluation by
evaluation: kW, -NPV, and which device forms the evaluation used (net-billing
split, demand envelope / staged).  Usage:
  DGEN_LIB=ablate/libdgen_btrace.so diag_flip.py CONFIG N SEED SAMPLE_SEED POS[,POS...] [alone]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgen_amd.config import EngineConfig  # noqa: E402
from dgen_amd.engine import Engine  # noqa: E402
from dgen_amd.synth import make_population, subset  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from tests import helpers  # noqa: E402


def main():
    cfg_name, n, seed, sseed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    pos = [int(p) for p in sys.argv[5].split(",")]
    alone = len(sys.argv) > 6 and sys.argv[6] == "alone"
    pop = make_population(cfg_name, n, seed=seed)
    idx = np.sort(np.random.default_rng(sseed).choice(n, 150, replace=False)) if n > 150 else np.arange(n)
    eng = Engine(0, EngineConfig(skip_demand_charges=0))
    L = eng.lib
    L.dgen_bt_set.argtypes = [ctypes.c_longlong]
    L.dgen_bt_read.argtypes = [ctypes.c_void_p]
    eng.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
    eng.set_tariffs(pop.tariffs, pop.demand)
    eng.set_switches(pop.switches)
    for p in pos:
        a = int(idx[p])
        P = subset(pop, [a]) if alone else pop
        dev_i = 0 if alone else a
        batch = eng.upload_agents(P.cols, P.n_scratch)
        out = eng.alloc_outputs(len(P.cols["load_kwh"]), hourly=True)
        L.dgen_bt_set(dev_i)
        eng.size(batch, out)
        torch.cuda.synchronize()
        buf = np.zeros(256)
        k = L.dgen_bt_read(buf.ctypes.data)
        dtr = buf[:4 * min(k, 64)].reshape(-1, 4)
        o = {c: out[c][dev_i].item() for c in ("system_kw", "nfev", "npv", "x_last", "status")}
        del out, batch
        torch.cuda.empty_cache()
        sub = subset(pop, [a])
        opop = helpers.oracle_population(sub.cols, pop.tariffs, pop.switches, pop.shapes, pop.cfs,
                                         pop.wholesale, demand=pop.demand)
        otr, res = orc.brent_trace(opop, orc.make_cfg(), 0)
        r = res[0]
        print(f"== pos {p} agent {a} {'alone' if alone else 'in batch'}: device nfev {o['nfev']} kw {o['system_kw']!r} "
              f"npv {o['npv']!r} | oracle nfev {r['nfev']} kw {r['system_kw']!r} npv {r['npv']!r}", flush=True)
        print(f"   tariff0 {int(sub.cols['tariff0'][0])} mo {int(pop.tariffs['mo'][sub.cols['tariff0'][0]])} "
              f"slot {int(sub.cols['scratch_slot'][0])}", flush=True)
        for j in range(max(len(dtr), len(otr))):
            d = dtr[j] if j < len(dtr) else [np.nan] * 4
            q = otr[j] if j < len(otr) else [np.nan] * 2
            rel = abs(d[1] - q[1]) / max(abs(q[1]), 1e-300) if j < len(otr) and j < len(dtr) else np.nan
            print(f"   {j:2d} dev x={d[0]!r:>22} f={d[1]!r:>24} nb={int(d[2]) if d[2]==d[2] else -1} "
                  f"env={int(d[3]) if d[3]==d[3] else -1} | orc x={q[0]!r:>22} f={q[1]!r:>24} rel={rel:.3e}",
                  flush=True)


if __name__ == "__main__":
    main()
