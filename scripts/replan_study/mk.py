"""Inputs for the hourly re-plan study: the first n agents
of a synthetic population in device order (64-lane waves), sized by the oracle
(daily rule), as hourly load / PV arrays plus battery bank and power.
Usage: python scripts/replan_study/mk.py N [config] [outdir]; then
gcc -O2 -o sim sim.c -lm && ./sim N [outdir]  (CPU only; test infrastructure)."""
import os
import numpy as np, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
OUT = sys.argv[3] if len(sys.argv) > 3 else '/tmp/replan_study'
os.makedirs(OUT, exist_ok=True)
from dgen_amd.synth import make_population, subset
from dgen_amd.engine import profile_order
from oracle import oracle as orc
from tests import helpers
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
cfgname = sys.argv[2] if len(sys.argv) > 2 else "res_1m_nem_tou"
pop = make_population(cfgname, 200000, seed=7)
order = profile_order(pop.cols)[:n]     # device order: first n agents (contiguous waves)
sp = subset(pop, order)
opop = helpers.oracle_population(sp.cols, pop.tariffs, pop.switches, pop.shapes, pop.cfs, pop.wholesale,
                                 demand=getattr(pop, 'demand', None))
ref = opop.run(orc.make_cfg())
cfg = orc.make_cfg()
L = np.zeros((n, 8760)); PV = np.zeros((n, 8760)); B = np.zeros(n); P = np.zeros(n)
for i, r in enumerate(ref):
    lr, cr = sp.cols["load_row"][i], sp.cols["cf_row"][i]
    ssum = orc.np_sum(pop.shapes[lr].astype(np.float64))
    ls = sp.cols["load_kwh"][i] / ssum
    kw = r["system_kw"]
    cs6 = (((kw * 1000.0) * 0.96) / 1000.0) / 1e6
    L[i] = pop.shapes[lr].astype(np.float64) * ls
    PV[i] = pop.cfs[cr].astype(np.float64) * cs6
    bank, power = orc.batt_size(kw / 0.8 / 2.0, kw / 0.8, 240.0, cfg)
    B[i] = bank; P[i] = power
for nm, a in (('load', L), ('pv', PV), ('bank', B), ('power', P)):
    a.tofile(os.path.join(OUT, nm + '.bin'))
print(n, "agents; bank mean", B.mean(), "power mean", P.mean(), "unique load rows per 64:",
      np.mean([len(set(sp.cols['load_row'][k:k+64])) for k in range(0, n, 64)]))
