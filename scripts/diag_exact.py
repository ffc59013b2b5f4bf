"""Which agents do the certified Brent paths list for the exact re-run?

Sizes a population with the fast search alone (mode 0), then subsets of it
(by billing path class, initial metering option, rate-switch candidates)
with mode 1, and prints each subset's listed count next to its Brent
evaluation counts.  Diagnostic only (GPU).

    python scripts/diag_exact.py national_mixed 20000
"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from dgen_amd.config import EngineConfig  # noqa: E402
from dgen_amd.engine import Engine, outputs_to_host, path_class  # noqa: E402
from dgen_amd.synth import make_population, subset  # noqa: E402


def size(eng, pop, mode):
    eng.set_exact(mode)
    eng.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
    eng.set_tariffs(pop.tariffs, pop.demand if not pop.skip_demand_charges else None)
    eng.set_switches(pop.switches)
    b = eng.upload_agents(pop.cols, pop.n_scratch)
    o = eng.alloc_outputs(b.n, hourly=False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    eng.size(b, o)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    return outputs_to_host(o), eng.exact_count(), dt


def main():
    cfg, n = sys.argv[1], int(sys.argv[2])
    pop = make_population(cfg, n, seed=20260000 + 5 + 211)
    eng = Engine(0, EngineConfig(skip_demand_charges=1 if pop.skip_demand_charges else 0))
    o0, _, dt0 = size(eng, pop, 0)
    o1, k1, dt1 = size(eng, pop, 1)
    print(f"{cfg} n={n}: mode 0 {dt0 * 1e3:.1f} ms, mode 1 {dt1 * 1e3:.1f} ms, listed {k1}", flush=True)
    c = pop.cols
    pc = path_class(c)
    mo = pop.tariffs["mo"][c["tariff0"]]
    sw = c["sw_solar_cnt"] > 0
    nf = o0["nfev"]
    print("nfev hist (mode 0):", dict(zip(*[a.tolist() for a in np.unique(nf, return_counts=True)])), flush=True)
    groups = {
        "class0": pc == 0, "class1": pc == 1, "class2": pc == 2,
        "class2_mo2": (pc == 2) & (mo == 2), "class2_mo0": (pc == 2) & (mo == 0),
        "switch": sw, "noswitch": ~sw, "res": (c["flags"] & 1) == 1, "com": (c["flags"] & 1) == 0,
        "nfev>=12": nf >= 12, "nfev<=8": nf <= 8,
    }
    for name, m in groups.items():
        idx = np.flatnonzero(m)
        if idx.size == 0:
            continue
        idx = idx[:4000]
        sp = subset(pop, idx)
        _, k, dt = size(eng, sp, 1)
        print(f"  {name:12s} n={idx.size:6d} listed {k:5d} ({100.0 * k / idx.size:6.2f} %) "
              f"{dt * 1e3:8.1f} ms  nfev mean {nf[idx].mean():.2f}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
