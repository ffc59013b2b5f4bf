#!/usr/bin/env python3
"""Diagnostic (not product): size the demand-charge parity population with
the library named by DGEN_LIB and check the LAST evaluation's per-year outputs
(bill_w_pv / bill_wo_pv / cfev_pv at x_last) of agents 0-5 against the
oracle's Utilityrate5 restatement at the same kW -- no instrumentation in the
kernel, so the build under test is the unmodified one."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
    ts_dc = oracle_tariffs(pop.tariffs, pop.demand)
    cfg = orc.make_cfg()
    c = pop.cols
    for i in range(6):
        lr, cr, tix = int(c["load_row"][i]), int(c["cf_row"][i]), int(o["tariff_final"][i])
        load = pop.shapes[lr].astype(np.float64) * (c["load_kwh"][i] / orc.np_sum(pop.shapes[lr]))
        N = int(c["econ_life"][i])
        x = float(o["x_last"][i])
        kws = ((x * 1000.0) * 0.96) / 1000.0
        gen = pop.cfs[cr].astype(np.float64) / 1e6 * kws
        a = orc.ur5(ts_dc[tix], cfg, gen, load, None, N, c["inflation"][i] * 100,
                    c["escalator"][i] * 100, c["pv_deg"][i] * 100)
        bw, bwo, ev = o["bill_w_pv"][i, 1:N + 1], o["bill_wo_pv"][i, 1:N + 1], o["cfev_pv"][i, 1:N + 1]
        rel = lambda p, q: float(np.max(np.abs(p - q) / np.maximum(1.0, np.abs(q))))
        print(f"agent {i}: kw {o['system_kw'][i]:.6f} x_last {x:.6f} nfev {o['nfev'][i]} npv {o['npv'][i]:.3f}")
        print(f"   bill_w rel {rel(bw, a['bill_w'][1:N + 1]):.2e} (dev {bw[0]:.4f} / orc {a['bill_w'][1]:.4f}; "
              f"y{N} {bw[-1]:.4f} / {a['bill_w'][N]:.4f})")
        print(f"   bill_wo rel {rel(bwo, a['bill_wo'][1:N + 1]):.2e} ev rel {rel(ev, a['aev'][1:N + 1]):.2e}")
        total = ((c["capex"][i] * x + 0.0) * c["ccm"][i]) + 0.0
        li = orc.LoanIn(nyears=N, market=0 if (c["flags"][i] & 1) else 1, loan_term=int(c["loan_term"][i]),
                        depr_fed_type=0 if (c["flags"][i] & 1) else 2,
                        depr_sta_type=0 if (c["flags"][i] & 1) else 2, pad=0,
                        debt_fraction_pct=100.0 - (c["down_payment"][i] * 100.0),
                        fed_tax_pct=(c["tax_rate"][i] * 100.0) * 0.7, sta_tax_pct=(c["tax_rate"][i] * 100.0) * 0.3,
                        real_disc_pct=c["real_discount"][i] * 100.0, inflation_pct=c["inflation"][i] * 100.0,
                        itc_fed_pct=c["itc_frac"][i], total_cost=total)
        cl = orc.cashloan(li, cfg, a["aev"])
        cf = o["cash_flow"][i, :N + 1]
        print(f"   npv dev {o['npv'][i]:.4f} orc {cl['npv']:.4f}; cash_flow[0] dev {cf[0]:.4f} orc {-total:.4f}; "
              f"cf_payback rel {rel(cf[1:], cl['cf_payback'][1:N + 1]):.2e}")
        d = np.nonzero(np.abs(cf[1:] - cl['cf_payback'][1:N + 1]) > 1e-6 * np.maximum(1, np.abs(cf[1:])))[0]
        if d.size:
            print("   cf_payback differs in years", (d + 1).tolist()[:30])
            print("     dev", np.round(cf[1:][d[:6]], 3).tolist(), "\n     orc", np.round(cl['cf_payback'][1:N + 1][d[:6]], 3).tolist())
        print("   dev bill_w first 6:", np.round(bw[:6], 4).tolist())
        print("   orc bill_w first 6:", np.round(a["bill_w"][1:7], 4).tolist())


if __name__ == "__main__":
    main()
