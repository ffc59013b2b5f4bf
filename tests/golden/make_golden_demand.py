#!/usr/bin/env python3
"""Generate tests/golden/tariffs_dc.json: the reference's normalize_tariff +
process_tariff outputs for tariffs WITH demand charges, captured with the
reference's module switch flipped (financial_functions.SKIP_DEMAND_CHARGES =
False), so the demand branch of process_tariff (ff:604-615) runs.

Same harness as make_golden.py (the reference's own Python imported in this
container with stub modules for the DB / cloud / colour packages and a fake
PySAM that records the ElectricityRates field writes).  Run from the repo root:
    python tests/golden/make_golden_demand.py
Only the compile is pinned by this: the SSC demand-charge arithmetic has no
reference-side fixture (parity unpinned).
"""
import json
import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import make_golden as mg  # noqa: E402


def sched(on_start, on_end, base, on):
    return [[on if on_start <= h < on_end else base for h in range(24)] for _ in range(12)]


def demand_cases(rng):
    e = {"e_prices": [[0.11, 0.24]], "e_wkday_12by24": sched(14, 20, 0, 1),
         "e_wkend_12by24": sched(0, 0, 0, 1), "fixed_charge": 20.0}
    cases = []
    cases.append(("dc_flat_ur", dict(e, ur_dc_flat_mat=[[m, 1, 1e38, 9.5 + m * 0.25] for m in range(12)])))
    cases.append(("dc_tou_ur", dict(e, ur_dc_tou_mat=[[1, 1, 50, 4.0], [1, 2, 1e38, 6.5],
                                                       [2, 1, 50, 11.0], [2, 2, 1e38, 14.25]],
                                    ur_dc_sched_weekday=sched(12, 19, 1, 2),
                                    ur_dc_sched_weekend=sched(0, 0, 1, 2))))
    cases.append(("dc_both_ur", dict(e, ur_dc_flat_mat=[[m, 1, 100, 5.0] for m in range(12)]
                                     + [[m, 2, 1e38, 7.0] for m in range(12)],
                                     ur_dc_tou_mat=[[1, 1, 1e38, 0.0], [2, 1, 1e38, 8.0],
                                                    [3, 1, 1e38, 13.0]],
                                     ur_dc_sched_weekday=[[1 if h < 8 else (3 if 15 <= h < 20 else 2)
                                                           for h in range(24)]] * 12,
                                     ur_dc_sched_weekend=sched(0, 0, 1, 1))))
    cases.append(("dc_legacy_tou", dict(e, d_tou_levels=[[1e9, 1e9]], d_tou_prices=[[3.0, 12.0]],
                                        d_wkday_12by24=sched(13, 19, 0, 1),
                                        d_wkend_12by24=sched(0, 0, 0, 0), d_tou_exists=True)))
    cases.append(("dc_legacy_flat_12", dict(e, d_flat_levels=[[1e9] * 12],
                                            d_flat_prices=[[5.0 + 0.5 * m for m in range(12)]],
                                            d_flat_exists=True)))
    cases.append(("dc_flag_only", dict(e, d_flat_exists=True)))
    cases.append(("dc_enable_zero", dict(e, ur_dc_enable=0, ur_dc_tou_mat=[[1, 1, 1e38, 4.0]])))
    cases.append(("dc_nonfinite", dict(e, ur_dc_tou_mat=[[1, 1, float("nan"), 4.0]],
                                       ur_dc_sched_weekday=sched(0, 0, 1, 1))))
    cases.append(("dc_tier_gap", dict(e, ur_dc_tou_mat=[[1, 1, 20, 4.0], [1, 3, 1e38, 6.0]],
                                      ur_dc_sched_weekday=sched(0, 0, 1, 1),
                                      ur_dc_sched_weekend=sched(0, 0, 1, 1))))
    cases.append(("dc_period9", dict(e, ur_dc_tou_mat=[[9, 1, 1e38, 4.0]],
                                     ur_dc_sched_weekday=sched(0, 0, 9, 9),
                                     ur_dc_sched_weekend=sched(0, 0, 9, 9))))
    cases.append(("dc_ragged_sched", dict(e, ur_dc_tou_mat=[[1, 1, 1e38, 4.0], [2, 1, 1e38, 9.0]],
                                          ur_dc_sched_weekday=[[2] * 20] * 10)))
    cases.append(("dc_str_form", str(dict(e, ur_dc_tou_mat=[[1, 1, 1e38, 2.5], [2, 1, 1e38, 7.75]],
                                          ur_dc_sched_weekday=sched(16, 21, 1, 2),
                                          ur_dc_sched_weekend=sched(0, 0, 1, 1)))))
    cases.append(("dc_mo2", dict(e, ur_metering_option=2,
                                 ur_dc_flat_mat=[[m, 1, 1e38, 8.0] for m in range(12)])))
    for k in range(12):
        P = int(rng.integers(1, 5))
        T = int(rng.integers(1, 3))
        rows = []
        for p in range(P):
            for t in range(T):
                cap = 1e38 if t == T - 1 else float(rng.choice([20, 50, 100, 250]))
                rows.append([p + 1, t + 1, cap, float(np.round(rng.uniform(1, 20), 3))])
        d = dict(e, ur_dc_tou_mat=rows,
                 ur_dc_sched_weekday=(rng.integers(0, P, size=(12, 24)) + 1).tolist(),
                 ur_dc_sched_weekend=(rng.integers(0, P, size=(12, 24)) + 1).tolist())
        if k % 3 == 0:
            d["ur_dc_flat_mat"] = [[m, 1, 1e38, float(np.round(rng.uniform(2, 15), 2))] for m in range(12)]
        cases.append((f"dc_rand{k:02d}", d))
    return cases


def main():
    warnings.filterwarnings("ignore")
    ff, _ = mg.install_stubs()
    ff.SKIP_DEMAND_CHARGES = False          # the extension mode's switch (ff:35)
    out = []
    for name, raw in demand_cases(np.random.default_rng(20260005)):
        td = ff.normalize_tariff(raw, net_sell_rate_scalar=0.0)
        u = mg.FakeUtilityrate()
        ff.process_tariff(u, td, 0.0, ts_sell_rate=None)
        out.append({"name": name, "raw": raw, "normalized": td, "process": mg.er_fields(u)})
    with open(os.path.join(HERE, "tariffs_dc.json"), "w") as f:
        json.dump(mg._jsonable(out), f)
    print(f"tariffs_dc={len(out)}")


if __name__ == "__main__":
    main()
