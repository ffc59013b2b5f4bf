"""Generate the committed golden fixtures under tests/golden/.

Run IN THE BUILD CONTAINER ONLY (it reads /root/reference, which does not exist
on the GPU box):  python tests/golden/make_golden.py

What it does
------------
* Imports the reference's own Python hot path (financial_functions.py,
  agent_mutation/elec.py) with sys.modules stubs for the DB / cloud / colour
  packages it imports but does not use on this path.
* Replaces PySAM (nrel-pysam==7.1.0, absent here) by fake modules that record
  every field write and whose execute() calls the CPU oracle primitives
  (oracle/orc.c).  The reference's driver therefore runs unmodified: bracket and
  xatol (ff:440-444), scipy's bounded Brent (ff:445-447), rate-switch
  stickiness (elec.py:838-863), last-evaluation capture (ff:449-474),
  naep mixing (ff:543-544), payback rounding (ff:557) and the tariff compile
  (ff:575-1007) are the reference's code.  Only the SSC arithmetic is the
  oracle's restatement (parity unpinned).
* Writes:
    tariffs.json  normalize_tariff + process_tariff outputs (bit-exact targets)
    brent.json    scipy x-sequences / res.x / nfev on closed-form objectives
    agents.json + agents.npz   full boundary captures (inputs + output row)
"""
from __future__ import annotations

import json
import os
import sys
import types
import warnings
from unittest.mock import MagicMock

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/dgen_os/python"
sys.path.insert(0, REPO)

from oracle import oracle as orc  # noqa: E402

NH = 8760
CFG = orc.make_cfg()


# ----------------------------------------------------------------------------
# fake PySAM
# ----------------------------------------------------------------------------
class Group:
    def __init__(self, owner, name):
        object.__setattr__(self, "_owner", owner)
        object.__setattr__(self, "_name", name)
        object.__setattr__(self, "_vals", {})

    def __setattr__(self, k, v):
        self._vals[k] = v
        self._owner._log.append((self._name, k))

    def __getattr__(self, k):
        vals = object.__getattribute__(self, "_vals")
        if k in vals:
            return vals[k]
        raise AttributeError(k)

    def export(self):
        return dict(self._vals)


class Module:
    groups: tuple = ()

    def __init__(self):
        object.__setattr__(self, "_log", [])
        for g in self.groups:
            object.__setattr__(self, g, Group(self, g))


class FakeUtilityrate(Module):
    groups = ("Lifetime", "SystemOutput", "ElectricityRates", "Load", "Outputs")

    def execute(self):
        ER, L, SO = self.ElectricityRates, self.Lifetime, self.SystemOutput
        mat = getattr(ER, "ur_ec_tou_mat", [])
        t = orc.tariff_from_fields(mat, ER.ur_metering_option, ER.ur_monthly_fixed_charge,
                                   ER.ur_ec_sched_weekday, ER.ur_ec_sched_weekend)
        ts = None
        if int(getattr(ER, "ur_en_ts_sell_rate", 0)) == 1:
            ts = np.asarray(ER.ur_ts_sell_rate, dtype=np.float64)
        out = orc.ur5(t, CFG, np.asarray(SO.gen, dtype=float), np.asarray(self.Load.load, dtype=float),
                      ts, int(L.analysis_period), float(L.inflation_rate),
                      float(ER.rate_escalation[0]), float(SO.degradation[0]))
        O = self.Outputs
        O.annual_energy_value = out["aev"].tolist()
        O.utility_bill_w_sys = out["bill_w"].tolist()
        O.utility_bill_wo_sys = out["bill_wo"].tolist()
        O.utility_bill_w_sys_year1 = float(out["bill_w"][1])
        O.utility_bill_wo_sys_year1 = float(out["bill_wo"][1])
        O.year1_hourly_e_fromgrid = out["e_fromgrid"].tolist()


class FakeCashloan(Module):
    groups = ("FinancialParameters", "SystemCosts", "BatterySystem", "LCOS", "SystemOutput",
              "TaxCreditIncentives", "Depreciation", "Outputs")

    def execute(self):
        FP = self.FinancialParameters
        li = orc.LoanIn(
            nyears=int(FP.analysis_period), market=int(FP.market), loan_term=int(FP.loan_term),
            depr_fed_type=int(self.Depreciation.depr_fed_type),
            depr_sta_type=int(self.Depreciation.depr_sta_type), pad=0,
            debt_fraction_pct=float(FP.debt_fraction), fed_tax_pct=float(FP.federal_tax_rate[0]),
            sta_tax_pct=float(FP.state_tax_rate[0]), real_disc_pct=float(FP.real_discount_rate),
            inflation_pct=float(FP.inflation_rate),
            itc_fed_pct=float(self.TaxCreditIncentives.itc_fed_percent[0]),
            total_cost=float(self.SystemCosts.total_installed_cost))
        out = orc.cashloan(li, CFG, np.asarray(self.SystemOutput.annual_energy_value, dtype=float))
        O = self.Outputs
        O.npv = out["npv"]
        O.payback = out["payback"]
        O.cf_payback_with_expenses = out["cf_payback"].tolist()
        O.cf_energy_value = out["cf_energy_value"].tolist()


class FakeBattery(Module):
    groups = ("BatterySystem", "BatteryCell", "Lifetime", "Load", "SystemOutput",
              "BatteryDispatch", "Outputs")

    def execute(self):
        BS = self.BatterySystem
        bank = float(BS.batt_computed_bank_capacity)
        power = float(BS.batt_power_discharge_max_kwdc)
        sg, g2l = orc.batt_dispatch(np.asarray(self.Load.load, float),
                                    np.asarray(self.SystemOutput.gen, float), bank, power, CFG)
        self.SystemOutput.gen = sg.tolist()
        O = self.Outputs
        O.grid_to_load = g2l.tolist()
        O.batt_bank_installed_capacity = bank
        O.batt_bank_replacement = [0.0]


def battery_model_sizing(model, desired_power, desired_capacity, desired_voltage=500, tol=None,
                         **_):
    bank, power = orc.batt_size(desired_power, desired_capacity, desired_voltage, CFG)
    BS = model.BatterySystem
    BS.batt_computed_bank_capacity = bank
    BS.batt_power_discharge_max_kwdc = power
    BS.batt_power_charge_max_kwdc = power


def _no_default(*a, **k):
    raise RuntimeError("PySAM default configs are unavailable offline")


def install_stubs():
    for m in ["google", "google.cloud", "google.cloud.sql", "google.cloud.sql.connector",
              "colorama", "colorlog", "pg8000", "pg8000.native", "psycopg2", "psycopg2.extras",
              "psycopg2.extensions", "openpyxl"]:
        sys.modules[m] = MagicMock()
    pysam = types.ModuleType("PySAM")
    sys.modules["PySAM"] = pysam
    mods = {}
    for sub in ["Battery", "BatteryTools", "Utilityrate5", "Cashloan", "CustomGeneration",
                "Pvsamv1", "Pvwattsv8"]:
        mod = types.ModuleType("PySAM." + sub)
        sys.modules["PySAM." + sub] = mod
        setattr(pysam, sub, mod)
        mods[sub] = mod
        mod.default = _no_default
        mod.from_existing = _no_default
    mods["Battery"].new = FakeBattery
    mods["Utilityrate5"].new = FakeUtilityrate
    mods["Cashloan"].new = FakeCashloan
    mods["BatteryTools"].battery_model_sizing = battery_model_sizing
    sys.path.insert(0, REF)
    import financial_functions as ff  # noqa
    import agent_mutation.elec as elec  # noqa
    return ff, elec


# ----------------------------------------------------------------------------
# synthetic profiles (same generator family as dgen_amd.synth, small)
# ----------------------------------------------------------------------------
def make_profiles(rng):
    hours = np.arange(NH)
    hod = hours % 24
    doy = hours // 24
    shapes = []
    for k in range(5):
        diurnal = 1.0 + 0.6 * np.sin((hod - 7 - k) / 24 * 2 * np.pi) ** 2 + 0.3 * (hod >= 17) * (hod <= 21)
        seasonal = 1.0 + 0.35 * np.cos((doy - 200 + 15 * k) / 365 * 2 * np.pi)
        noise = rng.lognormal(0.0, 0.25, NH)
        x = diurnal * seasonal * noise
        shapes.append((x / x.sum()).astype(np.float32))
    cfs = []
    for k in range(5):
        sun = np.clip(np.sin((hod - 6 + 0.3 * k) / 13 * np.pi), 0, None) * (hod >= 6) * (hod <= 19)
        season = 0.75 + 0.25 * np.cos((doy - 172) / 365 * 2 * np.pi)
        cloud = np.clip(rng.normal(0.85, 0.2, NH), 0.05, 1.0)
        cf = sun * season * cloud
        target = 1250 + 150 * k
        cf = cf * (target / cf.sum())
        cfs.append(np.round(np.clip(cf, 0, 1) * 1e6).astype(np.int32))
    ws = []
    for k in range(3):
        w = 0.03 + 0.015 * np.sin((hod - 14) / 24 * 2 * np.pi) + rng.normal(0, 0.004, NH)
        ws.append(np.clip(w, 0.005, None))
    ws[2] = ws[2].copy()
    ws[2][100] = np.nan            # non-finite series -> TS sell disabled (ff:759)
    return np.stack(shapes), np.stack(cfs), np.stack(ws)


# ----------------------------------------------------------------------------
# tariff cases
# ----------------------------------------------------------------------------
def sched_tou(on_start, on_end, base=0, on=1):
    return [[on if on_start <= h < on_end else base for h in range(24)] for _ in range(12)]


def tariff_cases(rng):
    cases = []
    # Appendix C known answers
    cases.append(("K1", {"e_prices": [[0.12, 0.28]], "e_wkday_12by24": sched_tou(16, 21),
                         "e_wkend_12by24": sched_tou(0, 0), "fixed_charge": 10}))
    cases.append(("K2", {"e_prices": [[0.10, 0.20], [0.15, 0.25]],
                         "e_levels": [[500, 600], [1e9, 1e9]],
                         "e_wkday_12by24": sched_tou(12, 24), "e_wkend_12by24": sched_tou(0, 0)}))
    cases.append(("K3", {"ur_ec_tou_mat": [[1, 1, 300, 0, 0.11, 0], [1, 2, 1e38, 0, 0.14, 0],
                                           [3, 1, 1e38, 0, 0.31, 0]],
                         "ur_ec_sched_weekday": [[3 if 14 <= h < 20 else 1 for h in range(24)]
                                                 for _ in range(12)],
                         "ur_ec_sched_weekend": [[1] * 24 for _ in range(12)],
                         "ur_monthly_fixed_charge": 7.5}))
    cases.append(("K4", "{'e_prices': [[0.2]], 'fixed_charge': nan, 'energy_rate_unit': 'kWh'}"))
    cases.append(("K5", {"e_prices": [[0.1]], "d_flat_prices": [[5.0] * 12],
                         "d_flat_levels": [[1e9] * 12], "d_flat_exists": True}))
    cases.append(("mo2_tou", {"e_prices": [[0.11, 0.31]], "e_wkday_12by24": sched_tou(15, 20),
                              "e_wkend_12by24": sched_tou(0, 0), "fixed_charge": 12.0,
                              "ur_metering_option": 2}))
    cases.append(("daily_unit", {"e_prices": [[0.09, 0.19], [0.13, 0.23]],
                                 "e_levels": [[20, 20], [1e9, 1e9]], "energy_rate_unit": "kWh daily",
                                 "e_wkday_12by24": sched_tou(8, 20), "e_wkend_12by24": sched_tou(0, 0)}))
    cases.append(("tier3_tou2", {"ur_ec_tou_mat": [[1, 1, 350, 0, 0.10, 0.02], [1, 2, 800, 0, 0.14, 0.02],
                                                   [1, 3, 1e38, 0, 0.21, 0.02], [2, 1, 400, 0, 0.16, 0.03],
                                                   [2, 2, 700, 0, 0.22, 0.03], [2, 3, 1e38, 0, 0.30, 0.03]],
                                 "ur_ec_sched_weekday": sched_tou(13, 19, 1, 2),
                                 "ur_ec_sched_weekend": sched_tou(0, 0, 1, 2),
                                 "ur_monthly_fixed_charge": 9.0, "ur_metering_option": 0}))
    cases.append(("empty_dict", {}))
    cases.append(("json_str", json.dumps({"e_prices": [[0.17, 0.23, 0.41]],
                                          "e_wkday_12by24": [[(h // 8) for h in range(24)]] * 12,
                                          "e_wkend_12by24": [[0] * 24] * 12,
                                          "fixed_charge": "12.5"})))
    cases.append(("mismatched_levels", {"e_prices": [[0.1, 0.2]], "e_levels": [[100]],
                                        "e_wkday_12by24": sched_tou(10, 14)}))
    cases.append(("ragged_sched", {"e_prices": [[0.1, 0.2]], "e_wkday_12by24": [[1] * 10] * 6}))
    # kWh/kW tier units (ff:778-779): caps x the month's peak import (x days for 3)
    cases.append(("kwkw_unit", {"e_prices": [[0.11, 0.24], [0.17, 0.33]], "e_levels": [[180, 180], [1e9, 1e9]],
                                "energy_rate_unit": "kWh/kW", "e_wkday_12by24": sched_tou(14, 19),
                                "e_wkend_12by24": sched_tou(0, 0), "fixed_charge": 30.0}))
    cases.append(("kwkw_daily_nb", {"ur_ec_tou_mat": [[1, 1, 6.0, 3, 0.12, 0.04], [1, 2, 1e38, 3, 0.19, 0.04],
                                                      [2, 1, 6.0, 3, 0.21, 0.05], [2, 2, 1e38, 3, 0.29, 0.05]],
                                    "ur_ec_sched_weekday": sched_tou(16, 21, 1, 2),
                                    "ur_ec_sched_weekend": sched_tou(0, 0, 1, 2),
                                    "ur_monthly_fixed_charge": 15.0, "ur_metering_option": 2}))
    cases.append(("unit_mode", {"ur_ec_tou_mat": [[1, 1, 1e38, 2, 0.1, 0], [2, 1, 1e38, 0, 0.2, 0],
                                                  [3, 1, 1e38, 0, 0.3, 0]],
                                "ur_ec_sched_weekday": sched_tou(9, 17, 1, 3),
                                "ur_ec_sched_weekend": sched_tou(0, 0, 1, 2)}))
    # random legacy / ur_* mixes (P 1..4, T 1..3, prices U[0.06,0.40], fixed U[0,25])
    for k in range(36):
        P = int(rng.integers(1, 5))
        T = int(rng.integers(1, 4))
        prices = np.round(rng.uniform(0.06, 0.40, size=(T, P)), 5)
        prices = np.sort(prices, axis=0)
        fixed = float(np.round(rng.uniform(0, 25), 2))
        wk = rng.integers(0, P, size=(12, 24))
        we = rng.integers(0, P, size=(12, 24))
        mo = int(rng.choice([0, 0, 0, 2]))
        if T > 1:
            lv = np.sort(rng.choice([200, 300, 500, 800, 1000, 1e9], size=(T, P)), axis=0)
            lv[-1, :] = 1e38 if rng.random() < 0.7 else 1e9
        else:
            lv = None
        if k % 2 == 0:
            d = {"e_prices": prices.tolist(), "e_wkday_12by24": wk.tolist(),
                 "e_wkend_12by24": we.tolist(), "fixed_charge": fixed, "ur_metering_option": mo}
            if lv is not None:
                d["e_levels"] = lv.tolist()
        else:
            rows = []
            for p in range(P):
                for t in range(T):
                    cap = 1e38 if lv is None else float(lv[t, p])
                    rows.append([p + 1, t + 1, cap, 0, float(prices[t, p]), 0.0])
            d = {"ur_ec_tou_mat": rows, "ur_ec_sched_weekday": (wk + 1).tolist(),
                 "ur_ec_sched_weekend": (we + 1).tolist(), "ur_monthly_fixed_charge": fixed,
                 "ur_metering_option": mo}
        if k % 7 == 3:
            d = str(d)                       # python-dict-ish string form
        cases.append((f"rand{k:02d}", d))
    return cases


def er_fields(util):
    ER = util.ElectricityRates
    keep = {}
    for k, v in ER._vals.items():
        keep[k] = v
    return keep


def run_tariffs(ff, rng, ws_row):
    out = []
    for name, raw in tariff_cases(rng):
        td = ff.normalize_tariff(raw, net_sell_rate_scalar=0.0)
        rec = {"name": name, "raw": raw, "normalized": td, "process": {}}
        for variant, ts in (("ts_none", None), ("ts_8760", ws_row * 1.1)):
            u = FakeUtilityrate()
            ff.process_tariff(u, td, 0.0, ts_sell_rate=ts)
            rec["process"][variant] = er_fields(u)
        out.append(rec)
    return out


# ----------------------------------------------------------------------------
# Brent
# ----------------------------------------------------------------------------
def run_brent(rng):
    from scipy import optimize
    cases = []
    Ls = [0.5, 3.0, 4.7, 4.8, 5.0, 7.142857142857143, 7.5, 10.0, 20.0, 50.0, 100.0, 200.0,
          500.0, 1000.0, 4444.0, 6000.0]
    for L in Ls:
        low, high = L * 0.8, L * 1.25
        tol = max(2, int(max(1, high - low) * 1e-3))
        for kind in ("interior", "low_bound", "high_bound", "flat", "kink"):
            if kind == "interior":
                x0, c2, c1 = low + (high - low) * rng.uniform(0.2, 0.8), 1.0 + rng.random(), 0.0
            elif kind == "low_bound":
                x0, c2, c1 = 0.0, 0.0, 1.0
            elif kind == "high_bound":
                x0, c2, c1 = 0.0, 0.0, -3.0
            elif kind == "flat":
                x0, c2, c1 = 0.0, 0.0, 0.0
            else:
                x0, c2, c1 = L * 1.04, 2.5, -0.01
            xs = []

            def f(x):
                xs.append(float(x))
                d = x - x0
                return c2 * d * d + c1 * x
            res = optimize.minimize_scalar(f, bounds=(low, high), method="bounded",
                                           options={"xatol": tol})
            cases.append({"L": L, "kind": kind, "low": low, "high": high, "xatol": tol,
                          "c2": c2, "x0": x0, "c1": c1, "xs": xs, "x": float(res.x),
                          "nfev": int(res.nfev)})
    return cases


# ----------------------------------------------------------------------------
# agents
# ----------------------------------------------------------------------------
BASE_RES = dict(
    sector_abbr="res", inflation_rate=0.025, economic_lifetime_yrs=25, pv_degradation_factor=0.005,
    down_payment_fraction=0.3, tax_rate=0.2574, loan_term_yrs=20, real_discount_rate=0.05,
    itc_fraction_of_capex=0.3, system_capex_per_kw=4637.5, system_capex_per_kw_combined=4500.0,
    batt_capex_per_kwh_combined=431.0, cap_cost_multiplier=1.0, value_of_resiliency_usd=0.0,
    elec_price_multiplier=1.0, elec_price_escalator=0.0, system_om_per_kw=0.0,
    system_variable_om_per_kw=0.0, batt_capex_per_kw=0.0, batt_capex_per_kwh=0.0, batt_om_per_kw=0.0,
    batt_om_per_kwh=0.0, batt_capex_per_kw_combined=0.0, batt_om_per_kw_combined=0.0,
    batt_om_per_kwh_combined=0.0, linear_constant_combined=0.0, customers_in_bin=10.0,
    nem_system_kw_limit=100.0, tilt=20, azimuth=180)
BASE_COM = dict(BASE_RES, sector_abbr="com", down_payment_fraction=1.0, loan_term_yrs=30,
                real_discount_rate=0.0378, system_capex_per_kw=1672.9,
                system_capex_per_kw_combined=1600.0, batt_capex_per_kwh_combined=197.3)


def agent_specs(tariffs):
    t = {name: raw for name, raw in tariffs}
    specs = []

    def add(tag, base, **kw):
        d = dict(base)
        d.update(kw)
        d["tag"] = tag
        specs.append(d)

    add("res_K1", BASE_RES, state_abbr="DE", load_kwh_per_customer_in_bin=10000.0, tariff="K1",
        load_row=0, cf_row=1, wholesale_row=0, eia_id=101)
    add("res_tier", BASE_RES, state_abbr="DE", load_kwh_per_customer_in_bin=8200.0, tariff="K2",
        load_row=1, cf_row=0, wholesale_row=0, eia_id=101)
    add("res_K3", BASE_RES, state_abbr="MD", load_kwh_per_customer_in_bin=12500.0, tariff="K3",
        load_row=2, cf_row=2, wholesale_row=1, eia_id=102)
    add("res_K4str", BASE_RES, state_abbr="PA", load_kwh_per_customer_in_bin=6100.0, tariff="K4",
        load_row=3, cf_row=3, wholesale_row=1, eia_id=103)
    add("res_sticky", BASE_RES, state_abbr="DE", load_kwh_per_customer_in_bin=10000.0,
        tariff="K1", load_row=0, cf_row=0, wholesale_row=0, eia_id=201,
        elec_price_escalator=0.005)
    add("res_two_rows", BASE_RES, state_abbr="DE", load_kwh_per_customer_in_bin=9000.0,
        tariff="K1", load_row=1, cf_row=1, wholesale_row=0, eia_id=202)
    add("res_storage_sw", BASE_RES, state_abbr="NJ", load_kwh_per_customer_in_bin=11000.0,
        tariff="tier3_tou2", load_row=4, cf_row=4, wholesale_row=0, eia_id=203,
        value_of_resiliency_usd=150.0)
    add("res_mo2_ts", BASE_RES, state_abbr="AZ", load_kwh_per_customer_in_bin=14000.0,
        tariff="mo2_tou", load_row=2, cf_row=4, wholesale_row=1, eia_id=104,
        elec_price_multiplier=1.15)
    add("res_mo2_nan_ts", BASE_RES, state_abbr="AZ", load_kwh_per_customer_in_bin=9500.0,
        tariff="mo2_tou", load_row=3, cf_row=2, wholesale_row=2, eia_id=104)
    add("res_CA", BASE_RES, state_abbr="CA", load_kwh_per_customer_in_bin=7000.0, tariff="K1",
        load_row=4, cf_row=3, wholesale_row=0, eia_id=105, elec_price_escalator=-0.004)
    add("res_CA_tier", BASE_RES, state_abbr="CA", load_kwh_per_customer_in_bin=15500.0,
        tariff="tier3_tou2", load_row=0, cf_row=4, wholesale_row=1, eia_id=105)
    add("com_250MWh", BASE_COM, state_abbr="DE", load_kwh_per_customer_in_bin=250000.0,
        tariff="tier3_tou2", load_row=1, cf_row=1, wholesale_row=0, eia_id=301)
    add("com_5GWh", BASE_COM, state_abbr="MD", load_kwh_per_customer_in_bin=5.0e6, tariff="K2",
        load_row=2, cf_row=0, wholesale_row=1, eia_id=302, down_payment_fraction=0.2)
    add("com_mo2", BASE_COM, state_abbr="TX", load_kwh_per_customer_in_bin=80000.0,
        tariff="mo2_tou", load_row=3, cf_row=1, wholesale_row=1, eia_id=303)
    add("res_small", BASE_RES, state_abbr="DE", load_kwh_per_customer_in_bin=3200.0, tariff="K1",
        load_row=1, cf_row=2, wholesale_row=0, eia_id=101)
    add("res_daily", BASE_RES, state_abbr="VA", load_kwh_per_customer_in_bin=13000.0,
        tariff="daily_unit", load_row=4, cf_row=0, wholesale_row=0, eia_id=106,
        cap_cost_multiplier=1.1, inflation_rate=0.03)
    add("res_json", BASE_RES, state_abbr="VA", load_kwh_per_customer_in_bin=10500.0,
        tariff="json_str", load_row=2, cf_row=3, wholesale_row=0, eia_id=106, itc_fraction_of_capex=0.26)
    add("com_rand", BASE_COM, state_abbr="NY", load_kwh_per_customer_in_bin=42000.0,
        tariff="rand05", load_row=0, cf_row=2, wholesale_row=0, eia_id=304, tax_rate=0.21,
        loan_term_yrs=15, down_payment_fraction=0.5)
    add("res_rand", BASE_RES, state_abbr="NY", load_kwh_per_customer_in_bin=9300.0,
        tariff="rand10", load_row=3, cf_row=4, wholesale_row=1, eia_id=107,
        economic_lifetime_yrs=20, loan_term_yrs=10)
    add("com_kwkw", BASE_COM, state_abbr="OH", load_kwh_per_customer_in_bin=180000.0,
        tariff="kwkw_unit", load_row=0, cf_row=3, wholesale_row=0, eia_id=305)
    add("res_kwkw_daily_nb", BASE_RES, state_abbr="AZ", load_kwh_per_customer_in_bin=11500.0,
        tariff="kwkw_daily_nb", load_row=2, cf_row=1, wholesale_row=1, eia_id=108)
    for s in specs:
        s["tariff_dict"] = t[s["tariff"]]
    return specs


def switch_table(tariffs):
    t = {name: raw for name, raw in tariffs}
    rows = [
        # sticky DG switch: solar rows for eia 201, < 7 kW only
        ("solar", "DG_201_small", t["tier3_tou2"], 201, "R", 0.0, 7.0, 125.0),
        ("solar", "DG_201_big", t["K2"], 201, "R", 7.5, 1000.0, 300.0),
        # two overlapping rows -> len != 1 -> never switches
        ("solar", "DG_202_a", t["K2"], 202, "R", 0.0, 100.0, 50.0),
        ("solar", "DG_202_b", t["K3"], 202, "R", 5.0, 100.0, 60.0),
        # storage switch on bank capacity (kWh)
        ("storage", "ST_203", t["K3"], 203, "R", 1.0, 1000.0, 250.0),
        ("solar", "DG_203", t["K1"], 203, "R", 0.0, 2.0, 10.0),
        # commercial solar switch in the middle of the bracket
        ("solar", "DG_301", t["K1"], 301, "C", 150.0, 10000.0, 2000.0),
        ("storage", "ST_301", t["mo2_tou"], 301, "C", 0.0, 1e9, 0.0),
        # res row for a com agent's utility: sector mismatch -> ignored
        ("solar", "DG_302_res", t["K1"], 302, "R", 0.0, 1e9, 0.0),
        ("solar", "DG_105", t["K2"], 105, "R", 0.0, 1e9, 42.0),
    ]
    return pd.DataFrame(rows, columns=["tech", "rate_id_alias", "json", "eia_id", "res_com",
                                       "min_kw_limit", "max_kw_limit", "one_time_charge"])


class _Cur:
    def close(self):
        pass


class _Con:
    def cursor(self):
        return _Cur()


OUT_SCALARS = ["system_kw", "annual_energy_production_kwh", "naep", "capacity_factor",
               "price_per_kwh", "npv", "payback_period", "batt_kw", "batt_kwh",
               "nem_system_kw_limit"]
OUT_ARRAYS = ["cash_flow", "cf_energy_value_pv_only", "utility_bill_w_sys_pv_only",
              "utility_bill_wo_sys_pv_only", "cf_energy_value_pv_batt", "utility_bill_w_sys_pv_batt",
              "utility_bill_wo_sys_pv_batt"]
OUT_HOURLY = ["baseline_net_hourly", "adopter_net_hourly_pvonly", "adopter_net_hourly_with_batt",
              "adopter_net_hourly", "pv_per_kw_hourly"]


def run_agents(ff, elec, shapes, cfs, ws, tariffs):
    specs = agent_specs(tariffs)
    rst = switch_table(tariffs)
    state = {}

    def load_prof(con, agent):
        df = pd.DataFrame({"consumption_hourly": [shapes[state["load_row"]].astype(np.float64).tolist()]})
        df["load_kwh_per_customer_in_bin"] = agent.loc["load_kwh_per_customer_in_bin"]
        return df.apply(elec.scale_array_sum, axis=1,
                        args=("consumption_hourly", "load_kwh_per_customer_in_bin"))

    def solar_prof(con, agent):
        return pd.DataFrame({"solar_cf_profile": [cfs[state["cf_row"]].tolist()],
                             "scale_offset": [1e6]})

    elec.get_and_apply_agent_load_profiles = load_prof
    elec.get_and_apply_normalized_hourly_resource_solar = solar_prof

    # count evaluations through the objective
    orig = ff.calc_system_performance
    xs_log = []

    def counted(kw, *a, **k):
        xs_log.append((float(kw), bool(a[7]) if len(a) > 7 else bool(k.get("en_batt", True))))
        return orig(kw, *a, **k)
    ff.calc_system_performance = counted

    recs, hourly = [], {}
    for i, s in enumerate(specs):
        state["load_row"], state["cf_row"] = s["load_row"], s["cf_row"]
        row = {k: v for k, v in s.items() if k not in ("tag", "tariff", "load_row", "cf_row",
                                                         "wholesale_row")}
        row["agent_id"] = i
        row["bldg_id"] = 1000 + s["load_row"]
        row["solar_re_9809_gid"] = 5000 + s["cf_row"]
        row["tariff_id"] = 900 + i
        row["wholesale_prices"] = ws[s["wholesale_row"]]
        agent = pd.Series(row, name=i)
        xs_log.clear()
        out = ff.calc_system_size_and_performance(_Con(), agent, None, rst)
        pv_x = [x for x, b in xs_log if not b]
        rec = {"tag": s["tag"], "inputs": {k: v for k, v in s.items() if k != "tariff_dict"},
               "tariff_name": s["tariff"], "evals_pv": pv_x,
               "evals_batt": [x for x, b in xs_log if b],
               "final_tariff_id": out["tariff_id"] if not isinstance(out["tariff_id"], np.generic)
               else out["tariff_id"].item(),
               "final_tariff_dict": out["tariff_dict"]}
        for k in OUT_SCALARS:
            rec[k] = float(out[k])
        for k in OUT_ARRAYS:
            rec[k] = [float(v) for v in out[k]]
        for k in OUT_HOURLY:
            hourly[f"{i}:{k}"] = np.asarray(out[k], dtype=np.float64)
        recs.append(rec)
    ff.calc_system_performance = orig
    return recs, hourly, rst


# ----------------------------------------------------------------------------
# diffusion
# ----------------------------------------------------------------------------
MMS_CSV = "/root/reference/dgen_os/data_share/NREL_max_market_share.csv"


def diffusion_inputs(rng, n=1500):
    """Synthetic agent frame + max-market-share curves + Bass parameters."""
    raw = pd.read_csv(MMS_CSV)
    cur = raw[(raw.metric == "payback_period") & (raw.business_model == "host_owned_retrofit")]
    rows = []
    for sec, scale in (("res", 1.0), ("com", 0.8), ("ind", 0.6)):
        for pb, v in zip(cur.metric_value, cur.max_market_share):
            rows.append((float(pb), sec, float(v) * scale, "payback_period", "NREL", "host_owned"))
        rows.append((30.1, sec, 0.0, "payback_period", "NREL", "host_owned"))   # SQL union row
        rows.append((5.0, sec, 0.5, "payback_period", "NREL", "tpo"))           # filtered by the merge
    for pb in np.arange(0, 50, 0.5):
        rows.append((float(pb), "res", 0.3, "monthly_bill_savings", "NREL", "host_owned"))
    mms_df = pd.DataFrame(rows, columns=["payback_period", "sector_abbr", "max_market_share",
                                         "metric", "source", "business_model"])
    states = ["DE", "CA", "NY", "TX", "ZZ"]
    bp = []
    for st in states[:-1]:
        for sec in ("res", "com", "ind"):
            bp.append((st, sec, "solar", float(rng.uniform(0.0005, 0.003)), float(rng.uniform(0.3, 0.5)),
                       float(rng.uniform(2.0, 12.0))))
            bp.append((st, sec, "storage", 0.01, 0.2, 1.0))
    bass = pd.DataFrame(bp, columns=["state_abbr", "sector_abbr", "tech", "bass_param_p",
                                     "bass_param_q", "teq_yr1"])
    st = rng.choice(states, n)
    sec = rng.choice(["res", "com", "ind"], n)
    pb = np.round(rng.uniform(-2, 35, n), 3)
    special = [np.nan, 1e99, 30.1, 15.05, 0.0, 30.0, -1.0, 29.95, 0.04999999]
    pb[:len(special)] = special
    msly = rng.uniform(0, 0.2, n)
    msly[::37] = 0.0
    df = pd.DataFrame({
        "state_abbr": st, "sector_abbr": sec, "payback_period": pb,
        "market_share_last_year": msly,
        "developable_agent_weight": np.where(rng.random(n) < 0.05, 0.0, rng.uniform(0, 500, n)),
        "system_kw": rng.uniform(0, 200, n), "system_capex_per_kw": rng.uniform(1500, 5000, n),
        "adopters_cum_last_year": rng.uniform(0, 50, n), "market_value_last_year": rng.uniform(0, 1e5, n),
        "system_kw_cum_last_year": rng.uniform(0, 300, n), "batt_kw_cum_last_year": rng.uniform(0, 30, n),
        "batt_kwh_cum_last_year": rng.uniform(0, 60, n),
        "initial_number_of_adopters": rng.uniform(0, 5, n), "initial_pv_kw": rng.uniform(0, 10, n),
        "initial_batt_kw": 0.0, "initial_batt_kwh": 0.0, "initial_market_share": 0.0,
        "initial_market_value": 0.0,
    }, index=pd.Index(np.arange(100, 100 + n), name="agent_id"))
    return df, mms_df, bass


def run_diffusion(ff, rng):
    import diffusion_functions_elec as dfe
    df, mms_df, bass = diffusion_inputs(rng)
    out_mms = ff.calc_max_market_share(df, mms_df)
    d2 = out_mms.copy()
    d2.index = df.index
    res = {}
    for first in (True, False):
        out, mly = dfe.calc_diffusion_solar(d2, first, bass, 2026 if first else 2027)
        res["first" if first else "later"] = {"df": out.to_dict(orient="list"),
                                              "columns": list(out.columns),
                                              "market_last_year": mly.to_dict(orient="list"),
                                              "mly_columns": list(mly.columns)}
    return {"inputs": df.reset_index().to_dict(orient="list"), "mms_df": mms_df.to_dict(orient="list"),
            "bass": bass.to_dict(orient="list"),
            "mms_out": {"columns": list(out_mms.columns),
                        "max_market_share": out_mms["max_market_share"].tolist()},
            "diffusion": res}


def _jsonable(o):
    if isinstance(o, dict):
        return {str(k): _jsonable(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_jsonable(v) for v in o]
    if isinstance(o, np.ndarray):
        return _jsonable(o.tolist())
    if isinstance(o, (np.integer,)):
        return int(o)
    if isinstance(o, (np.floating,)):
        return float(o)
    if isinstance(o, (np.bool_,)):
        return bool(o)
    return o


def main():
    warnings.filterwarnings("ignore")
    ff, elec = install_stubs()
    rng = np.random.default_rng(20260001)
    shapes, cfs, ws = make_profiles(rng)
    tariffs = tariff_cases(np.random.default_rng(20260002))

    tar = run_tariffs(ff, np.random.default_rng(20260002), ws[0])
    with open(os.path.join(HERE, "tariffs.json"), "w") as f:
        json.dump(_jsonable(tar), f)

    br = run_brent(np.random.default_rng(20260003))
    with open(os.path.join(HERE, "brent.json"), "w") as f:
        json.dump(_jsonable(br), f)

    recs, hourly, rst = run_agents(ff, elec, shapes, cfs, ws, tariffs)
    meta = {"cfg": orc.DEFAULT_CFG, "agents": recs,
            "switch_table": _jsonable(rst.to_dict(orient="records")),
            "tariff_cases": _jsonable([[n, r] for n, r in tariffs])}
    with open(os.path.join(HERE, "agents.json"), "w") as f:
        json.dump(_jsonable(meta), f)
    dif = run_diffusion(ff, np.random.default_rng(20260004))
    with open(os.path.join(HERE, "diffusion.json"), "w") as f:
        json.dump(_jsonable(dif), f)
    np.savez_compressed(os.path.join(HERE, "agents.npz"), shapes=shapes, cfs=cfs, wholesale=ws,
                        **{k.replace(":", "__"): v for k, v in hourly.items()})
    print(f"tariffs={len(tar)} brent={len(br)} agents={len(recs)}")
    for r in recs:
        print(f"  {r['tag']:16s} kw={r['system_kw']:.4f} evals={len(r['evals_pv'])} "
              f"npv={r['npv']:.2f} pb={r['payback_period']} tariff={r['final_tariff_id']}")


if __name__ == "__main__":
    main()
