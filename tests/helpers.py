"""Shared test helpers: golden fixtures -> product columns / oracle population."""
from __future__ import annotations

import json
import os
from functools import lru_cache

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


@lru_cache(maxsize=None)
def golden_agents():
    with open(os.path.join(GOLDEN, "agents.json")) as f:
        meta = json.load(f)
    z = np.load(os.path.join(GOLDEN, "agents.npz"), allow_pickle=False)
    arrays = {k: z[k] for k in z.files}
    return meta, arrays


@lru_cache(maxsize=None)
def golden_tariffs():
    with open(os.path.join(GOLDEN, "tariffs.json")) as f:
        return json.load(f)


@lru_cache(maxsize=None)
def golden_brent():
    with open(os.path.join(GOLDEN, "brent.json")) as f:
        return json.load(f)


def golden_population():
    """PopulationBuilder over the golden agents (product host path)."""
    from dgen_amd.columnar import PopulationBuilder
    meta, arr = golden_agents()
    tariffs = {name: raw for name, raw in meta["tariff_cases"]}
    table = pd.DataFrame(meta["switch_table"])
    b = PopulationBuilder(table)
    ws = arr["wholesale"]
    for i, a in enumerate(meta["agents"]):
        s = a["inputs"]
        b.add(load_row=s["load_row"], cf_row=s["cf_row"], sector_abbr=s["sector_abbr"],
              state_abbr=s["state_abbr"], eia_id=s["eia_id"], tariff_dict=tariffs[s["tariff"]],
              wholesale=ws[s["wholesale_row"]], load_kwh=s["load_kwh_per_customer_in_bin"],
              price_mult=s["elec_price_multiplier"], econ_life=s["economic_lifetime_yrs"],
              loan_term=s["loan_term_yrs"], inflation=s["inflation_rate"],
              pv_deg=s["pv_degradation_factor"], escalator=s["elec_price_escalator"],
              down_payment=s["down_payment_fraction"], tax_rate=s["tax_rate"],
              real_discount=s["real_discount_rate"], itc_frac=s["itc_fraction_of_capex"],
              capex=s["system_capex_per_kw"], capex_combined=s["system_capex_per_kw_combined"],
              batt_capex_kwh=s["batt_capex_per_kwh_combined"], ccm=s["cap_cost_multiplier"],
              vor=s["value_of_resiliency_usd"])
    cols = b.columns()
    return b, cols, arr["shapes"], arr["cfs"], b.wholesale.array()


def oracle_tariffs(records, demand=None):
    """Device tariff records (+ the dgen_demand table) -> orc.Tariff list."""
    from oracle import oracle as orc
    out = []
    for r in records:
        t = orc.Tariff()
        t.P, t.T, t.mo, t.unit = int(r["P"]), int(r["T"]), int(r["mo"]), int(r["unit"])
        t.fixed = float(r["fixed"])
        for k in range(orc.MAXT):
            t.cap[k] = float(r["cap"][k])
        for p in range(orc.MAXP):
            for k in range(orc.MAXT):
                t.buy[p][k] = float(r["buy"][p, k])
                t.sell[p][k] = float(r["sell"][p, k])
        for m in range(12):
            for h in range(24):
                t.wkday[m][h] = int(r["wkday"][m, h])
                t.wkend[m][h] = int(r["wkend"][m, h])
        dc = int(r["dc"])
        if dc > 0:
            d = demand[dc - 1]
            t.dc_on = 1
            for p in range(orc.DCP):
                t.dc_tou_nt[p] = int(d["tou_nt"][p])
                for k in range(orc.DCT):
                    t.dc_tou_cap[p][k] = float(d["tou_cap"][p, k])
                    t.dc_tou_price[p][k] = float(d["tou_price"][p, k])
            for m in range(12):
                t.dc_flat_nt[m] = int(d["flat_nt"][m])
                for k in range(orc.DCT):
                    t.dc_flat_cap[m][k] = float(d["flat_cap"][m, k])
                    t.dc_flat_price[m][k] = float(d["flat_price"][m, k])
                for h in range(24):
                    t.dc_wkday[m][h] = int(d["wkday"][m, h])
                    t.dc_wkend[m][h] = int(d["wkend"][m, h])
        out.append(t)
    return out


def oracle_population(cols, tariff_records, switches, shapes, cfs, wholesale, demand=None):
    """orc.Population mirroring product columns (same tables, same indices)."""
    from oracle import oracle as orc
    n = len(cols["load_kwh"])
    sw_solar, sw_storage = [], []
    for i in range(n):
        for k, dst in (("solar", sw_solar), ("storage", sw_storage)):
            off, cnt = int(cols[f"sw_{k}_off"][i]), int(cols[f"sw_{k}_cnt"][i])
            dst.append([(float(r["min_kw"]), float(r["max_kw"]), float(r["one_time_charge"]),
                         int(r["tariff"])) for r in switches[off:off + cnt]])
    ocols = {
        "load_row": cols["load_row"], "cf_row": cols["cf_row"],
        "wholesale_row": cols["wholesale_row"], "load_kwh": cols["load_kwh"],
        "price_mult": cols["price_mult"], "inflation": cols["inflation"], "pv_deg": cols["pv_deg"],
        "escalator": cols["escalator"], "down_payment": cols["down_payment"],
        "tax_rate": cols["tax_rate"], "real_discount": cols["real_discount"],
        "itc_frac": cols["itc_frac"], "capex": cols["capex"],
        "capex_combined": cols["capex_combined"],
        "batt_capex_kwh_combined": cols["batt_capex_kwh"], "ccm": cols["ccm"], "vor": cols["vor"],
        "is_res": (cols["flags"] & 1).astype(int), "is_ca": ((cols["flags"] >> 1) & 1).astype(int),
        "econ_life": cols["econ_life"], "loan_term": cols["loan_term"], "tariff0": cols["tariff0"],
    }
    return orc.Population(ocols, shapes, cfs, wholesale, oracle_tariffs(tariff_records, demand),
                          sw_solar, sw_storage)


def final_tariff_id(builder, agent_tariff_id, final_index, switched):
    if switched:
        r = builder.switches.row_of_tariff.get(int(final_index))
        if r is not None:
            return r["rate_id_alias"]
    return agent_tariff_id


def golden_rows():
    """The golden agents as reference-style agent rows (pd.Series) + a
    ProfileStore + the rate switch table, as make_golden.py built them."""
    from dgen_amd.profiles import ProfileStore
    meta, arr = golden_agents()
    tariffs = {name: raw for name, raw in meta["tariff_cases"]}
    store = ProfileStore()
    rows = []
    for i, a in enumerate(meta["agents"]):
        s = dict(a["inputs"])
        lr, cr, wr = s.pop("load_row"), s.pop("cf_row"), s.pop("wholesale_row")
        s.pop("tag")
        s["tariff_dict"] = tariffs[s.pop("tariff")]
        s["agent_id"] = i
        s["bldg_id"] = 1000 + lr
        s["solar_re_9809_gid"] = 5000 + cr
        s["tariff_id"] = 900 + i
        s["wholesale_prices"] = arr["wholesale"][wr]
        store.add_load((s["bldg_id"], s["sector_abbr"], s["state_abbr"]), arr["shapes"][lr])
        store.add_solar((s["solar_re_9809_gid"], s["tilt"], s["azimuth"]), arr["cfs"][cr])
        rows.append(pd.Series(s, name=i))
    return rows, store, pd.DataFrame(meta["switch_table"])


@lru_cache(maxsize=None)
def golden_attach():
    """(meta, hourly): attach.json cases + the f32 planes from attach.npz,
    hourly[name] = (baseline, pvonly, with_batt) as float64 [n, n_hours]."""
    with open(os.path.join(GOLDEN, "attach.json")) as f:
        meta = json.load(f)
    z = np.load(os.path.join(GOLDEN, "attach.npz"), allow_pickle=False)
    hourly = {}
    for c in meta["cases"]:
        k = c["name"]
        hourly[k] = tuple(z[f"{k}__{p}"].astype(np.float64) for p in ("baseline", "pvonly", "with_batt"))
    return meta, hourly


def _dec(cell):
    """finance_series.json cell -> the Python value the reference saw."""
    f = lambda x: float(x) if isinstance(x, str) and x in ("nan", "inf", "-inf") else x
    if "list" in cell:
        return [f(x) for x in cell["list"]]
    if "array" in cell:
        return np.asarray([f(x) for x in cell["array"]], dtype=float)
    return f(cell["scalar"])


@lru_cache(maxsize=None)
def golden_finance():
    """finance_series.json with the input rows decoded (lists, numpy arrays,
    scalars, non-finite floats) -- cases[k]['rows'] are dicts per agent."""
    with open(os.path.join(GOLDEN, "finance_series.json")) as f:
        meta = json.load(f)
    for c in meta["cases"]:
        c["rows"] = [{k: _dec(v) for k, v in r.items()} for r in c["rows"]]
    return meta


@lru_cache(maxsize=None)
def golden_tariffs_dc():
    """tariffs_dc.json: the reference's compile with SKIP_DEMAND_CHARGES
    flipped (tests/golden/make_golden_demand.py)."""
    with open(os.path.join(GOLDEN, "tariffs_dc.json")) as f:
        return json.load(f)


# tests/golden/market.json column -> device SoA / loop column (dgen_amd.market)
MARKET_COLS = {"load_kwh_per_customer_in_bin": "load_kwh", "customers_in_bin": "customers_in_bin",
               "load_kwh_in_bin": "load_kwh_in_bin", "elec_price_multiplier": "price_mult",
               "elec_price_escalator": "escalator", "pv_degradation_factor": "pv_deg",
               "system_capex_per_kw": "capex", "system_capex_per_kw_combined": "capex_combined",
               "batt_capex_per_kwh_combined": "batt_capex_kwh", "value_of_resiliency_usd": "vor",
               "itc_fraction_of_capex": "itc_frac", "inflation_rate": "inflation",
               "economic_lifetime_yrs": "econ_life", "loan_term_yrs": "loan_term",
               "down_payment_fraction": "down_payment", "real_discount_rate": "real_discount",
               "tax_rate": "tax_rate"}


@lru_cache(maxsize=None)
def golden_market():
    """market.json (tests/golden/make_golden_market.py): agents, the reference's
    input tables as DataFrames, and per year the merged columns (None -> NaN)."""
    with open(os.path.join(GOLDEN, "market.json")) as f:
        meta = json.load(f)
    nan = lambda v: np.array([np.nan if x is None else x for x in v], dtype=np.float64)
    meta["agents"] = pd.DataFrame(meta["agents"])
    T = {k: pd.DataFrame(v) for k, v in meta["tables"].items()}
    meta["tables"] = {"load_growth": T["load_growth"], "elec_price": T["elec"], "pv_tech": T["pv_tech"],
                      "pv_price": T["pv_price"], "pv_plus_batt_price": T["pvb_price"], "vor": T["vor"],
                      "financing": T["fin"], "itc": T["itc"]}
    for y in meta["years"]:
        y["columns"] = {k: nan(v) for k, v in y["columns"].items()}
        if "initial" in y:
            y["initial"]["columns"] = {k: nan(v) for k, v in y["initial"]["columns"].items()}
    return meta


# ---------------------------------------------------------------------------
# Brent paths: the device's fast search bills from
# re-associated sums, a few ulps from the oracle's hour order; scipy's bounded
# Brent divides differences of nearly equal objective values in its parabolic
# step, so such a difference can move the search path.  The certified paths
# (dgen_set_exact, on by default) re-run every agent whose path a bound on that
# difference does not settle in the oracle's arithmetic, so every agent is on
# the oracle's path (same_path); with them off (exact_brent = 0), a divergent
# agent ends within scipy's xatol and equals the oracle's driver evaluated at
# the device's own search end (at_device_point).
# ---------------------------------------------------------------------------
def xatol_of(load_kwh: float, naep: float) -> float:
    """ff:440-444: bracket (0.8, 1.25) x load / naep, xatol = max(2, int(1e-3 x span))."""
    hi_lo = (load_kwh / naep) * 1.25 - (load_kwh / naep) * 0.8
    return max(2.0, float(int(max(hi_lo, 1.0) * 1e-3)))


def same_path(o, i: int, r) -> bool:
    """Device agent i (o: host outputs) took the oracle result r's Brent path."""
    return (int(o["nfev"][i]) == int(r["nfev"])
            and abs(o["system_kw"][i] - r["system_kw"]) <= 1e-9 * max(1.0, abs(r["system_kw"]))
            and abs(o["x_last"][i] - r["x_last"]) <= 1e-9 * max(1.0, abs(r["x_last"])))


def at_device_point(o, i: int, opop, j: int, cfg, r, xatol: float, hourly: bool = False):
    """Oracle outputs of agent j of opop evaluated once at device agent i's
    search end -- its kW, last x and sticky tariff state (tariff_final and
    switched as the device reports them: size with the battery run off, so no
    storage switch follows the search).  The device's kW must be within
    scipy's xatol of the oracle's search result."""
    kw, xl = float(o["system_kw"][i]), float(o["x_last"][i])
    assert abs(kw - r["system_kw"]) <= xatol, ("kW beyond xatol", i, kw, r["system_kw"], xatol)
    e = opop.eval_at(cfg, j, kw, xl, int(o["tariff_final"][i]), int(o["switched"][i]), hourly=hourly)
    e["nfev"] = int(o["nfev"][i])
    return e
