"""ctypes view of the CPU oracle (oracle/orc.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker / timed CPU baseline.  The product
package (dgen_amd/) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Dict, List, Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liborc.so")

NH = 8760
MAXP = 12
MAXT = 6
DCP = 8
DCT = 4
MAXY = 50

_c_double = ctypes.c_double
_c_int32 = ctypes.c_int32
_dp = ctypes.POINTER(ctypes.c_double)


class Tariff(ctypes.Structure):
    _fields_ = [
        ("P", _c_int32), ("T", _c_int32), ("mo", _c_int32), ("unit", _c_int32),
        ("fixed", _c_double),
        ("cap", _c_double * MAXT),
        ("buy", (_c_double * MAXT) * MAXP),
        ("sell", (_c_double * MAXT) * MAXP),
        ("wkday", (ctypes.c_uint8 * 24) * 12),
        ("wkend", (ctypes.c_uint8 * 24) * 12),
        ("dc_on", _c_int32),
        ("dc_tou_nt", _c_int32 * DCP), ("dc_flat_nt", _c_int32 * 12),
        ("dc_tou_cap", (_c_double * DCT) * DCP), ("dc_tou_price", (_c_double * DCT) * DCP),
        ("dc_flat_cap", (_c_double * DCT) * 12), ("dc_flat_price", (_c_double * DCT) * 12),
        ("dc_wkday", (ctypes.c_uint8 * 24) * 12),
        ("dc_wkend", (ctypes.c_uint8 * 24) * 12),
    ]


class Cfg(ctypes.Structure):
    _fields_ = [
        ("nm_yearend_sell_rate", _c_double), ("loan_rate_pct", _c_double),
        ("insurance_rate_pct", _c_double), ("itc_fed_max", _c_double),
        ("depr_sl_years", _c_int32),
        ("batt_v_nom", _c_double), ("batt_q_full", _c_double),
        ("batt_min_soc", _c_double), ("batt_max_soc", _c_double),
        ("batt_init_soc", _c_double), ("batt_eta_in", _c_double),
        ("batt_eta_out", _c_double), ("batt_update_hours", _c_int32),
        ("batt_loss_model", _c_int32), ("batt_r_cell", _c_double), ("batt_conv_eff", _c_double),
        ("batt_v_cell_empty", _c_double), ("batt_v_cell_full", _c_double),
        ("batt_month_floor", _c_int32),
    ]


class Switch(ctypes.Structure):
    _fields_ = [("min_kw", _c_double), ("max_kw", _c_double),
                ("one_time_charge", _c_double), ("tariff", _c_int32), ("pad", _c_int32)]


class Agent(ctypes.Structure):
    _fields_ = [
        ("shape", ctypes.POINTER(ctypes.c_float)),
        ("cf", ctypes.POINTER(ctypes.c_int32)),
        ("wholesale", _dp),
        ("load_kwh", _c_double), ("price_mult", _c_double),
        ("is_res", _c_int32), ("is_ca", _c_int32), ("econ_life", _c_int32), ("loan_term", _c_int32),
        ("inflation", _c_double), ("pv_deg", _c_double), ("escalator", _c_double),
        ("down_payment", _c_double), ("tax_rate", _c_double), ("real_discount", _c_double),
        ("itc_frac", _c_double),
        ("capex", _c_double), ("capex_combined", _c_double), ("batt_capex_kwh_combined", _c_double),
        ("ccm", _c_double), ("vor", _c_double),
        ("tariff0", _c_int32), ("n_sw_solar", _c_int32), ("n_sw_storage", _c_int32),
        ("sw_solar", ctypes.POINTER(Switch)), ("sw_storage", ctypes.POINTER(Switch)),
    ]


class Result(ctypes.Structure):
    _fields_ = [
        ("system_kw", _c_double), ("x_last", _c_double), ("annual_kwh", _c_double),
        ("naep", _c_double), ("capacity_factor", _c_double), ("price_per_kwh", _c_double),
        ("npv", _c_double), ("payback_raw", _c_double), ("payback_period", _c_double),
        ("first_with", _c_double), ("first_without", _c_double),
        ("batt_kw", _c_double), ("batt_kwh", _c_double), ("npv_pv_batt", _c_double),
        ("nfev", _c_int32), ("tariff_final", _c_int32), ("switched", _c_int32), ("status", _c_int32),
        ("cash_flow", _c_double * (MAXY + 1)),
        ("cf_energy_value_pv_only", _c_double * (MAXY + 1)),
        ("bill_w_pv_only", _c_double * (MAXY + 1)),
        ("bill_wo_pv_only", _c_double * (MAXY + 1)),
        ("cf_energy_value_pv_batt", _c_double * (MAXY + 1)),
        ("bill_w_pv_batt", _c_double * (MAXY + 1)),
        ("bill_wo_pv_batt", _c_double * (MAXY + 1)),
        ("baseline", _dp), ("net_pvonly", _dp), ("net_with_batt", _dp),
    ]


class LoanIn(ctypes.Structure):
    _fields_ = [
        ("nyears", _c_int32), ("market", _c_int32), ("loan_term", _c_int32),
        ("depr_fed_type", _c_int32), ("depr_sta_type", _c_int32), ("pad", _c_int32),
        ("debt_fraction_pct", _c_double), ("fed_tax_pct", _c_double), ("sta_tax_pct", _c_double),
        ("real_disc_pct", _c_double), ("inflation_pct", _c_double), ("itc_fed_pct", _c_double),
        ("total_cost", _c_double),
    ]


# PySAM config defaults the reference never sets; mirrored by dgen_amd.config.
DEFAULT_CFG = dict(
    nm_yearend_sell_rate=0.02, loan_rate_pct=7.5, insurance_rate_pct=0.0, itc_fed_max=1e38,
    depr_sl_years=7, batt_v_nom=3.6, batt_q_full=3.2, batt_min_soc=0.10, batt_max_soc=0.95,
    batt_init_soc=0.30, batt_eta_in=0.9408, batt_eta_out=0.9408, batt_update_hours=24,
    batt_loss_model=0, batt_r_cell=0.001, batt_conv_eff=0.96, batt_v_cell_empty=3.0, batt_v_cell_full=4.2,
    batt_month_floor=0,
)


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_pairwise_sum.restype = _c_double
        L.orc_pairwise_sum.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.orc_np_sum.restype = _c_double
        L.orc_np_sum.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.orc_np_round1.restype = _c_double
        L.orc_np_round1.argtypes = [_c_double]
        L.orc_tariff_from_mat.restype = ctypes.c_int
        L.orc_tariff_from_mat.argtypes = [ctypes.POINTER(Tariff), ctypes.c_void_p, ctypes.c_int,
                                          ctypes.c_int, _c_double, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_ur5.restype = ctypes.c_int
        L.orc_ur5.argtypes = [ctypes.POINTER(Tariff), ctypes.POINTER(Cfg), ctypes.c_void_p,
                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, _c_double, _c_double,
                              _c_double, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_void_p]
        L.orc_cashloan.restype = ctypes.c_int
        L.orc_cashloan.argtypes = [ctypes.POINTER(LoanIn), ctypes.POINTER(Cfg), ctypes.c_void_p,
                                   _dp, _dp, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_batt_size.restype = None
        L.orc_batt_size.argtypes = [_c_double, _c_double, _c_double, ctypes.POINTER(Cfg), _dp, _dp]
        L.orc_batt_dispatch.restype = None
        L.orc_batt_dispatch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _c_double, _c_double,
                                        ctypes.POINTER(Cfg), ctypes.c_void_p, ctypes.c_void_p]
        L.orc_brent_quadratic.restype = ctypes.c_int
        L.orc_brent_quadratic.argtypes = [_c_double, _c_double, _c_double, _c_double, _c_double,
                                          _c_double, ctypes.c_void_p, ctypes.c_int, _dp]
        L.orc_size_agent.restype = ctypes.c_int
        L.orc_size_agent.argtypes = [ctypes.POINTER(Agent), ctypes.POINTER(Tariff), ctypes.c_int,
                                     ctypes.POINTER(Cfg), ctypes.POINTER(Result)]
        L.orc_size_batch.restype = ctypes.c_int
        L.orc_size_batch.argtypes = [ctypes.POINTER(Agent), ctypes.c_int64, ctypes.POINTER(Tariff),
                                     ctypes.c_int, ctypes.POINTER(Cfg), ctypes.POINTER(Result),
                                     ctypes.c_int]
        L.orc_eval_at.restype = ctypes.c_int
        L.orc_eval_at.argtypes = [ctypes.POINTER(Agent), ctypes.POINTER(Tariff), ctypes.c_int,
                                  ctypes.POINTER(Cfg), _c_double, _c_double, ctypes.c_int, ctypes.c_int,
                                  ctypes.POINTER(Result)]
        L.orc_set_trace.restype = None
        L.orc_set_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_trace_count.restype = ctypes.c_int
        _lib = L
    return _lib


def make_cfg(**over) -> Cfg:
    d = dict(DEFAULT_CFG)
    d.update(over)
    return Cfg(**d)


def np_sum(a: np.ndarray) -> float:
    a = np.ascontiguousarray(a, dtype=np.float64)
    return lib().orc_np_sum(a.ctypes.data, a.size)


def np_round1(x: float) -> float:
    return lib().orc_np_round1(float(x))


def tariff_from_fields(mat: Sequence[Sequence[float]], mo: int, fixed: float,
                       wk: Sequence[Sequence[int]], we: Sequence[Sequence[int]]) -> Tariff:
    m = np.ascontiguousarray(np.asarray(mat, dtype=np.float64).reshape(-1, 6) if len(mat) else
                             np.zeros((0, 6)))
    wka = np.ascontiguousarray(np.asarray(wk, dtype=np.int32).reshape(12, 24))
    wea = np.ascontiguousarray(np.asarray(we, dtype=np.int32).reshape(12, 24))
    t = Tariff()
    rc = lib().orc_tariff_from_mat(ctypes.byref(t), m.ctypes.data, m.shape[0], int(mo),
                                   float(fixed), wka.ctypes.data, wea.ctypes.data)
    if rc != 0:
        raise ValueError(f"orc_tariff_from_mat failed: {rc}")
    return t


def ur5(t: Tariff, cfg: Cfg, gen, load, ts_sell, nyears, inflation_pct, escal_pct, degr_pct):
    gen = np.ascontiguousarray(gen, dtype=np.float64)
    load = np.ascontiguousarray(load, dtype=np.float64)
    ts = None if ts_sell is None else np.ascontiguousarray(ts_sell, dtype=np.float64)
    bw = np.zeros(nyears + 1); bwo = np.zeros(nyears + 1); aev = np.zeros(nyears + 1)
    efg = np.zeros(NH)
    rc = lib().orc_ur5(ctypes.byref(t), ctypes.byref(cfg), gen.ctypes.data, load.ctypes.data,
                       None if ts is None else ts.ctypes.data, int(nyears), float(inflation_pct),
                       float(escal_pct), float(degr_pct), bw.ctypes.data, bwo.ctypes.data,
                       aev.ctypes.data, efg.ctypes.data)
    if rc != 0:
        raise ValueError(f"orc_ur5 failed: {rc}")
    return dict(bill_w=bw, bill_wo=bwo, aev=aev, e_fromgrid=efg)


def cashloan(li: LoanIn, cfg: Cfg, aev):
    aev = np.ascontiguousarray(aev, dtype=np.float64)
    n = li.nyears
    cfpb = np.zeros(n + 1); cfev = np.zeros(n + 1)
    npv = ctypes.c_double(); pb = ctypes.c_double()
    rc = lib().orc_cashloan(ctypes.byref(li), ctypes.byref(cfg), aev.ctypes.data,
                            ctypes.byref(npv), ctypes.byref(pb), cfpb.ctypes.data, cfev.ctypes.data)
    if rc != 0:
        raise ValueError(f"orc_cashloan failed: {rc}")
    return dict(npv=npv.value, payback=pb.value, cf_payback=cfpb, cf_energy_value=cfev)


def batt_size(desired_kw, desired_kwh, desired_v, cfg: Cfg):
    b = ctypes.c_double(); p = ctypes.c_double()
    lib().orc_batt_size(float(desired_kw), float(desired_kwh), float(desired_v), ctypes.byref(cfg),
                        ctypes.byref(b), ctypes.byref(p))
    return b.value, p.value


def batt_dispatch(load, pv, bank, power, cfg: Cfg):
    load = np.ascontiguousarray(load, dtype=np.float64)
    pv = np.ascontiguousarray(pv, dtype=np.float64)
    sg = np.zeros(NH); g2l = np.zeros(NH)
    lib().orc_batt_dispatch(load.ctypes.data, pv.ctypes.data, float(bank), float(power),
                            ctypes.byref(cfg), sg.ctypes.data, g2l.ctypes.data)
    return sg, g2l


def brent_quadratic(lo, hi, xatol, c2, x0, c1, maxn=600):
    xs = np.zeros(maxn)
    xo = ctypes.c_double()
    n = lib().orc_brent_quadratic(lo, hi, xatol, c2, x0, c1, xs.ctypes.data, maxn, ctypes.byref(xo))
    return xs[:min(n, maxn)].copy(), xo.value, n


class Population:
    """Host arrays for a batch of oracle agents (keeps every buffer alive)."""

    def __init__(self, cols: Dict[str, np.ndarray], shapes: np.ndarray, cfs: np.ndarray,
                 wholesale: Optional[np.ndarray], tariffs: List[Tariff],
                 sw_solar: List[List[tuple]], sw_storage: List[List[tuple]]):
        n = len(cols["load_kwh"])
        self.n = n
        self.shapes = np.ascontiguousarray(shapes, dtype=np.float32)
        self.cfs = np.ascontiguousarray(cfs, dtype=np.int32)
        self.wholesale = None if wholesale is None else np.ascontiguousarray(wholesale, np.float64)
        self.tariffs = (Tariff * len(tariffs))(*tariffs)
        self.n_tariffs = len(tariffs)
        self.agents = (Agent * n)()
        self._sw = []
        for i in range(n):
            a = self.agents[i]
            a.shape = self.shapes[cols["load_row"][i]].ctypes.data_as(ctypes.POINTER(ctypes.c_float))
            a.cf = self.cfs[cols["cf_row"][i]].ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
            wr = int(cols["wholesale_row"][i])
            a.wholesale = (self.wholesale[wr].ctypes.data_as(_dp) if (self.wholesale is not None
                                                                       and wr >= 0) else None)
            for k in ("load_kwh", "price_mult", "inflation", "pv_deg", "escalator", "down_payment",
                      "tax_rate", "real_discount", "itc_frac", "capex", "capex_combined",
                      "batt_capex_kwh_combined", "ccm", "vor"):
                setattr(a, k, float(cols[k][i]))
            for k in ("is_res", "is_ca", "econ_life", "loan_term", "tariff0"):
                setattr(a, k, int(cols[k][i]))
            for nm, rows in (("solar", sw_solar[i]), ("storage", sw_storage[i])):
                arr = (Switch * max(1, len(rows)))()
                for j, (lo, hi, otc, tix) in enumerate(rows):
                    arr[j] = Switch(lo, hi, otc, tix, 0)
                self._sw.append(arr)
                setattr(a, "n_sw_" + nm, len(rows))
                setattr(a, "sw_" + nm, ctypes.cast(arr, ctypes.POINTER(Switch)))

    def run(self, cfg: Cfg, hourly: bool = False, threads: int = 1, idx=None):
        """Size agents (all, or the given indices). Returns list of dict results."""
        idxs = range(self.n) if idx is None else idx
        out = []
        for i in idxs:
            r = Result()
            bufs = None
            if hourly:
                bufs = [np.zeros(NH), np.zeros(NH), np.zeros(NH)]
                r.baseline = bufs[0].ctypes.data_as(_dp)
                r.net_pvonly = bufs[1].ctypes.data_as(_dp)
                r.net_with_batt = bufs[2].ctypes.data_as(_dp)
            lib().orc_size_agent(ctypes.byref(self.agents[i]), self.tariffs, self.n_tariffs,
                                 ctypes.byref(cfg), ctypes.byref(r))
            out.append(result_to_dict(r, int(self.agents[i].econ_life), bufs))
        return out

    def eval_at(self, cfg: Cfg, i: int, kw_star: float, x_last: float, tariff: int, switched: int,
                hourly: bool = False) -> dict:
        """Agent i's driver outputs for a search that ended at (kw_star,
        x_last) with the given sticky tariff state (orc_eval_at)."""
        r = Result()
        bufs = None
        if hourly:
            bufs = [np.zeros(NH), np.zeros(NH), np.zeros(NH)]
            r.baseline = bufs[0].ctypes.data_as(_dp)
            r.net_pvonly = bufs[1].ctypes.data_as(_dp)
            r.net_with_batt = bufs[2].ctypes.data_as(_dp)
        rc = lib().orc_eval_at(ctypes.byref(self.agents[i]), self.tariffs, self.n_tariffs, ctypes.byref(cfg),
                               float(kw_star), float(x_last), int(tariff), int(switched), ctypes.byref(r))
        if rc < -3:
            raise ValueError(f"orc_eval_at failed: {rc}")
        return result_to_dict(r, int(self.agents[i].econ_life), bufs)

    def run_parallel(self, cfg: Cfg, threads: int = 0, idx=None):
        """As run() without hourly outputs, the agents sized by the OpenMP batch
        entry (orc_size_batch) over `threads` (0: OMP_NUM_THREADS or all CPUs)."""
        import os
        idxs = list(range(self.n)) if idx is None else [int(i) for i in idx]
        if threads <= 0:
            threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
        sub = (Agent * len(idxs))(*[self.agents[i] for i in idxs])
        res = (Result * len(idxs))()
        lib().orc_size_batch(sub, len(idxs), self.tariffs, self.n_tariffs, ctypes.byref(cfg), res, int(threads))
        return [result_to_dict(res[k], int(sub[k].econ_life)) for k in range(len(idxs))]

    def run_batch_timed(self, cfg: Cfg, threads: int, idx: Sequence[int]):
        """Batch entry used for the CPU baseline (OpenMP over `threads`)."""
        sub = (Agent * len(idx))(*[self.agents[i] for i in idx])
        res = (Result * len(idx))()
        bad = lib().orc_size_batch(sub, len(idx), self.tariffs, self.n_tariffs, ctypes.byref(cfg),
                                   res, int(threads))
        return res, bad


def result_to_dict(r: Result, n_years: int, hourly=None) -> dict:
    d = {k: getattr(r, k) for k, _ in Result._fields_
         if k not in ("baseline", "net_pvonly", "net_with_batt") and not k.startswith(("cash", "cf_", "bill"))}
    for k in ("cash_flow", "cf_energy_value_pv_only", "bill_w_pv_only", "bill_wo_pv_only",
              "cf_energy_value_pv_batt", "bill_w_pv_batt", "bill_wo_pv_batt"):
        d[k] = np.array(getattr(r, k)[: n_years + 1])
    if hourly is not None:
        d["baseline_net_hourly"], d["adopter_net_hourly_pvonly"], d["adopter_net_hourly_with_batt"] = hourly
    return d


def brent_trace(opop, cfg: Cfg, i: int, maxn: int = 600):
    """Diagnostics: size agent i of `opop` (an OraclePopulation) and return the
    (x, f) pairs of its bounded-Brent evaluations, in order."""
    buf = np.zeros(2 * maxn)
    L = lib()
    L.orc_set_trace(buf.ctypes.data, maxn)
    try:
        res = opop.run(cfg, idx=[i])
        n = min(L.orc_trace_count(), maxn)
    finally:
        L.orc_set_trace(None, 0)
    return buf[:2 * n].reshape(n, 2), res
