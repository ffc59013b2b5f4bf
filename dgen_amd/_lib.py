"""ctypes binding of libdgen_hip.so (include/dgen_hip.h).

The product path has no CPU fallback: if the library is missing or a call
fails, this raises.  Struct layouts mirror the header field for field and are
checked against sizeof() probes in tests/test_abi.py.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

from . import build as _build

NH = 8760
NSLOT = 576
MAXP = 12
MAXT = 6
MAXY = 50
NB_CAPM = 192   # include/dgen_hip.h DGEN_NB_CAPM (mixed hours per month of a net-billing record)
DCR_CAP = 1024  # include/dgen_hip.h DGEN_DCR_CAP (kept hours per battery-case demand record)

ST_BOUNDS = 0x01
ST_TARIFF = 0x02
ST_EMPTY_EC = 0x04
ST_UNIT = 0x08
ST_YEARS = 0x10
ST_SCRATCH = 0x20
ST_ZERO_LOAD = 0x40
ST_DEMAND = 0x80
ST_FATAL = ST_BOUNDS | ST_TARIFF | ST_YEARS | ST_SCRATCH | ST_UNIT | ST_DEMAND

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f64 = ctypes.c_double


class Cfg(ctypes.Structure):
    _fields_ = [
        ("skip_demand_charges", _i32), ("force_net_billing", _i32),
        ("nm_yearend_sell_rate", _f64), ("loan_rate_pct", _f64), ("insurance_rate_pct", _f64),
        ("itc_fed_max", _f64), ("depr_sl_years", _i32), ("pad0", _i32),
        ("batt_v_nom", _f64), ("batt_q_full", _f64), ("batt_min_soc", _f64),
        ("batt_max_soc", _f64), ("batt_init_soc", _f64), ("batt_eta_in", _f64),
        ("batt_eta_out", _f64), ("batt_update_hours", _i32), ("batt_loss_model", _i32),
        ("batt_r_cell", _f64), ("batt_conv_eff", _f64), ("batt_v_cell_empty", _f64),
        ("batt_v_cell_full", _f64), ("batt_month_floor", _i32), ("pad1", _i32),
    ]


class Tables(ctypes.Structure):
    _fields_ = [
        ("shapes", _vp), ("shape_sum", _vp), ("shape_slots", _vp),
        ("cfs", _vp), ("cf_naep", _vp), ("cf_slots", _vp),
        ("wholesale", _vp), ("tariffs", _vp), ("switches", _vp),
        ("n_shapes", _i64), ("n_cfs", _i64), ("n_wholesale", _i64), ("n_switches", _i64),
        ("n_tariffs", _i32), ("max_periods", _i32),
        ("demand", _vp), ("n_demand", _i32), ("peak_units", _i32),
        ("max_dc_periods", _i32), ("no_net", _i32), ("pad_t", _i32),
        ("bt_tariff", _vp), ("bt_shape_max", _vp), ("bt_cf_max", _vp), ("bt_ts_max", _vp),
    ]


AGENT_COLUMNS = [
    # (name, numpy dtype)
    ("load_row", "int32"), ("cf_row", "int32"), ("wholesale_row", "int32"), ("tariff0", "int32"),
    ("sw_solar_off", "int32"), ("sw_solar_cnt", "int32"), ("sw_storage_off", "int32"),
    ("sw_storage_cnt", "int32"), ("scratch_slot", "int32"), ("flags", "uint8"),
    ("econ_life", "int32"), ("loan_term", "int32"), ("load_kwh", "float64"),
    ("price_mult", "float64"), ("inflation", "float64"), ("pv_deg", "float64"),
    ("escalator", "float64"), ("down_payment", "float64"), ("tax_rate", "float64"),
    ("real_discount", "float64"), ("itc_frac", "float64"), ("capex", "float64"),
    ("capex_combined", "float64"), ("batt_capex_kwh", "float64"), ("ccm", "float64"),
    ("vor", "float64"),
]


class Agents(ctypes.Structure):
    _fields_ = [(name, _vp) for name, _ in AGENT_COLUMNS] + [("max_years", _i32)]


OUTPUT_SCALARS = [
    ("system_kw", "float64"), ("x_last", "float64"), ("annual_kwh", "float64"),
    ("naep", "float64"), ("capacity_factor", "float64"), ("price_per_kwh", "float64"),
    ("npv", "float64"), ("payback_raw", "float64"), ("payback_period", "float64"),
    ("first_with", "float64"), ("first_without", "float64"), ("batt_kw", "float64"),
    ("batt_kwh", "float64"), ("npv_pv_batt", "float64"), ("nfev", "int32"),
    ("tariff_final", "int32"), ("switched", "int32"), ("status", "int32"),
]
OUTPUT_YEARLY = ["cash_flow", "cfev_pv", "bill_w_pv", "bill_wo_pv", "cfev_batt", "bill_w_batt",
                 "bill_wo_batt"]
OUTPUT_HOURLY = ["baseline", "net_pvonly", "net_with_batt"]


class Outputs(ctypes.Structure):
    _fields_ = ([(name, _vp) for name, _ in OUTPUT_SCALARS]
                + [(name, _vp) for name in OUTPUT_YEARLY]
                + [(name, _vp) for name in OUTPUT_HOURLY]
                + [("hourly_f64", ctypes.c_int32), ("pad_", ctypes.c_int32)])


class DgenError(RuntimeError):
    pass


_LIB: Optional[ctypes.CDLL] = None

ABI_VERSION = 14   # include/dgen_hip.h DGEN_ABI_VERSION
DEFAULT_CHUNKS = 1   # include/dgen_hip.h DGEN_DEFAULT_CHUNKS
DEFAULT_HOURLY_MONTHS = 1   # include/dgen_hip.h DGEN_DEFAULT_HOURLY_MONTHS
DEFAULT_HOURLY_SPLIT = 2   # include/dgen_hip.h DGEN_DEFAULT_HOURLY_SPLIT

EXPORTED = [
    "dgen_abi_version", "dgen_last_error", "dgen_open", "dgen_close", "dgen_prep_shapes",
    "dgen_prep_cfs", "dgen_workspace_bytes", "dgen_size_agents", "dgen_brent_selftest",
    "dgen_kernel_times", "dgen_last_paths", "dgen_set_dc_prebuild", "dgen_segment_sums", "dgen_max_market_share", "dgen_diffusion",
    "dgen_set_pipeline", "dgen_set_hourly_segment", "dgen_set_battery", "dgen_set_nb_scan", "dgen_set_ts_rows", "dgen_set_nem_rows", "dgen_set_dc_records", "dgen_set_exact", "dgen_exact_count", "dgen_hourly_planes", "dgen_export_plane", "dgen_state_hourly_rows", "dgen_batt_attach", "dgen_export_weights", "dgen_state_hourly",
    "dgen_finance_series", "dgen_year_inputs", "dgen_initial_market_shares", "dgen_rows_seq_sum",
]


def lib_path() -> str:
    # DGEN_LIB: load an alternative build (ablation / A-B timing of kernel variants)
    return os.environ.get("DGEN_LIB") or _build.OUT


def load(build_if_missing: bool = True) -> ctypes.CDLL:
    """Load libdgen_hip.so; build it first if it is missing and hipcc exists."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = lib_path()
    if not os.path.exists(path):
        if not build_if_missing:
            raise DgenError(f"{path} is missing: run python -m dgen_amd.build")
        _build.build()
    L = ctypes.CDLL(path)
    L.dgen_abi_version.restype = _i32
    L.dgen_last_error.restype = _i32
    L.dgen_last_error.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    L.dgen_open.restype = _i32
    L.dgen_open.argtypes = [_i32, ctypes.POINTER(Cfg), ctypes.POINTER(_vp)]
    L.dgen_close.restype = _i32
    L.dgen_close.argtypes = [_vp]
    L.dgen_prep_shapes.restype = _i32
    L.dgen_prep_shapes.argtypes = [_vp, _vp, _i64, _vp, _vp, _vp]
    L.dgen_prep_cfs.restype = _i32
    L.dgen_prep_cfs.argtypes = [_vp, _vp, _i64, _vp, _vp, _vp]
    L.dgen_workspace_bytes.restype = ctypes.c_size_t
    L.dgen_workspace_bytes.argtypes = [_i64, _i64]
    L.dgen_size_agents.restype = _i32
    L.dgen_size_agents.argtypes = [_vp, ctypes.POINTER(Tables), ctypes.POINTER(Agents),
                                   ctypes.POINTER(Outputs), _i64, _vp, ctypes.c_size_t, _i64, _vp]
    L.dgen_brent_selftest.restype = _i32
    L.dgen_brent_selftest.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _i32, _vp,
                                      _vp, _vp]
    L.dgen_set_dc_prebuild.restype = _i32
    L.dgen_set_dc_prebuild.argtypes = [_vp, _i32]
    L.dgen_last_paths.restype = _i32
    L.dgen_last_paths.argtypes = [_vp, ctypes.POINTER(_i32), _i32]
    L.dgen_kernel_times.restype = _i32
    L.dgen_kernel_times.argtypes = [_vp, ctypes.POINTER(_f64), ctypes.POINTER(_f64),
                                    ctypes.POINTER(_f64)]
    L.dgen_set_pipeline.restype = _i32
    L.dgen_set_pipeline.argtypes = [_vp, _i32]
    L.dgen_finance_series.restype = _i32
    L.dgen_finance_series.argtypes = [_vp, ctypes.POINTER(Outputs), _vp, _i64, _vp, _vp]
    L.dgen_set_hourly_segment.restype = _i32
    L.dgen_set_hourly_segment.argtypes = [_vp, _i32]
    L.dgen_set_battery.restype = _i32
    L.dgen_set_battery.argtypes = [_vp, _i32]
    L.dgen_set_nb_scan.restype = _i32
    L.dgen_set_nb_scan.argtypes = [_vp, _i32]
    L.dgen_set_ts_rows.restype = _i32
    L.dgen_set_ts_rows.argtypes = [_vp, _i64, _i64]
    L.dgen_set_nem_rows.restype = _i32
    L.dgen_set_nem_rows.argtypes = [_vp, _i64]
    L.dgen_set_dc_records.restype = _i32
    L.dgen_set_dc_records.argtypes = [_vp, _i32]
    L.dgen_set_exact.restype = _i32
    L.dgen_set_exact.argtypes = [_vp, _i32]
    L.dgen_exact_count.restype = _i32
    L.dgen_exact_count.argtypes = [_vp, ctypes.POINTER(ctypes.c_int64)]
    L.dgen_hourly_planes.restype = _i32
    L.dgen_hourly_planes.argtypes = L.dgen_size_agents.argtypes
    L.dgen_export_plane.restype = _i32
    L.dgen_export_plane.argtypes = [_vp, ctypes.POINTER(Tables), ctypes.POINTER(Agents), ctypes.POINTER(Outputs),
                                    _vp, _vp, _vp, _vp, _i64, _vp, ctypes.c_size_t, _i64, _vp]
    L.dgen_state_hourly_rows.restype = _i32
    L.dgen_state_hourly_rows.argtypes = [_vp, ctypes.POINTER(Tables), ctypes.POINTER(Agents), ctypes.POINTER(Outputs),
                                         _vp, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp]
    L.dgen_segment_sums.restype = _i32
    L.dgen_segment_sums.argtypes = [_vp, _vp, _vp, _vp, _vp, _i32, _i32, _i64, _vp, _i64, _vp, _vp]
    L.dgen_rows_seq_sum.restype = _i32
    L.dgen_rows_seq_sum.argtypes = [_vp, _vp, _i64, _vp, _i64, _vp, _vp]
    if L.dgen_abi_version() != ABI_VERSION:
        raise DgenError("libdgen_hip.so ABI version mismatch")
    _LIB = L
    return L


def last_error() -> str:
    buf = ctypes.create_string_buffer(512)
    load().dgen_last_error(buf, 512)
    return buf.value.decode(errors="replace")


def check(rc: int, what: str) -> int:
    if rc < 0:
        raise DgenError(f"{what} failed ({rc}): {last_error()}")
    return rc
