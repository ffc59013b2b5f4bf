"""Device engine: resident profile/tariff tables + batched sizing on one GPU.

PyTorch-ROCm is used only for device memory and the stream; all compute is in
libdgen_hip.so (hand-written gfx950 kernels) reached through the C-ABI.  There
is no CPU fallback: without a HIP device or the library every call raises.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np

from . import _lib
from .config import EngineConfig

SWITCH_DTYPE = np.dtype([("min_kw", "<f8"), ("max_kw", "<f8"), ("one_time_charge", "<f8"),
                         ("tariff", "<i4"), ("pad", "<i4")])


def _torch():
    import torch
    return torch


def _ptr(t) -> Optional[int]:
    return None if t is None else int(t.data_ptr())


@dataclass
class AgentBatch:
    n: int
    n_scratch: int
    cols: Dict[str, object]          # name -> device tensor
    workspace: object                # uint8 device tensor
    c_agents: _lib.Agents = field(default=None)
    # device row j holds caller agent perm[j] (None: caller order)
    perm: Optional[np.ndarray] = None
    # build the battery case's net-billing split in the hourly scan (dgen_set_nb_scan)
    nb_scan: bool = True
    # device rows holding every TS-capable agent (dgen_set_ts_rows)
    ts_rows: tuple = (0, 2 ** 62)
    # no agent can bill net hourly (dgen_tables.no_net, Engine._no_net_of)
    no_net: bool = False
    # leading device rows without a scratch slot (dgen_set_nem_rows)
    nem_rows: int = 0
    # Engine._tables_gen when no_net / nb_scan were decided: a later
    # set_tariffs / set_switches makes size() fall back to the general forms
    tables_gen: int = 0


def path_class(cols: Dict[str, np.ndarray]) -> np.ndarray:
    """The battery case's billing path per agent, from its columns: 0 = bins
    only (NEM, no scratch slot), 1 = hourly imports billed from the split the
    scan builds (a scratch slot, no TS sell rate: CA or no wholesale row), 2 =
    the other scratch-slot agents (TS sell rate, demand charges).  k_hourly_batt
    runs one agent per lane, and the paths' per-hour work differs (bins vs
    classification vs plane stores): grouped, a wave runs one of them."""
    sl = np.asarray(cols["scratch_slot"]) >= 0
    ts = (np.asarray(cols["wholesale_row"]) >= 0) & ((np.asarray(cols["flags"]) & 2) == 0)
    return np.where(~sl, 0, np.where(ts, 2, 1)).astype(np.int8)


def profile_order(cols: Dict[str, np.ndarray], major: str = "load",
                  group: Optional[np.ndarray] = None, by_path: bool = True) -> np.ndarray:
    """Device order for a batch: agents grouped by (load_row, cf_row)
    (major="cf": by (cf_row, load_row)).

    k_hourly_batt runs one agent per lane and streams the agent's two profile
    rows day by day; when the 64 lanes of a wave share a row, its loads are one
    broadcast line instead of 64.  Load-major shares the larger table (the
    load shapes) inside a wave and leaves the per-lane reads on the smaller cf
    table, which stays cache-resident (measured at 1M agents: 35.2 ms vs
    38.0 ms cf-major, 45.3 ms caller order).  The
    reference's agent order carries no meaning (size_chunk returns rows keyed
    by agent_id, ff:1149-1218), so the host columnarizer is free to choose it.
    by_path: the battery case's billing path (path_class) is the next key
    out, so a wave's lanes run one path of the scan (and the scan-built
    net-billing split is decided per agent, not per batch).  group (optional)
    is the outermost key: the model-year loop passes the state so each state's
    members are one contiguous column range of the hourly planes and
    k_state_hourly streams them coalesced.  Stable, so ties keep caller
    order."""
    lr, cr = np.asarray(cols["load_row"]), np.asarray(cols["cf_row"])
    keys = (lr, cr) if major == "cf" else (cr, lr)
    if by_path:
        keys = keys + (path_class(cols),)
    if group is not None:
        keys = keys + (np.asarray(group),)
    return np.lexsort(keys).astype(np.int64)


def tariff_price_bounds(recs: np.ndarray, dem: Optional[np.ndarray]) -> np.ndarray:
    """dgen_tables.bt_tariff: per tariff [max |buy|, |sell| over its periods
    and tiers ($/kWh); the largest month's flat demand price + every TOU
    period's ($/kW, 0 without a demand record); the kWh/kW tier caps'
    sensitivity to the month peak (2 x energy price x sum of caps, x 31 for
    daily caps; 0 for other units)] -- the certified Brent paths' bounds
    (k_brent_certify)."""
    n = recs.size
    out = np.zeros((n, 3), np.float64)
    for j in range(n):
        r = recs[j]
        P, T = int(r["P"]), int(r["T"])
        e = max(float(np.abs(r["buy"][:P, :T]).max(initial=0.0)), float(np.abs(r["sell"][:P, :T]).max(initial=0.0)))
        out[j, 0] = e
        dc = int(r["dc"])
        if dem is not None and 0 < dc <= len(dem):
            d = dem[dc - 1]
            tou = sum(float(np.abs(d["tou_price"][p, :int(d["tou_nt"][p])]).max(initial=0.0))
                      for p in range(d["tou_price"].shape[0]))
            flat = max(float(np.abs(d["flat_price"][m, :int(d["flat_nt"][m])]).max(initial=0.0)) for m in range(12))
            out[j, 1] = flat + tou
        u = int(r["unit"])
        if u in (1, 3):
            out[j, 2] = 2.0 * e * float(np.abs(r["cap"][:T]).sum()) * (31.0 if u == 3 else 1.0)
    return out


class Engine:
    def __init__(self, device: int = 0, cfg: Optional[EngineConfig] = None):
        torch = _torch()
        if not torch.cuda.is_available():
            raise _lib.DgenError("no HIP device visible: the dGen MI355X engine has no CPU path")
        self.lib = _lib.load()
        self.device = int(device)
        self.cfg = cfg or EngineConfig()
        torch.cuda.set_device(self.device)
        self.dev = torch.device("cuda", self.device)
        h = ctypes.c_void_p()
        c = self.cfg.to_c()
        _lib.check(self.lib.dgen_open(self.device, ctypes.byref(c), ctypes.byref(h)), "dgen_open")
        self.ctx = h
        _lib.check(self.lib.dgen_set_exact(self.ctx, self.cfg.exact_mode()), "dgen_set_exact")
        self.tables = _lib.Tables()
        self.chunks = _lib.DEFAULT_CHUNKS
        self.hb_months = _lib.DEFAULT_HOURLY_MONTHS
        self.battery = True
        self._keep: Dict[str, object] = {}
        self._tables_gen = 0            # bumped by set_tariffs / set_switches

    # ------------------------------------------------------------------ utils
    def stream_handle(self) -> int:
        return int(_torch().cuda.current_stream(self.dev).cuda_stream)

    def _to_dev(self, a, dtype):
        torch = _torch()
        if isinstance(a, torch.Tensor):
            return a.to(device=self.dev, dtype=dtype).contiguous()
        return torch.from_numpy(np.array(a, copy=True, order="C")).to(device=self.dev, dtype=dtype)

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.dgen_close(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ----------------------------------------------------------------- tables
    def load_profiles(self, shapes, cfs, wholesale=None):
        """Upload kwh_load_profile rows (float32 [R, 8760]), solar cf x 1e6 rows
        (int32 [C, 8760]) and optional wholesale $/kWh rows (float64 [W, 8760]);
        precompute numpy-order row sums and slot sums on device."""
        torch = _torch()
        sh = self._to_dev(shapes, torch.float32)
        cf = self._to_dev(cfs, torch.int32)
        if sh.dim() != 2 or sh.shape[1] != _lib.NH or cf.dim() != 2 or cf.shape[1] != _lib.NH:
            raise ValueError("profile tables must be [rows, 8760]")
        R, C = sh.shape[0], cf.shape[0]
        s_sum = torch.empty(R, dtype=torch.float64, device=self.dev)
        s_slots = torch.empty((R, _lib.NSLOT), dtype=torch.float64, device=self.dev)
        c_naep = torch.empty(C, dtype=torch.float64, device=self.dev)
        c_slots = torch.empty((C, _lib.NSLOT), dtype=torch.float64, device=self.dev)
        st = self.stream_handle()
        _lib.check(self.lib.dgen_prep_shapes(self.ctx, _ptr(sh), R, _ptr(s_sum), _ptr(s_slots), st),
                   "dgen_prep_shapes")
        _lib.check(self.lib.dgen_prep_cfs(self.ctx, _ptr(cf), C, _ptr(c_naep), _ptr(c_slots), st),
                   "dgen_prep_cfs")
        ws = None
        if wholesale is not None and len(wholesale):
            ws = self._to_dev(wholesale, torch.float64)
            if ws.dim() != 2 or ws.shape[1] != _lib.NH:
                raise ValueError("wholesale table must be [rows, 8760]")
        # row maxima for the certified Brent paths' error bounds (dgen_set_exact)
        sh_max = sh.abs().amax(dim=1).to(torch.float64).contiguous()
        cf_max = cf.abs().amax(dim=1).to(torch.float64).contiguous()
        ws_max = (torch.nan_to_num(ws.abs(), nan=0.0, posinf=0.0).amax(dim=1).contiguous()
                  if ws is not None else None)
        self._keep.update(shapes=sh, shape_sum=s_sum, shape_slots=s_slots, cfs=cf,
                          cf_naep=c_naep, cf_slots=c_slots, wholesale=ws,
                          bt_shape_max=sh_max, bt_cf_max=cf_max, bt_ts_max=ws_max)
        T = self.tables
        T.shapes, T.shape_sum, T.shape_slots = _ptr(sh), _ptr(s_sum), _ptr(s_slots)
        T.cfs, T.cf_naep, T.cf_slots = _ptr(cf), _ptr(c_naep), _ptr(c_slots)
        T.wholesale = _ptr(ws)
        T.bt_shape_max, T.bt_cf_max, T.bt_ts_max = _ptr(sh_max), _ptr(cf_max), _ptr(ws_max)
        T.n_shapes, T.n_cfs = R, C
        T.n_wholesale = 0 if ws is None else ws.shape[0]

    def set_tariffs(self, records: np.ndarray, demand: Optional[np.ndarray] = None):
        """Upload compiled tariff records (+ the demand-charge records their
        ``dc`` field indexes, TariffTable.demand_array(); billed only when the
        engine's cfg.skip_demand_charges is 0).  Tariffs whose tiers are in
        kWh/kW get a zero-charge record for their month peaks when they have
        none (tariff.attach_peak_records)."""
        from .tariff import TARIFF_DTYPE, attach_peak_records
        recs = np.ascontiguousarray(records, dtype=TARIFF_DTYPE)
        if recs.size == 0:
            raise ValueError("empty tariff table")
        self._tariff_mo = recs["mo"].copy()
        # kWh/kW tier units (codes 1, 3): month peaks from a demand record
        recs, dem, peak_units = attach_peak_records(recs, demand)
        self.tables.peak_units = int(peak_units)
        if int(recs["dc"].max()) > dem.size or int(recs["dc"].min()) < 0:
            raise ValueError("tariff dc index outside the demand table")
        self.tables.n_demand = int(dem.size)
        self.tables.max_dc_periods = (int(max(dem["wkday"].max(), dem["wkend"].max())) + 1) if dem.size else 0
        self.tables.demand = None
        self._keep.pop("demand", None)
        if dem.size:
            d = self._to_dev(np.frombuffer(dem.tobytes(), dtype=np.uint8), _torch().uint8)
            self._keep["demand"] = d
            self.tables.demand = _ptr(d)
        raw = np.frombuffer(recs.tobytes(), dtype=np.uint8)
        t = self._to_dev(raw, _torch().uint8)
        self._keep["tariffs"] = t
        self.tariff_records = recs
        self.tables.tariffs = _ptr(t)
        bt = self._to_dev(tariff_price_bounds(recs, dem), _torch().float64)
        self._keep["bt_tariff"] = bt
        self.tables.bt_tariff = _ptr(bt)
        self.tables.n_tariffs = int(recs.size)
        self.tables.max_periods = int(recs["P"].max())
        self.tables.no_net = 0                # set per batch by size() (AgentBatch.no_net)
        self._tables_gen += 1

    def set_switches(self, sw: np.ndarray):
        sw = np.ascontiguousarray(sw, dtype=SWITCH_DTYPE)
        if sw.size == 0:
            sw = np.zeros(1, dtype=SWITCH_DTYPE)
        raw = np.frombuffer(sw.tobytes(), dtype=np.uint8)
        t = self._to_dev(raw, _torch().uint8)
        self._keep["switches"] = t
        self.tables.switches = _ptr(t)
        self.tables.n_switches = int(sw.size)
        self._switch_tariff = sw["tariff"].copy()
        self._tables_gen += 1

    def profile_sums(self):
        """(shape row sums, cf naep) as host arrays (for tests / host checks)."""
        return (self._keep["shape_sum"].cpu().numpy(), self._keep["cf_naep"].cpu().numpy())

    # ------------------------------------------------------------------ batch
    def upload_agents(self, cols: Dict[str, np.ndarray], n_scratch: Optional[int] = None,
                      order: Optional[np.ndarray] = None) -> AgentBatch:
        """Upload agent columns.  `order` (a permutation, e.g. profile_order(cols))
        lays the batch out on device as cols[...][order]; outputs then come back in
        that order and outputs_to_host(out, batch.perm) restores caller order."""
        torch = _torch()
        n = len(cols["load_kwh"])
        if order is not None:
            order = np.asarray(order, dtype=np.int64)
            if order.shape != (n,) or not np.array_equal(np.sort(order), np.arange(n)):
                raise ValueError("order must be a permutation of range(n)")
            cols = {k: np.asarray(v)[order] for k, v in cols.items()}
            # scratch slots renumbered in device order: the workspace plane is
            # [365][n_scratch][24], so neighbouring lanes then store to
            # neighbouring slots (a wave's day is one contiguous 12 KB run)
            sl = np.asarray(cols["scratch_slot"])
            need = sl >= 0
            renum = np.full(n, -1, dtype=np.int32)
            renum[need] = np.arange(int(need.sum()), dtype=np.int32)
            cols["scratch_slot"] = renum
        dev = {}
        tmap = {"int32": torch.int32, "uint8": torch.uint8, "float64": torch.float64}
        for name, dt in _lib.AGENT_COLUMNS:
            if name not in cols:
                raise KeyError(f"agent column {name!r} missing")
            v = cols[name]
            if len(v) != n:
                raise ValueError(f"agent column {name!r} has length {len(v)} != {n}")
            dev[name] = self._to_dev(np.asarray(v, dtype=dt) if not isinstance(v, torch.Tensor) else v,
                                     tmap[dt])
        if n_scratch is None:
            slots = dev["scratch_slot"]
            n_scratch = int(slots.max().item()) + 1 if n > 0 else 0
            n_scratch = max(n_scratch, 0)
        self.validate_agents(dev, n)
        wsb = int(self.lib.dgen_workspace_bytes(n, n_scratch))
        ws = torch.empty(max(wsb, 8), dtype=torch.uint8, device=self.dev)
        ca = _lib.Agents(**{name: _ptr(dev[name]) for name, _ in _lib.AGENT_COLUMNS})
        ca.max_years = int(dev["econ_life"].max().item()) if n else 0
        return AgentBatch(n=n, n_scratch=n_scratch, cols=dev, workspace=ws, c_agents=ca, perm=order,
                          nb_scan=self._nb_scan_pays(cols, n, n_scratch), ts_rows=self._ts_rows_of(cols, n),
                          no_net=self._no_net_of(cols, n), nem_rows=self._nem_rows_of(cols, n),
                          tables_gen=self._tables_gen)

    def _nem_rows_of(self, cols, n: int) -> int:
        """dgen_set_nem_rows: the length of the batch's leading run of device
        rows without a scratch slot (bins-only agents; profile_order puts them
        first), which a batch with scratch slots sizes with the bins-only
        kernels.  0 when the columns are not host arrays or DGEN_NEM_SPLIT=0."""
        import os
        if os.environ.get("DGEN_NEM_SPLIT", "1") == "0":
            return 0
        try:
            sl = np.asarray(cols["scratch_slot"])
        except Exception:
            return 0
        if sl.ndim != 1 or sl.size != n:
            return 0
        has = np.flatnonzero(sl >= 0)
        return int(has[0]) if has.size else n

    def _ts_rows_of(self, cols, n: int):
        """dgen_set_ts_rows: the device rows [lo, hi) holding every agent that
        can bill the TS sell rate (path_class 2); (0, 0) when there is none.
        Host columns only (device tensors: the whole batch)."""
        try:
            pc = path_class(cols)
        except Exception:
            return (0, 2 ** 62)
        ix = np.flatnonzero(pc == 2)
        return (int(ix[0]), int(ix[-1]) + 1) if ix.size else (0, 0)

    def _no_net_of(self, cols, n: int) -> bool:
        """True when no agent of the batch can bill net hourly (metering
        options 2, 3): neither its initial tariff nor any rate-switch candidate
        (solar or storage rows).  dgen_tables.no_net then lets the demand-charge
        kernels run their instantiations without the net-billing paths (fewer
        registers; results identical, the paths are unreachable).  False when
        the tariff or switch table is unknown."""
        mo = getattr(self, "_tariff_mo", None)
        if mo is None or n == 0:
            return False
        net = np.isin(mo, (2, 3))
        if not net.any():
            return True
        try:                   # device-tensor columns: keep the net-billing forms
            t0 = np.asarray(cols["tariff0"], np.int64)
            offs = {k: (np.asarray(cols[f"sw_{k}_off"], np.int64), np.asarray(cols[f"sw_{k}_cnt"], np.int64))
                    for k in ("solar", "storage")}
        except Exception:
            return False
        if ((t0 < 0) | (t0 >= net.size)).any() or net[t0].any():
            return False
        swt = getattr(self, "_switch_tariff", None)
        if swt is None:
            return False
        sw_net = np.zeros(swt.size, bool)
        okr = (swt >= 0) & (swt < net.size)
        sw_net[okr] = net[swt[okr]]
        csum = np.concatenate([[0], np.cumsum(sw_net.astype(np.int64))])
        for off, cnt in offs.values():
            lo = np.clip(off, 0, swt.size)
            hi = np.clip(off + cnt, 0, swt.size)
            if ((csum[hi] - csum[lo]) > 0).any():
                return False
        return True

    def _nb_scan_pays(self, cols, n: int, n_scratch: int) -> bool:
        """dgen_set_nb_scan: the battery case's net-billing split is built in
        the hourly scan for every agent that bills net (the scan decides per
        agent; profile_order groups those agents into their own waves; the TS
        sell-rate agents get a scan of their own when hourly planes are
        requested, dgen_size_agents' ts_split), so an agent's battery-case
        outputs do not depend on the other agents of its batch.  They do
        depend on the hourly flag for the TS agents: without planes their split
        comes from k_batt_finance's plane pass, whose sums re-associate (the
        four battery-case money outputs move by ~1e-9 relative; sizing and
        every discrete decision are the same bits,
        test_ts_agent_outputs_with_and_without_planes).  The scan form
        is compiled in only when the batch holds such an agent (its
        instantiation carries the export sums: more registers, and with the
        demand records a spill), which changes no result.  DGEN_NB_SCAN=0 turns it off (A/B: the finance kernel's build
        over the system-output plane; the two builds re-associate the split's
        sums, ~1e-9 relative on the battery-case bills and NPV)."""
        import os
        if os.environ.get("DGEN_NB_SCAN", "1") == "0":
            return False
        mo_t = getattr(self, "_tariff_mo", None)
        if n == 0 or n_scratch == 0 or mo_t is None:
            return n_scratch > 0
        try:
            sl = np.asarray(cols["scratch_slot"])
            mo = mo_t[np.asarray(cols["tariff0"], np.int64)]
        except Exception:          # device-tensor columns: keep it on
            return True
        return bool(((sl >= 0) & ((mo == 2) | (mo == 3))).any())

    def validate_agents(self, dev, n):
        """Host-side bounds checks before any kernel indexes a table."""
        T = self.tables
        if T.n_tariffs <= 0 or not T.shapes:
            raise _lib.DgenError("tables not loaded")
        def rng(name, lo, hi):
            v = dev[name]
            if n and (int(v.min().item()) < lo or int(v.max().item()) >= hi):
                raise ValueError(f"agent column {name!r} out of range [{lo}, {hi})")
        rng("load_row", 0, T.n_shapes)
        rng("cf_row", 0, T.n_cfs)
        rng("wholesale_row", -1, max(T.n_wholesale, 0))
        rng("tariff0", 0, T.n_tariffs)
        for k in ("solar", "storage"):
            off, cnt = dev[f"sw_{k}_off"], dev[f"sw_{k}_cnt"]
            if n and (int(off.min().item()) < 0 or int(cnt.min().item()) < 0
                      or int((off.long() + cnt.long()).max().item()) > T.n_switches):
                raise ValueError(f"rate-switch ({k}) offsets out of range")

    def alloc_outputs(self, n: int, hourly=True, hourly_f64: bool = False) -> Dict[str, object]:
        """Device output buffers for n agents.  hourly_f64: the three hourly
        planes as float64 (the reference's fp64 lists, the kernels' own
        values) instead of float32 (half the bytes; the default).  hourly
        "with_batt": the with-battery plane alone (float32; the model-year
        loop's export, attachment.state_hourly_rows)."""
        torch = _torch()
        out = {}
        for name, dt in _lib.OUTPUT_SCALARS:
            out[name] = torch.empty(n, dtype=torch.float64 if dt == "float64" else torch.int32,
                                    device=self.dev)
        for name in _lib.OUTPUT_YEARLY:
            out[name] = torch.zeros((n, _lib.MAXY + 1), dtype=torch.float64, device=self.dev)
        for name in _lib.OUTPUT_HOURLY:
            # hour-quad tiles (include/dgen_hip.h): [NH / 4][n][4]
            want = hourly is True or (hourly == "with_batt" and name == "net_with_batt")
            out[name] = (torch.empty((_lib.NH // 4, n, 4), dtype=torch.float64 if hourly_f64 else torch.float32,
                                     device=self.dev) if want else None)
        return out

    @staticmethod
    def c_outputs(out: Dict[str, object]) -> _lib.Outputs:
        fields = {name: _ptr(out[name]) for name, _ in _lib.OUTPUT_SCALARS}
        fields.update({name: _ptr(out[name]) for name in _lib.OUTPUT_YEARLY})
        fields.update({name: _ptr(out.get(name)) for name in _lib.OUTPUT_HOURLY})
        planes = [out.get(name) for name in _lib.OUTPUT_HOURLY if out.get(name) is not None]
        dts = {p.dtype for p in planes}
        if len(dts) > 1:
            raise TypeError("hourly planes must share one dtype")
        torch = _torch()
        fields["hourly_f64"] = int(bool(planes) and planes[0].dtype == torch.float64)
        return _lib.Outputs(**fields)

    def size(self, batch: AgentBatch, out: Dict[str, object], c_out: Optional[_lib.Outputs] = None):
        """Launch the sizing kernels for `batch` on the current stream (async)."""
        co = c_out if c_out is not None else self.c_outputs(out)
        # no_net / nb_scan were decided against the tables of upload time; after
        # a set_tariffs / set_switches take the forms that are right for any
        # table (the net-billing instantiations, the scan-built split on)
        fresh = batch.tables_gen == self._tables_gen
        self.tables.no_net = int(batch.no_net and fresh)
        nb_scan = batch.nb_scan or (not fresh and batch.n_scratch > 0)
        if nb_scan != getattr(self, "_nb_scan", True):
            _lib.check(self.lib.dgen_set_nb_scan(self.ctx, _lib.NB_CAPM if nb_scan else 0),
                       "dgen_set_nb_scan")
            self._nb_scan = nb_scan
        if int(batch.nem_rows) != getattr(self, "_nem_rows", 0):
            _lib.check(self.lib.dgen_set_nem_rows(self.ctx, int(batch.nem_rows)), "dgen_set_nem_rows")
            self._nem_rows = int(batch.nem_rows)
        if tuple(batch.ts_rows) != getattr(self, "_ts_rows", (0, 2 ** 62)):
            _lib.check(self.lib.dgen_set_ts_rows(self.ctx, int(batch.ts_rows[0]), int(batch.ts_rows[1])),
                       "dgen_set_ts_rows")
            self._ts_rows = tuple(batch.ts_rows)
        _lib.check(self.lib.dgen_size_agents(self.ctx, ctypes.byref(self.tables),
                                             ctypes.byref(batch.c_agents), ctypes.byref(co),
                                             batch.n, _ptr(batch.workspace),
                                             batch.workspace.numel(), batch.n_scratch,
                                             self.stream_handle()),
                   "dgen_size_agents")

    def hourly_planes(self, batch: AgentBatch, c_out: _lib.Outputs):
        """The hourly planes of `batch`, already sized with the outputs `c_out`
        points to (async, dgen_hourly_planes): the 8760-h scan alone."""
        _lib.check(self.lib.dgen_hourly_planes(self.ctx, ctypes.byref(self.tables),
                                               ctypes.byref(batch.c_agents), ctypes.byref(c_out),
                                               batch.n, _ptr(batch.workspace), batch.workspace.numel(),
                                               batch.n_scratch, self.stream_handle()),
                   "dgen_hourly_planes")

    def export_plane(self, batch: AgentBatch, c_out: _lib.Outputs, weights, plane) -> bool:
        """The per-state export's combined plane of `batch` (already sized with
        the outputs `c_out` points to; async, dgen_export_plane): the 8760-h scan
        alone, writing per agent-hour the f64 value dgen_state_hourly adds from
        the three planes, into `plane` (float64 hour-quad tiles [NH/4, n, 4]).
        False (nothing launched) for the loss model and the hourly re-plan,
        whose scans export through hourly_planes."""
        if self.cfg.batt_loss_model == 1 or self.cfg.batt_update_hours == 1:
            return False
        w = [x.contiguous() for x in weights]
        if any(x.numel() != batch.n for x in w) or plane.numel() < _lib.NH * batch.n:
            raise ValueError("export_plane: one weight per agent and NH x n plane values")
        _lib.check(self.lib.dgen_export_plane(self.ctx, ctypes.byref(self.tables), ctypes.byref(batch.c_agents),
                                              ctypes.byref(c_out), _ptr(w[0]), _ptr(w[1]), _ptr(w[2]),
                                              _ptr(plane), batch.n, _ptr(batch.workspace),
                                              batch.workspace.numel(), batch.n_scratch, self.stream_handle()),
                   "dgen_export_plane")
        return True

    def set_pipeline(self, chunks: int):
        """Chunk-pipeline depth of size() (dgen_set_pipeline; 1 = no overlap)."""
        _lib.check(self.lib.dgen_set_pipeline(self.ctx, int(chunks)), "dgen_set_pipeline")
        self.chunks = int(chunks)

    def set_hourly_segment(self, months: int):
        """Months per k_hourly_batt launch (dgen_set_hourly_segment)."""
        _lib.check(self.lib.dgen_set_hourly_segment(self.ctx, int(months)), "dgen_set_hourly_segment")
        self.hb_months = int(months)

    def set_battery(self, on: bool):
        """PV+battery forward run on (the reference, ff:479) or off (the PV-only
        variant, dgen_set_battery)."""
        _lib.check(self.lib.dgen_set_battery(self.ctx, int(bool(on))), "dgen_set_battery")
        self.battery = bool(on)

    def set_dc_records(self, cap=True):
        """Battery-case demand records built in the hourly scan
        (dgen_set_dc_records): True = DGEN_DCR_CAP kept hours per agent (the
        default), an int = that capacity (an agent beyond it falls back), False
        = the finance kernel's staged pass over all 8760 hours of the
        system-output plane.  Results are bit-identical."""
        c = _lib.DCR_CAP if cap is True else int(cap)
        _lib.check(self.lib.dgen_set_dc_records(self.ctx, c), "dgen_set_dc_records")

    def set_dc_prebuild(self, on: bool = True):
        """Demand envelopes of the first-evaluation tariffs prebuilt by their
        own kernel (default) or built inside the search (dgen_set_dc_prebuild;
        bit-identical results)."""
        _lib.check(self.lib.dgen_set_dc_prebuild(self.ctx, 1 if on else 0), "dgen_set_dc_prebuild")

    def last_paths(self) -> Dict[str, int]:
        """The record forms the last size() call took (dgen_last_paths): what
        the kernels actually did, for the bench's byte accounting."""
        a = (ctypes.c_int32 * 7)()
        _lib.check(self.lib.dgen_last_paths(self.ctx, a, 7), "dgen_last_paths")
        keys = ("nb_scan", "dcr_on", "ts_split", "dc", "max_periods", "dc_periods", "dc_prebuild")
        return dict(zip(keys, (int(v) for v in a)))

    def set_exact(self, mode: int):
        """Certified Brent paths (dgen_set_exact): 1 (default) re-runs the
        agents whose search a device/oracle difference bound does not settle
        in the reference's arithmetic, 2 every agent, 0 none."""
        _lib.check(self.lib.dgen_set_exact(self.ctx, int(mode)), "dgen_set_exact")
        self.cfg.exact_brent = int(mode)

    def exact_count(self) -> int:
        """Agents the last size() call re-ran in the reference's arithmetic
        (synchronises the device)."""
        v = ctypes.c_int64(0)
        _lib.check(self.lib.dgen_exact_count(self.ctx, ctypes.byref(v)), "dgen_exact_count")
        return int(v.value)

    def kernel_times(self):
        """Average per-launch device time (ms) of the three sizing kernels over
        the calls since the last query, from HIP events on the launch stream."""
        a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        cnt = _lib.check(self.lib.dgen_kernel_times(self.ctx, ctypes.byref(a), ctypes.byref(b),
                                                    ctypes.byref(c)), "dgen_kernel_times")
        return a.value, b.value, c.value, cnt

    def segment_sums(self, v1, seg_off, w1=None, v2=None, w2=None):
        """Weighted sums of k planes of n agents over contiguous segments
        (device, deterministic order).  v1/v2: [k, n] float32/float64 device
        tensors; seg_off: [S+1] offsets; returns a [S, k] float64 device tensor."""
        torch = _torch()
        if v1.dim() == 1:
            v1 = v1.view(1, -1)
            v2 = None if v2 is None else v2.view(1, -1)
        k, n = v1.shape
        f32 = v1.dtype == torch.float32
        if v1.dtype not in (torch.float32, torch.float64) or (v2 is not None and v2.dtype != v1.dtype):
            raise TypeError("segment_sums: values must be float32 or float64 (same dtype)")
        so = self._to_dev(seg_off, torch.int64)
        if so.numel() < 1 or int(so[0].item()) < 0 or int(so[-1].item()) > n or \
                bool((so[1:] < so[:-1]).any().item()):
            raise ValueError("segment offsets must be non-decreasing within [0, n]")
        S = so.numel() - 1
        out = torch.empty((S, k), dtype=torch.float64, device=self.dev)
        f = lambda t: None if t is None else self._to_dev(t, torch.float64)
        w1d, w2d = f(w1), f(w2)
        keep = (v1.contiguous(), None if v2 is None else v2.contiguous(), w1d, w2d)
        _lib.check(self.lib.dgen_segment_sums(self.ctx, _ptr(keep[0]), _ptr(w1d), _ptr(keep[1]),
                                              _ptr(w2d), int(f32), int(k), int(n), _ptr(so), S,
                                              _ptr(out), self.stream_handle()),
                   "dgen_segment_sums")
        torch.cuda.current_stream(self.dev).synchronize()
        del keep
        return out

    def rows_seq_sum(self, rows, seg_off):
        """[R, k] float64 device rows -> [S, k]: each segment's rows added in row
        order (dgen_rows_seq_sum; async on the current stream)."""
        torch = _torch()
        if rows.dtype != torch.float64 or rows.dim() != 2:
            raise TypeError("rows_seq_sum: rows must be a [R, k] float64 tensor")
        so = self._to_dev(np.asarray(seg_off, np.int64), torch.int64)
        S = so.numel() - 1
        if S < 0 or (S > 0 and (int(so[0].item()) < 0 or int(so[-1].item()) > rows.shape[0])):
            raise ValueError("segment offsets outside the rows")
        r = rows.contiguous()
        out = torch.empty((max(S, 0), rows.shape[1]), dtype=torch.float64, device=self.dev)
        _lib.check(self.lib.dgen_rows_seq_sum(self.ctx, _ptr(r), int(rows.shape[1]), _ptr(so), S, _ptr(out),
                                              self.stream_handle()), "dgen_rows_seq_sum")
        self._keep["_seq"] = (r, so)          # alive until the next call (stream order)
        return out

    def brent_selftest(self, lo, hi, xatol, c2, x0, c1, maxn=64):
        torch = _torch()
        f = lambda v: self._to_dev(np.asarray(v, dtype=np.float64), torch.float64)
        tl, th, ta, t2, t0, t1 = (f(v) for v in (lo, hi, xatol, c2, x0, c1))
        n = tl.numel()
        xs = torch.zeros((n, maxn), dtype=torch.float64, device=self.dev)
        xo = torch.zeros(n, dtype=torch.float64, device=self.dev)
        nf = torch.zeros(n, dtype=torch.int32, device=self.dev)
        _lib.check(self.lib.dgen_brent_selftest(self.ctx, _ptr(tl), _ptr(th), _ptr(ta), _ptr(t2),
                                                _ptr(t0), _ptr(t1), n, _ptr(xs), maxn, _ptr(xo),
                                                _ptr(nf), self.stream_handle()),
                   "dgen_brent_selftest")
        torch.cuda.synchronize(self.dev)
        return xs.cpu().numpy(), xo.cpu().numpy(), nf.cpu().numpy()


def hourly_plane(t):
    """A hourly output plane in its device tiles [NH/4][n][4] -> the logical
    time-major [NH][n] (a copy, on the same device)."""
    q, n, four = t.shape
    return t.permute(0, 2, 1).reshape(q * four, n)


def hourly_agent_major(t):
    """Tiled plane [NH/4][n][4] -> [n][NH] (a copy): each agent's 8760-h list."""
    q, n, four = t.shape
    return t.permute(1, 0, 2).reshape(n, q * four)


def tile_hourly(p):
    """Logical time-major [NH][n] plane -> the device tile layout [NH/4][n][4]."""
    nh, n = p.shape
    if nh % 4:
        raise ValueError("hourly planes need a multiple of 4 hours")
    return p.reshape(nh // 4, 4, n).permute(0, 2, 1).contiguous()


_STAGE: Dict[int, object] = {}      # pinned host staging buffers (reused across calls)
_POOL: Dict[str, object] = {}


def _host_empty(shape, dtype) -> np.ndarray:
    """Uninitialised host array on an anonymous mapping advised for huge pages:
    a multi-GB hourly plane is then first-touched 2 MB at a time instead of
    4 KB at a time (the page faults, not the copy, bound a pageable download).
    The mapping lives as long as the array (numpy keeps the buffer)."""
    import mmap
    nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
    if nbytes < (64 << 20):
        return np.empty(shape, dtype)
    m = mmap.mmap(-1, nbytes, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    try:
        m.madvise(14)                   # MADV_HUGEPAGE (advice only)
    except (AttributeError, OSError, ValueError):
        pass
    return np.frombuffer(m, dtype=dtype).reshape(shape)


def _staging(k: int, nbytes: int):
    torch = _torch()
    t = _STAGE.get(k)
    if t is None or t.numel() < nbytes:
        t = _STAGE[k] = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    return t


_D2H_LOCK = None


def hourly_to_host(t, inv=None, chunk: int = 4096, threads: Optional[int] = None) -> np.ndarray:
    """One hour-quad-tiled plane [NH/4][n][4] -> host [n][NH] (caller order when
    `inv` gathers it): per chunk of agents, a device gather into agent-major
    order, an async copy into one of two pinned staging buffers, and host
    threads copying the previous chunk out into the destination while the
    next chunk crosses PCIe.  One download at a time (the staging buffers are
    shared; HostPlane runs it on a background thread), on t's device."""
    global _D2H_LOCK
    import threading
    if _D2H_LOCK is None:
        _D2H_LOCK = threading.Lock()
    torch = _torch()
    with _D2H_LOCK, torch.cuda.device(t.device):
        return _hourly_to_host(t, inv, chunk, threads)


def _hourly_to_host(t, inv, chunk, threads):
    torch = _torch()
    import os
    from concurrent.futures import ThreadPoolExecutor
    if threads is None:
        threads = int(os.environ.get("DGEN_D2H_THREADS", "8"))
    threads = max(1, int(threads))
    q, n, four = t.shape
    ncol = q * four
    rowb = ncol * t.element_size()
    dst = _host_empty((n, ncol), np.float64 if t.dtype == torch.float64 else np.float32)
    if n == 0:
        return dst
    chunk = max(1, min(chunk, n))
    pool = _POOL.get(("copy", threads))
    if pool is None:
        pool = _POOL[("copy", threads)] = ThreadPoolExecutor(threads, thread_name_prefix="dgen-d2h")
    tp = t.permute(1, 0, 2)
    pend = [[], []]
    for k, c0 in enumerate(range(0, n, chunk)):
        c1 = min(n, c0 + chunk)
        m, b = c1 - c0, k & 1
        for f in pend[b]:               # the buffer's previous chunk is out
            f.result()
        g = (tp.index_select(0, inv[c0:c1]) if inv is not None else tp[c0:c1]).reshape(m, ncol)
        hv = _staging(b, chunk * rowb)[: m * rowb].view(t.dtype).view(m, ncol)
        hv.copy_(g, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        hn = hv.numpy()

        def part(lo, hi, ev=ev, hn=hn, c0=c0):
            ev.synchronize()
            np.copyto(dst[c0 + lo:c0 + hi], hn[lo:hi])
        step = -(-m // threads)
        pend[b] = [pool.submit(part, lo, min(m, lo + step)) for lo in range(0, m, step)]
    for p in pend:
        for f in p:
            f.result()
    return dst


class HostPlane:
    """An hourly plane on its way to the host: the download runs on a background
    thread (pinned, chunked, threaded copy-out: hourly_to_host) while the caller
    goes on; result() waits for it and returns the [n][8760] array.  The device
    tensor is released once it has crossed."""

    _pool = None

    def __init__(self, t, inv):
        from concurrent.futures import ThreadPoolExecutor
        if HostPlane._pool is None:
            HostPlane._pool = ThreadPoolExecutor(1, thread_name_prefix="dgen-plane")
        self.n = int(t.shape[1])
        self._fut = HostPlane._pool.submit(hourly_to_host, t, inv)
        self._arr = None

    def result(self) -> np.ndarray:
        if self._arr is None:
            self._arr = self._fut.result()
            self._fut = None
        return self._arr

    def done(self) -> bool:
        return self._arr is not None or self._fut.done()


class DevicePlane:
    """An hourly plane left in HBM (size_frame(hourly="device")): consumers
    that reduce it on the device (attachment.export_state_hourly_with_storage
    _mix) read the tiled tensor in place and it never crosses PCIe; reading a
    cell downloads the whole plane once (result(), like HostPlane's).  Row j
    of the [n][8760] view is device column inv[j] (inv None: j)."""

    def __init__(self, t, inv):
        self.t = t
        self.inv = inv
        self.n = int(t.shape[1])
        self.width = int(t.shape[0]) * int(t.shape[2])      # hours per row, known without a download
        self._arr = None

    def device_columns(self) -> np.ndarray:
        """Device column of each plane row (host int64)."""
        return (np.arange(self.n, dtype=np.int64) if self.inv is None
                else self.inv.cpu().numpy().astype(np.int64))

    def result(self) -> np.ndarray:
        if self._arr is None:
            self._arr = hourly_to_host(self.t, self.inv)
        return self._arr

    def done(self) -> bool:
        return self._arr is not None


def outputs_to_host(out: Dict[str, object], perm: Optional[np.ndarray] = None,
                    hourly_async: bool = False, hourly_device: bool = False) -> Dict[str, object]:
    """Device outputs -> host numpy ([agent][year] yearly arrays, [agent][hour] hourly),
    in caller order when `perm` (AgentBatch.perm) is given.  The reorder to
    caller order (and the hourly tiles' transpose) is one device gather per
    array, so each crosses PCIe once, already in its final layout.
    hourly_async: the hourly planes come back as HostPlane (background
    download) instead of arrays, the scalars and yearly arrays at once;
    hourly_device: as DevicePlane (kept in HBM, downloaded only if a cell is
    read)."""
    torch = _torch()
    res = {}
    inv = None
    if perm is not None:
        p = np.asarray(perm, np.int64)
        iv = np.empty_like(p)
        iv[p] = np.arange(p.size, dtype=np.int64)
        dev = next(v.device for v in out.values() if v is not None and hasattr(v, "device"))
        inv = torch.as_tensor(iv, device=dev)
    host = lambda t: (t if inv is None else t.index_select(0, inv)).cpu().numpy()
    for name, _ in _lib.OUTPUT_SCALARS:
        res[name] = host(out[name])
    for name in _lib.OUTPUT_YEARLY:
        res[name] = host(out[name])
    for name in _lib.OUTPUT_HOURLY:
        t = out.get(name)
        if t is None:
            res[name] = None
        elif hourly_device:
            res[name] = DevicePlane(t, inv)
        elif hourly_async:
            res[name] = HostPlane(t, inv)
        elif t.shape[1] >= 16384:         # large planes: pinned, chunked, threaded
            res[name] = hourly_to_host(t, inv)
        elif inv is None:
            res[name] = hourly_agent_major(t).cpu().numpy()
        else:
            q, n, four = t.shape
            res[name] = t.permute(1, 0, 2).index_select(0, inv).reshape(n, q * four).cpu().numpy()
    return res
