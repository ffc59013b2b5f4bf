"""bench.py's algorithmic byte model (host logic, no GPU): which scratch-slot
agents move the battery case's f64 system-output plane (dgen_hip.hip
k_hourly_batt put_sys / put_nb / put_dcr / skip_plane) and the per-kernel
bytes that follow."""
import numpy as np

import bench
from dgen_amd.tariff import TARIFF_DTYPE


def _recs():
    r = np.zeros(5, TARIFF_DTYPE)
    r["P"] = [2, 3, 2, 4, 1]
    r["mo"] = [0, 2, 2, 0, 3]      # NEM, net billing, net billing, NEM, net billing + carryover
    r["dc"] = [0, 0, 1, 1, 0]      # tariffs 2 and 3 carry a demand record
    r["unit"] = [0, 0, 0, 0, 0]
    return r


def _cols(tariff, slot, ca=None, ws=None):
    n = len(tariff)
    return {"load_kwh": np.ones(n), "load_row": np.arange(n) % 3, "cf_row": np.arange(n) % 2,
            "econ_life": np.full(n, 25), "scratch_slot": np.asarray(slot),
            "flags": np.asarray(ca if ca is not None else np.zeros(n, int)) * 2,
            "wholesale_row": np.asarray(ws if ws is not None else np.full(n, -1))}


def test_scratch_paths_reference_mode():
    # reference mode (demand charges off): net-billing agents without a TS rate
    # take the scan-built split, with one (non-CA mo 2 with a wholesale row) the plane
    tf = np.array([0, 1, 1, 4, 2, 3])
    cols = _cols(tf, [-1, 0, 1, 2, 3, -1], ws=[-1, -1, 5, -1, -1, -1])
    plane, nb, dcr, mo2, P = bench.scratch_paths(cols, _recs(), tf, skip_dc=True)
    assert plane.tolist() == [False, False, True, False, False, False]
    assert nb.tolist() == [False, True, False, True, True, False]
    assert not dcr.any()
    assert mo2.tolist() == [False, True, True, True, True, False]
    assert P.tolist() == [2, 3, 3, 1, 2, 4]


def test_scratch_paths_demand_mode():
    # extension mode: a NEM agent with demand charges hands a demand record
    # (no plane); a net-billing agent with demand charges still writes the
    # plane (k_hourly_batt skips it only for one of the two records alone)
    tf = np.array([3, 2, 1])
    cols = _cols(tf, [0, 1, 2])
    plane, nb, dcr, _, _ = bench.scratch_paths(cols, _recs(), tf, skip_dc=False)
    assert plane.tolist() == [False, True, False]
    assert dcr.tolist() == [True, True, False]
    assert nb.tolist() == [False, True, True]
    # records off: every scratch agent billed hourly writes the plane
    plane, nb, dcr, _, _ = bench.scratch_paths(cols, _recs(), tf, skip_dc=False, nb_scan=False, dcr_on=False)
    assert plane.all() and not nb.any() and not dcr.any()
    # no battery run: nothing moves the plane
    plane, *_ = bench.scratch_paths(cols, _recs(), tf, skip_dc=False, battery=False)
    assert not plane.any()


def test_algorithmic_bytes_counts_the_plane_only_for_its_writers():
    tf = np.array([1, 1, 1, 0])
    cols = _cols(tf, [0, 1, 2, -1], ws=[-1, 4, -1, -1])
    paths = bench.scratch_paths(cols, _recs(), tf)
    upper = bench.algorithmic_bytes(cols, True, True)            # every slot agent: plane
    exact = bench.algorithmic_bytes(cols, True, True, paths)
    assert paths[0].sum() == 1
    for k in ("k_hourly_batt", "k_batt_finance"):
        assert exact[k] < upper[k]
    # exactly one plane written and read, plus its load row once
    assert exact["k_hourly_batt"] >= bench.SYS_BYTES
    assert exact["k_batt_finance"] >= bench.SYS_BYTES + bench.ROW_BYTES
    # no battery run: no finance bytes, no plane
    nob = bench.algorithmic_bytes(cols, True, False, bench.scratch_paths(cols, _recs(), tf, battery=False))
    assert nob["k_batt_finance"] == 0.0
    assert nob["k_hourly_batt"] < exact["k_hourly_batt"]


def test_scratch_paths_ts_scan():
    # with the TS agents' own scan (dgen_size_agents' ts_split) a non-CA net-billing
    # agent with a wholesale row hands a record too; a CA one always did
    tf = np.array([1, 1, 4])
    cols = _cols(tf, [0, 1, 2], ca=[0, 1, 0], ws=[5, 5, 5])
    plane, nb, *_ = bench.scratch_paths(cols, _recs(), tf, skip_dc=True)
    assert plane.tolist() == [True, False, False] and nb.tolist() == [False, True, True]
    plane, nb, *_ = bench.scratch_paths(cols, _recs(), tf, skip_dc=True, ts_scan=True)
    assert not plane.any() and nb.all()
    # the TS rows the scan reads are counted once each
    paths = bench.scratch_paths(cols, _recs(), tf, skip_dc=True, ts_scan=True)
    a = bench.algorithmic_bytes(cols, True, True, paths)
    b = bench.algorithmic_bytes(cols, True, True, paths, ts_rows=1)
    assert b["k_hourly_batt"] - a["k_hourly_batt"] == 8 * 8760
