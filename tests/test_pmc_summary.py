"""scripts/pmc_summary.py: a kernel family's PMC figures are the sum over its
template instantiations, each weighted by its own dispatches per call
(national k_hourly_batt ran three instantiations with
different sizes and dispatch counts)."""
import csv
import importlib.util
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("pmc_summary", os.path.join(REPO, "scripts", "pmc_summary.py"))
pmc = importlib.util.module_from_spec(spec)
spec.loader.exec_module(pmc)

HEAD = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id", "Grid_Size",
        "Kernel_Id", "Kernel_Name", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
        "Accum_VGPR_Count", "SGPR_Count", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]
KS = "void (anonymous namespace)::k_size_w<32, false, true, false>(dgen_tables, dgen_agents, dgen_outputs, dgen_cfg, long)"
KS2 = "void dgen_srch::k_size_w<32, false, false, false>(dgen_tables, dgen_agents, dgen_outputs, dgen_cfg, long)"
HB_BIG = "void (anonymous namespace)::k_hourly_batt<true, false, true, false>(dgen_tables, dgen_agents, dgen_outputs, int)"
HB_SMALL = "void (anonymous namespace)::k_hourly_batt<true, false, false, false>(dgen_tables, dgen_agents, dgen_outputs, int)"


def _write(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(HEAD)
        for i, (name, cnt, val) in enumerate(rows):
            w.writerow([i, i, "Agent 2", 1, 1, 1, 64, 1, name, 64, 0, 0, 64, 0, 32, cnt, val, 0, 1])


def _pass(path, counter, big, small, ks):
    """Two calls: per call 1 dispatch of each k_size_w instantiation, 8 of the
    big k_hourly_batt instantiation, 2 of the small one."""
    rows = []
    for _ in range(2):
        rows += [(KS, counter, ks), (KS2, counter, ks)]
        rows += [(HB_BIG, counter, big)] * 8 + [(HB_SMALL, counter, small)] * 2
    _write(path, rows)


def test_inst_name_keeps_template_arguments():
    assert pmc.inst_name(HB_BIG) == "k_hourly_batt<true, false, true, false>"
    assert pmc.inst_name(KS2) == "k_size_w<32, false, false, false>"
    assert pmc.family(pmc.inst_name(HB_SMALL)) == "k_hourly_batt"


def test_family_sums_instantiations_by_their_own_dispatch_counts(tmp_path):
    d = tmp_path / "p"
    d.mkdir()
    _pass(d / "a_counter_collection.csv", "FETCH_SIZE", 1000.0, 10.0, 50.0)
    _pass(d / "b_counter_collection.csv", "WRITE_SIZE", 4000.0, 2.0, 30.0)
    files = [str(d / "a_counter_collection.csv"), str(d / "b_counter_collection.csv")]
    for calls in (None, 2):
        res = pmc.summarize(files, agents=100, calls=calls)
        hb = res["k_hourly_batt"]
        assert hb["dispatches_per_call"] == 10
        assert hb["instantiations"]["k_hourly_batt<true, false, true, false>"]["dispatches_per_call"] == 8
        assert hb["instantiations"]["k_hourly_batt<true, false, false, false>"]["dispatches_per_call"] == 2
        rd = 2 * (8 * 1000.0 + 2 * 10.0) * 1024
        wr = (8 * 4000.0 + 2 * 2.0) * 1024
        assert hb["hbm_read_bytes_per_call"] == pytest.approx(rd)
        assert hb["hbm_write_bytes_per_call"] == pytest.approx(wr)
        assert hb["hbm_bytes_per_agent"] == pytest.approx((rd + wr) / 100)
        ks = res["k_size_w"]
        assert ks["dispatches_per_call"] == 2
        assert ks["hbm_bytes_per_agent"] == pytest.approx(2 * (2 * 50.0 + 30.0) * 1024 / 100)
