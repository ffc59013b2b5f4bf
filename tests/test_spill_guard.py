"""The build guard against spills ahead of a divergent join's exec restore
(dgen_amd/spill_guard.py): the scanner on hand-made
assembly, and the state the last build left."""
import json
import os

from dgen_amd import build as B
from dgen_amd import spill_guard as G

BAD = """_ZN12_GLOBAL__N_18k_size_wILi32ELb1ELb1ELb0EEEv11dgen_tablesPc:
\tv_mov_b32_e32 v1, 0
.LBB13_10:
\tbuffer_inv sc1
.LBB13_11:                            ;   in Loop: Header=BB13_9 Depth=1
\tv_accvgpr_write_b32 a12, v244
\tv_writelane_b32 v255, s62, 4
\tv_accvgpr_write_b32 a10, v242
\ts_or_b64 exec, exec, s[2:3]
\tglobal_load_dwordx4 v[4:7], v[116:117], off
"""

GOOD = """_ZN12_GLOBAL__N_18k_size_wILi32ELb1ELb1ELb0EEEv11dgen_tablesPc:
.LBB13_11:
\ts_or_b64 exec, exec, s[2:3]
\tv_accvgpr_write_b32 a12, v244
\tv_accvgpr_write_b32 a10, v242
.LBB13_12:
\tv_add_f64 v[0:1], v[2:3], v[4:5]
\tv_accvgpr_write_b32 a3, v1
\ts_or_b64 exec, exec, s[4:5]
"""

OTHER = BAD.replace("_ZN12_GLOBAL__N_18k_size_wILi32ELb1ELb1ELb0EEEv11dgen_tablesPc",
                    "_ZN12_GLOBAL__N_113k_hourly_battILb1EEEv11dgen_tables")


def _scan(tmp_path, text):
    p = tmp_path / "k.s"
    p.write_text(text)
    return G.scan(str(p))


def test_flags_spill_before_exec_restore(tmp_path):
    hits = _scan(tmp_path, BAD)
    (fn, blocks), = hits.items()
    assert "k_size_wILi32ELb1E" in fn
    assert blocks[0][0] == ".LBB13_11" and len(blocks[0][1]) == 2
    assert G.remedies(hits) == (["DGEN_NO2_SIZE_DC"], [])


def test_spill_after_restore_or_inside_block_is_not_flagged(tmp_path):
    # after the restore the spill runs with the join's full mask; a spill after
    # arithmetic belongs to the block body, not to the join's prologue
    assert _scan(tmp_path, GOOD) == {}


def test_kernel_without_remedy_is_fatal(tmp_path):
    macros, fatal = G.remedies(_scan(tmp_path, OTHER))
    assert macros == [] and len(fatal) == 1


def test_last_build_passed_the_guard():
    B.build()
    with open(B.GUARD) as f:
        g = json.load(f)
    assert set(g["withdrawn"]) <= set(G.REMEDY.values())
    # a withdrawn kernel was flagged in the first compile
    if g["withdrawn"]:
        assert g["flagged_first_build"]
    assert os.path.exists(B.OUT)
    # k_hourly_batt's next-day DMA wait is covered on every path
    assert g["vmem_ops_after_day_dma"] >= g["day_dma_wait_vmcnt"] > 0


DMA = """_ZN12_GLOBAL__N_113k_hourly_battILb1EEEv11dgen_tables:   ; @k
.LBB16_41:
\ts_waitcnt vmcnt(4)
\tds_read_b128 v[0:3], v9
.LBB16_60:
\tglobal_load_lds_dwordx4 v[2:3], off
\tglobal_load_lds_dwordx4 v[4:5], off
.LBB16_61:
\tglobal_store_dwordx4 v[0:1], v[4:7], off nt
\tglobal_store_dwordx4 v[0:1], v[4:7], off nt
\ts_cbranch_execz .LBB16_69
; %bb.68:
\tglobal_store_dwordx4 v[0:1], v[4:7], off
\tglobal_store_dwordx4 v[0:1], v[4:7], off
.LBB16_69:
\tglobal_store_dwordx4 v[0:1], v[4:7], off nt
STORES\ts_branch .LBB16_41
.Lfunc_end16:
"""


def test_day_dma_wait_counts_unconditional_ops(tmp_path):
    p = tmp_path / "d.s"
    p.write_text(DMA.replace("STORES", ""))
    assert G.day_dma_wait(str(p)) == (4, 3)       # the two skippable stores do not count
    p.write_text(DMA.replace("STORES", "\tglobal_store_dwordx4 v[0:1], v[4:7], off nt\n"))
    assert G.day_dma_wait(str(p)) == (4, 4)
    # a full drain on the way (s_waitcnt vmcnt(0)) covers the wait by itself
    p.write_text(DMA.replace("STORES", "\ts_waitcnt vmcnt(0)\n"))
    assert G.day_dma_wait(str(p)) == G.DRAINED
    # no DMA group (or no counted wait) at all is not "drained": the build fails
    p.write_text(DMA.replace("STORES", "").replace("global_load_lds_dwordx4", "global_load_dwordx4"))
    assert G.day_dma_wait(str(p)) is None
    p.write_text(DMA.replace("STORES", "").replace("vmcnt(4)", "vmcnt(0)"))
    assert G.day_dma_wait(str(p)) is None


COPY = BAD.replace("\tv_accvgpr_write_b32 a12, v244\n", "\tv_mov_b32_e32 v10, v244\n") \
          .replace("\tv_accvgpr_write_b32 a10, v242\n", "")


def test_flags_vgpr_copy_before_exec_restore(tmp_path):
    # a live-range-split copy ahead of the restore fills only the branch's lanes
    hits = _scan(tmp_path, COPY)
    (fn, blocks), = hits.items()
    assert blocks[0][1] == ["v_mov_b32_e32 v10, v244"]
    for ins in ("v_cndmask_b32_e64 v10, v1, v2, s[4:5]", "v_accvgpr_read_b32 v10, a3",
                "v_mov_b64_e32 v[10:11], v[244:245]"):
        assert _scan(tmp_path, COPY.replace("v_mov_b32_e32 v10, v244", ins)), ins
    # constants and SGPR sources are not copies of a live VGPR value
    for ins in ("v_mov_b32_e32 v10, 0", "v_mov_b32_e32 v10, s4", "v_mov_b64_e32 v[6:7], s[68:69]"):
        assert _scan(tmp_path, COPY.replace("v_mov_b32_e32 v10, v244", ins)) == {}, ins
