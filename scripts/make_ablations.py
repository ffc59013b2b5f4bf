#!/usr/bin/env python3
"""Build kernel variants for A/B timing into ablate/ (outside the product
library directory; diagnostic only: occupancy variants compute the same results, the no_* variants are
wrong by construction).  Each variant is a text edit of a temporary copy of
the source; nothing here is part of the product build.  Run a variant with
DGEN_LIB=ablate/libdgen_<name>.so python bench.py ..., or scripts/gpu.sh ab.
Delete ablate/ after the A/B: everything in the tree ships with every gpurun call."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "dgen_amd", "csrc", "dgen_hip.hip")
OUT = os.path.join(REPO, "ablate")
sys.path.insert(0, REPO)
from dgen_amd.build import FLAGS, hipcc  # noqa: E402

HB = "__global__ void __launch_bounds__(BLOCK, 2)\nk_hourly_batt("
KS = "__global__ void __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(3)))\nk_size_w("
KF = "__global__ void __launch_bounds__(WAVE)\nk_batt_finance_w("


def occ(decl, w):
    decl = decl.replace(" __attribute__((amdgpu_waves_per_eu(3)))", "")
    head = decl.split("\n")[0].split("__launch_bounds__")[0]
    lb = "__launch_bounds__(BLOCK)" if "BLOCK" in decl else "__launch_bounds__(WAVE)"
    return head + lb + f" __attribute__((amdgpu_waves_per_eu({w}, {w})))\n" + decl.split("\n")[1]


VARIANTS = {
    "base": [],
    # per-phase shader-cycle counters (bench.py prints them with DGEN_PHASE_PROF=1)
    "phase": [("#define DGEN_PHASE_PROF 0", "#define DGEN_PHASE_PROF 1")],
    # k_hourly_batt day-target counters in slots 12-15 (battery lane-days, lanes
    # whose whole need fits, wave-days where it fits for all lanes, saturated)
    "phase_day": [("#define DGEN_PHASE_PROF 0", "#define DGEN_PHASE_PROF 1"),
                  ("#define DGEN_DAY_COUNTERS 0", "#define DGEN_DAY_COUNTERS 1")],
    # NEM bins build: slot-sum loads in flight per batch (4 = the product)
    "bins_bb8": [("        constexpr int BB = 4;\n", "        constexpr int BB = 8;\n")],
    "bins_bb12": [("        constexpr int BB = 4;\n", "        constexpr int BB = 12;\n")],
    # hour-lane envelope build: days of loads in flight per lane
    "dcb16": [("constexpr int DCB_DAYS = 8; ", "constexpr int DCB_DAYS = 16;")],
    "dcb12": [("constexpr int DCB_DAYS = 8; ", "constexpr int DCB_DAYS = 12;")],
    "dcb4": [("constexpr int DCB_DAYS = 8; ", "constexpr int DCB_DAYS = 4; ")],
    "dcb6": [("constexpr int DCB_DAYS = 8; ", "constexpr int DCB_DAYS = 6; ")],
    # phase timers only (DGEN_PHASE_PROF slots, see dgen_hip.hip)
    "phase": [("#define DGEN_PHASE_PROF 0", "#define DGEN_PHASE_PROF 1")],
    # timing probes of the hour-lane envelope build (wrong results by construction)
    "dcb_nopass2": [("#define DGEN_PHASE_PROF 0", "#define DGEN_PHASE_PROF 1"),
                    ("        // pass 2: the lines above the bound, per day type\n        for (int dt = 0; dt < 2; dt++) {",
                     "        // pass 2: the lines above the bound, per day type\n        for (int dt = 0; dt < 0; dt++) {")],
    "dcb_noload": [("#define DGEN_PHASE_PROF 0", "#define DGEN_PHASE_PROF 1"),
                   ("                    const double L = (double)src.shape[h] * src.load_scale;\n                    const double gp = cf_per_kw(src.cf[h]);\n                    mL = L > mL",
                    "                    const double L = (double)(h & 255) * src.load_scale;\n                    const double gp = cf_per_kw(h * 77);\n                    mL = L > mL"),
                   ("                    const double L = (double)src.shape[h] * src.load_scale;\n                    const double gp = cf_per_kw(src.cf[h]);\n                    if (h != pah",
                    "                    const double L = (double)(h & 255) * src.load_scale;\n                    const double gp = cf_per_kw(h * 77);\n                    if (h != pah")],
    # k_size evaluates the demand envelopes from the global record, not the LDS stage
    "no_dcstage": [("    {\n        const int slot = A.scratch_slot[i];\n        c.nb = (nbws",
                    "    c.stg = nullptr;\n    {\n        const int slot = A.scratch_slot[i];\n        c.nb = (nbws")],
    "db_cf4": [("#define DGEN_NB_DB_CF 6", "#define DGEN_NB_DB_CF 4")],
    "db_cf12": [("#define DGEN_NB_DB_CF 6", "#define DGEN_NB_DB_CF 12")],
    "hb_w3": [(HB, occ(HB, 3))],
    "hb_w4": [(HB, occ(HB, 4))],
    "ks_w3": [(KS, occ(KS, 3))],
    "ks_w4": [(KS, occ(KS, 4))],
    "kf_w6": [(KF, occ(KF, 6))],
    "kf_w3": [(KF, occ(KF, 3))],
    "no_target": [("                target = day_target_sorted(dv, power, avail);",
                   "                target = 0.0; asm volatile(\"\" :: \"v\"(dv[0]), \"v\"(dv[23]), \"v\"(avail));")],
    "no_bisect": [("    if (s[0] <= power) {\n        double S = 0.0, SK = s[0];", "    if (true) {\n        double S = 0.0, SK = s[0];")],
    "no_sort": [("                sort24_desc(dv);", "")],
    # k_hourly_batt wave priority: the hour loop (stores) above the day's sort
    # / target, or the reverse
    "hb_prio": [("            const double ls2 = opaque(ls), cs2 = opaque(cs6), cl2 = opaque(cl6);",
                 "            __builtin_amdgcn_s_setprio(2);\n            const double ls2 = opaque(ls), cs2 = opaque(cs6), cl2 = opaque(cl6);"),
                ("            if (ROLL && d > d_lo) day_reread(dlane, r);",
                 "            __builtin_amdgcn_s_setprio(0);\n            if (ROLL && d > d_lo) day_reread(dlane, r);")],
    "hb_prio_rev": [("            const double ls2 = opaque(ls), cs2 = opaque(cs6), cl2 = opaque(cl6);",
                     "            __builtin_amdgcn_s_setprio(0);\n            const double ls2 = opaque(ls), cs2 = opaque(cs6), cl2 = opaque(cl6);"),
                    ("            if (ROLL && d > d_lo) day_reread(dlane, r);",
                     "            __builtin_amdgcn_s_setprio(2);\n            if (ROLL && d > d_lo) day_reread(dlane, r);")],
    # k_hourly_batt: odd waves of a block start about half a day later (phase
    # offset between the waves' sort and store phases)
    "hb_stagger": [("    WsLayout W = ws_layout(ws, n);\n    // battery-case bins",
                    "    WsLayout W = ws_layout(ws, n);\n    if ((threadIdx.x >> 6) & 1) { __builtin_amdgcn_s_sleep(127); __builtin_amdgcn_s_sleep(127); }\n    // battery-case bins")],
    "hb_stagger4": [("    WsLayout W = ws_layout(ws, n);\n    // battery-case bins",
                     "    WsLayout W = ws_layout(ws, n);\n    for (int k = 0; k < (int)(threadIdx.x >> 6); k++) __builtin_amdgcn_s_sleep(80);\n    // battery-case bins")],
    # k_hourly_batt without the day's deficits, sort and target (hour loop and
    # stores only; wrong results by construction: the write / VALU split)
    "no_day_target": [("            } else if (has_batt) {\n                // the day's deficits",
                       "            } else if (false) {\n                // the day's deficits")],
    "no_hourly_stores": [("st_f32(ob + ho4, off4, (float)ld);", "asm volatile(\"\" :: \"v\"(ld));"),
                         ("st_f32(op + ho4, off4, (float)fmax(dn, 0.0));", "asm volatile(\"\" :: \"v\"(dn));"),
                         ("st_f32(ow + ho4, off4, (float)st.g2l);", "asm volatile(\"\" :: \"v\"(st.g2l));")],
    "no_batt_day": [("            if (has_batt) {\n                // day statistics",
                     "            if (false) {\n                // day statistics")],
    # profile loads always from the agent's first two days (L1/L2-resident):
    # measures how much of the scan waits on the day loads
    "hot_loads": [("lds_dma16(shp + dd * 24 + 4 * q, dbase_s + q * 1024u);",
                   "lds_dma16(shp + (dd & 1) * 24 + 4 * q, dbase_s + q * 1024u);"),
                  ("lds_dma16(cfp + dd * 24 + 4 * q, dbase_s + (6 + q) * 1024u);",
                   "lds_dma16(cfp + (dd & 1) * 24 + 4 * q, dbase_s + (6 + q) * 1024u);")],
    # k_size: slot-sum bins without their global loads (constant slot sums)
    "ks_no_slot_loads": [("                    lv[k] = lm[dt * 24 + h0 + k];\n                    gv[k] = gm[dt * 24 + h0 + k];",
                          "                    lv[k] = 1.0 + k; gv[k] = 0.5 + k;")],
    # hourly planes written with plain (temporal) stores instead of nt
    "plain_stores": [("    asm volatile(\"global_store_dword %0, %1, %2 nt\" :: \"v\"(off), \"v\"(v), \"s\"(row) : \"memory\");",
                      "    *reinterpret_cast<float*>(row + off) = v;")],
    # k_size: Brent stops after its first evaluation (per-evaluation cost)
    "ks_one_eval": [("        if (!(fabs(xf - xm) > (tol2 - 0.5 * (b - a)))) break;", "        break;")],
    # k_size: no NEM bill (per-lane year bill replaced by a constant)
    "ks_no_bill": [("    return (t.P <= PREG) ? yl_bill_mo0_reg(t, S, gscale, yearend) : yl_bill_mo0(t, S, gscale, yearend);",
                    "    return 100.0 + gscale;")],
    # hourly planes in hour-quad tiles (16 B per lane, 1 KB per wave per store)
    "tile4": [("#define DGEN_HOURLY_TILE 1\n", "#define DGEN_HOURLY_TILE 4\n")],
    # k_size / k_batt_finance without the net-billing (mo 2) code (register pressure of the NEM path)
    "no_mo2": [("    return (t.P <= PREG) ? yl_bill_mo2_reg(t, src, s, with_gen) : yl_bill_mo2(t, src, s, with_gen, S);",
                "    return 0.0;"),
               ("        c.wo1 = yl_bill_mo2(t, c.src, 1.0, false, c.S);", "        c.wo1 = 0.0;"),
               ("        wb = yl_bill_mo2(t, c.src, c.s_y, true, c.S);", "        wb = 0.0;")],
    # NEM register bill with the month loop unrolled by 2 / fully
    "bill_unroll2": [("    double total = 0.0;\n    for (int m = 0; m < 12; m++) {\n#pragma unroll\n        for (int p = 0; p < PREG; p++) {\n            if (p < P) {\n                double nn",
                      "    double total = 0.0;\n#pragma unroll 2\n    for (int m = 0; m < 12; m++) {\n#pragma unroll\n        for (int p = 0; p < PREG; p++) {\n            if (p < P) {\n                double nn")],
    "bill_unroll12": [("    double total = 0.0;\n    for (int m = 0; m < 12; m++) {\n#pragma unroll\n        for (int p = 0; p < PREG; p++) {\n            if (p < P) {\n                double nn",
                       "    double total = 0.0;\n#pragma unroll\n    for (int m = 0; m < 12; m++) {\n#pragma unroll\n        for (int p = 0; p < PREG; p++) {\n            if (p < P) {\n                double nn")],
    # reference-mode k_size at 2 waves per SIMD (no spills) instead of 3
    "ks_occ2": [("amdgpu_waves_per_eu(DC ? 2 : 3)", "amdgpu_waves_per_eu(DC ? 2 : 2)")],
    # hourly-plane store cache policy (MI355X_MICROARCH.md: plain / sc0 / nt keep the
    # line in the XCD's L2, sc1 / sc0 sc1 write through and drop it)
    "st_sc1": [('global_store_dwordx4 %0, %1, %2 nt"', 'global_store_dwordx4 %0, %1, %2 sc1"')],
    "st_sc0sc1": [('global_store_dwordx4 %0, %1, %2 nt"', 'global_store_dwordx4 %0, %1, %2 sc0 sc1"')],
    "st_plain4": [('global_store_dwordx4 %0, %1, %2 nt"', 'global_store_dwordx4 %0, %1, %2"')],
    "no_bins": [("                    double2 b = bins[p * BLOCK];\n                    b.x += ld;\n                    b.y += st.sys;\n                    bins[p * BLOCK] = b;",
                 "                    asm volatile(\"\" :: \"v\"(p), \"v\"(st.sys));")],
    # --- demand-charge two-agent k_size diagnosis ---------------------------
    # agent-scope release before the envelope / split hand-offs (orders the
    # month lanes' stores before the wait at compiler level)
    "dc_rel": [("    // buffer_inv sc1, once per build.\n    __builtin_amdgcn_s_waitcnt(0);",
                "    // buffer_inv sc1, once per build.\n    __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"agent\");\n    __builtin_amdgcn_s_waitcnt(0);"),
               ("    // hand-off to the other lanes through global memory, as yl_dc_build\n    __builtin_amdgcn_s_waitcnt(0);",
                "    // hand-off to the other lanes through global memory, as yl_dc_build\n    __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"agent\");\n    __builtin_amdgcn_s_waitcnt(0);")],
    # no envelopes: every demand charge from the hourly pass (yl_demand)
    "dc_noenv": [("            if (c.dem_wo_pending) c.env_ok = c.env.lines && yl_dc_build(c.dem, c.src, c.tlo, c.thi, c.env, c.g);",
                  "            if (c.dem_wo_pending) c.env_ok = false;")],
    # envelopes built, evaluations from the hourly pass
    "dc_noeval": [("                const double v = c.env_ok ? yl_dc_eval(c.dem, c.env, kws, s, wg, c.S)\n                                          : yl_demand(c.dem, c.src, s, wg, c.S);",
                   "                const double v = yl_demand(c.dem, c.src, s, wg, c.S);")],
    # per-evaluation capture of the demand-charge objective for agents 0-3
    # (read back with dgen_debug_dcdbg; scripts/dbg_dc_eval.py)
    "dc_dbg": [("constexpr size_t DCW_BYTES =",
                "__device__ double g_dcdbg[4][24][64][6];\nconstexpr size_t DCW_BYTES ="),
               ("    Seg<LPA> g;\n    int y, N;\n    bool active;",
                "    Seg<LPA> g;\n    int y, N;\n    bool active;\n    int dbg_i, dbg_e;"),
               ("    c.dem_wo_pending = false;\n    c.env_ok = false;\n    c.env.lines = nullptr;",
                "    c.dem_wo_pending = false;\n    c.env_ok = false;\n    c.env.lines = nullptr;\n    c.dbg_i = (int)i; c.dbg_e = 0;"),
               ("                if (wg) wb += v;\n                else c.wo1 += v;",
                "                if (wg && c.dbg_i < 4 && c.dbg_e < 24) {\n"
                "                    double* r = g_dcdbg[c.dbg_i][c.dbg_e][c.g.lane];\n"
                "                    r[0] = kws; r[1] = s; r[2] = v; r[3] = wb; r[4] = c.env_ok ? 1.0 : 0.0; r[5] = c.r_y;\n"
                "                }\n"
                "                if (wg) wb += v;\n                else c.wo1 += v;"),
               ("            c.dem_wo_pending = false;\n        }\n    }",
                "            c.dem_wo_pending = false;\n            c.dbg_e++;\n        }\n    }"),
               ('extern "C" {', 'extern "C" {\nint32_t dgen_debug_dcdbg(void* dst) { return (int32_t)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_dcdbg), sizeof(g_dcdbg)); }')],
    # two-agent demand-charge k_size at 1 wave per SIMD (round 1's no-spill build; now 2 waves)
    # net-billing k_size (C2) at 2 waves per SIMD (no spills) instead of 3
    "ks_net_occ2": [("amdgpu_waves_per_eu(DC ? 2 : 3)", "amdgpu_waves_per_eu(DC || NET ? 2 : 3)")],
    # k_batt_finance at 2 / 4 waves per SIMD
    "kf_occ2": [("__global__ void __launch_bounds__(WAVE)\nk_batt_finance_w(",
                 "__global__ void __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(2, 2)))\nk_batt_finance_w(")],
    "kf_occ4": [("__global__ void __launch_bounds__(WAVE)\nk_batt_finance_w(",
                 "__global__ void __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(4)))\nk_batt_finance_w(")],
    # days per load batch of the cooperative net-billing build
    "nb_db_cf4": [("#define DGEN_NB_DB_CF 6", "#define DGEN_NB_DB_CF 4")],
    "nb_db_cf12": [("#define DGEN_NB_DB_CF 6", "#define DGEN_NB_DB_CF 12")],
    "nb_db_cf2": [("#define DGEN_NB_DB_CF 6", "#define DGEN_NB_DB_CF 2")],
    "nb_db_cf3": [("#define DGEN_NB_DB_CF 6", "#define DGEN_NB_DB_CF 3")],
    "nb_db_cf6": [("#define DGEN_NB_DB_CF 6", "#define DGEN_NB_DB_CF 6")],
    "nb_db_sys2": [("#define DGEN_NB_DB_SYS 4", "#define DGEN_NB_DB_SYS 2")],
    "nb_db_sys3": [("#define DGEN_NB_DB_SYS 4", "#define DGEN_NB_DB_SYS 3")],
    "nb_db_sys8": [("#define DGEN_NB_DB_SYS 4", "#define DGEN_NB_DB_SYS 8")],
    # k_hourly_batt's battery-case split (NB instantiation): off (LDS still
    # doubled: the occupancy cost alone) / without its mixed-entry stores
    "hb_nb_off": [("        put_nb = put_sys && mo2 && !ts_on;", "        put_nb = false && put_sys && mo2 && !ts_on;")],
    "hb_nb_nostore": [("                            nb_ent[n_m] = e;", "                            (void)e;")],
    # --- k_hourly_batt attribution on the current source (round 4; timing only,
    # results wrong by construction except hb_w3) ---------------------------
    # the three hourly-plane stores sunk (the day read-back then waits for the
    # DMA alone): the scan's VALU / LDS part
    "hb_nostores": [("                        st_f32x4(ob + q16, off16, qb);\n"
                     "                        st_f32x4(op + q16, off16, qp);\n"
                     "                        st_f32x4(ow + q16, off16, qw);\n",
                     "                        asm volatile(\"\" :: \"v\"(qb[0]), \"v\"(qb[1]), \"v\"(qb[2]), \"v\"(qb[3]),\n"
                     "                                     \"v\"(qp[0]), \"v\"(qp[1]), \"v\"(qp[2]), \"v\"(qp[3]));\n"
                     "                        asm volatile(\"\" :: \"v\"(qw[0]), \"v\"(qw[1]), \"v\"(qw[2]), \"v\"(qw[3]));\n"),
                    ("day_read<HB_STORES_AFTER_DMA * (F64 ? 2 : 1)>(dlane, r)", "day_read<0>(dlane, r)")],
    # the next-day DMA not waited for (LDS read races it): the cost of the
    # in-order vmcnt wait, which also waits for every store older than the DMA
    "hb_dma_nowait": [("day_read<HB_STORES_AFTER_DMA * (F64 ? 2 : 1)>(dlane, r)", "day_read<60>(dlane, r)")],
    # the day's deficits / sort / target skipped: the hour loop and its stores
    # 3 waves per SIMD (VGPR cap 168)
    "hb_w3b": [("__launch_bounds__(BLOCK, ROLL ? 1 : 2)\nk_hourly_batt(", "__launch_bounds__(BLOCK, ROLL ? 1 : 3)\nk_hourly_batt(")],
    "hb_notarget": [("            } else if (has_batt) {\n                // the day's deficits d_h",
                     "            } else if (false) {\n                // the day's deficits d_h")],
    # per-agent kernels' block size (k_hourly_batt: waves per block)
    "block64": [("constexpr int BLOCK = 128;", "constexpr int BLOCK = 64;"),
                 ("__launch_bounds__(BLOCK, 2)\nk_hourly_batt(", "__launch_bounds__(BLOCK, 8)\nk_hourly_batt(")],
    "block256": [("constexpr int BLOCK = 128;", "constexpr int BLOCK = 256;"),
                 ("__launch_bounds__(BLOCK, 2)\nk_hourly_batt(", "__launch_bounds__(BLOCK, 1)\nk_hourly_batt(")],
    # C3 k_size attribution: the NEM bins build's slot-sum loads replaced by
    # a constant / the no-system bill skipped (results wrong by construction)
    "ks_bins_const": [("                    lv[k] = lm[dt * 24 + h0 + k];\n                    gv[k] = gm[dt * 24 + h0 + k];",
                       "                    lv[k] = 1.0 + (double)(size_t)lm * 0.0;\n                    gv[k] = 0.5 + (double)(size_t)gm * 0.0;")],
    "ks_wo1_skip": [("        c.wo1 = yl_bill_nem(t, c.S, 0.0, c.yearend);\n        PH_ADD_KS(12",
                     "        c.wo1 = 1000.0;\n        PH_ADD_KS(12")],
    # NEM evaluation bill: months unrolled (ILP across months' tier charges)
    "bill_unroll2": [("    double total = 0.0;\n    for (int m = 0; m < 12; m++) {\n#pragma unroll\n        for (int p = 0; p < PREG; p++) {\n            if (p < P) {\n                double nn",
                      "    double total = 0.0;\n#pragma unroll 2\n    for (int m = 0; m < 12; m++) {\n#pragma unroll\n        for (int p = 0; p < PREG; p++) {\n            if (p < P) {\n                double nn")],
    "bill_unroll4": [("    double total = 0.0;\n    for (int m = 0; m < 12; m++) {\n#pragma unroll\n        for (int p = 0; p < PREG; p++) {\n            if (p < P) {\n                double nn",
                      "    double total = 0.0;\n#pragma unroll 4\n    for (int m = 0; m < 12; m++) {\n#pragma unroll\n        for (int p = 0; p < PREG; p++) {\n            if (p < P) {\n                double nn")],
    "ks_dc_occ1": [("amdgpu_waves_per_eu(DC ? 2 : 3)", "amdgpu_waves_per_eu(DC ? (LPA == WAVE ? 2 : 1) : 3)")],
    # k_batt_finance without its battery-case demand pass (what the rest costs)
    "kf_no_dem": [("            const double v = yl_demand_staged(dem, src, wg ? s_y : 1.0, wg, S, stage, g);",
                   "            const double v = 0.0 * (double)(size_t)stage;")],
    # C2 (net billing) split of k_size: evaluations without the split bill / without the build
    "ks_nb_noeval": [("        wb = c.nb_ok ? yl_bill_nb(t, c.src, c.s_y, c.nb, c.S) : yl_bill_mo2(t, c.src, c.s_y, true, c.S);",
                      "        wb = c.nb_ok ? 1000.0 - kws * c.s_y : yl_bill_mo2(t, c.src, c.s_y, true, c.S);")],
    "ks_nb_nobuild": [("        c.nb_ok = c.nb && yl_nb_build(t, c.src, c.tlo, c.thi, c.nb, c.S, c.g);",
                       "        c.nb_ok = c.nb != nullptr;"),
                      ("        wb = c.nb_ok ? yl_bill_nb(t, c.src, c.s_y, c.nb, c.S) : yl_bill_mo2(t, c.src, c.s_y, true, c.S);",
                       "        wb = c.nb_ok ? 1000.0 - kws * c.s_y : yl_bill_mo2(t, c.src, c.s_y, true, c.S);")],
    # k_hourly_batt: the day-start read-back waits for every outstanding store
    # (vmcnt(0)) instead of only the DMA: how much the scan waits on stores
    "hb_vm0": [("            else if (HOURLY && d > d_lo) day_read<HB_STORES_AFTER_DMA * (F64 ? 2 : 1)>(dlane, r);",
                "            else if (HOURLY && d > d_lo) day_read<0>(dlane, r);")],
    # year-lane kernels (k_nb_env, k_size_w, k_batt_finance_w): XCD-aware block
    # order, so agents adjacent in device order (sharing a load-shape row) run
    # on one XCD and its L2 serves the row (blocks are dealt round-robin to the
    # 8 XCDs)
    "xcd_yl": [("constexpr int WAVE = 64;\n",
                "constexpr int WAVE = 64;\n__device__ __forceinline__ unsigned xcd_map(unsigned b, unsigned nb) {\n"
                "    const unsigned q = nb / 8u, r = nb % 8u, x = b % 8u, k = b / 8u;\n"
                "    return x < r ? x * (q + 1u) + k : r * (q + 1u) + (x - r) * q + k;\n}\n"),
               ("    const int64_t i = i0 + (int64_t)blockIdx.x * (WAVE / LPA) + (LPA == WAVE ? 0 : lane / LPA);",
                "    const int64_t i = i0 + (int64_t)xcd_map(blockIdx.x, gridDim.x) * (WAVE / LPA) + (LPA == WAVE ? 0 : lane / LPA);")],
    # k_batt_finance net-billing: without the split build / bill
    "kf_nb_none": [("            nb_ok = yl_nb_build(t, src, s_lo, s_hi, nbp, S, g);\n            if (nb_ok) wb = yl_bill_nb(t, src, s_y, nbp, S);",
                    "            nb_ok = true; wb = 1000.0 * s_y + (double)(size_t)nbp * 0.0;")],
}

# Brent evaluation trace of one agent in k_size (diagnostics, results
# unchanged): per evaluation (kW, -NPV, net-billing split used, envelope used
# | staged << 1); dgen_bt_set(agent) / dgen_bt_read(out[256]) -> count
BTRACE = [("template <int LPA, bool DC, bool NET, bool PK>\n__global__ void __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(DC ? 2 : 3)))\nk_size_w(",
           "__device__ long long g_bt_agent = -1;\n__device__ int g_bt_n = 0;\n__device__ double g_bt[256];\n"
           "template <int LPA, bool DC, bool NET, bool PK>\n__global__ void __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(DC ? 2 : 3)))\nk_size_w("),
          ("            return yl_objective<LPA, DC, NET, PK>(c, x);\n",
           "            const double v_ = yl_objective<LPA, DC, NET, PK>(c, x);\n"
           "            if (i == g_bt_agent && sl == 0) { const int k_ = g_bt_n; if (k_ < 64) { g_bt[4 * k_] = x; g_bt[4 * k_ + 1] = v_;"
           " g_bt[4 * k_ + 2] = c.nb_ok ? 1.0 : 0.0; g_bt[4 * k_ + 3] = (c.env_ok ? 1.0 : 0.0) + (c.stg_ok ? 2.0 : 0.0); } g_bt_n = k_ + 1; }\n"
           "            return v_;\n"),
          ("int32_t dgen_last_paths(dgen_ctx* c, int32_t* out, int32_t n_out) {",
           "extern \"C\" int32_t dgen_bt_set(long long agent) {\n    int z = 0;\n"
           "    if (hipMemcpyToSymbol(HIP_SYMBOL(g_bt_agent), &agent, sizeof(agent)) != hipSuccess) return -1;\n"
           "    return hipMemcpyToSymbol(HIP_SYMBOL(g_bt_n), &z, sizeof(z)) == hipSuccess ? 0 : -1;\n}\n"
           "extern \"C\" int32_t dgen_bt_read(double* out) {\n    int n = 0;\n"
           "    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_bt_n), sizeof(n)) != hipSuccess) return -1;\n"
           "    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bt), sizeof(double) * 256) != hipSuccess) return -1;\n"
           "    return n;\n}\n"
           "int32_t dgen_last_paths(dgen_ctx* c, int32_t* out, int32_t n_out) {")]
VARIANTS["btrace"] = BTRACE

# in-kernel clock of k_hourly_batt (MI355X_MICROARCH.md DVFS item 6): thread 0 of
# each block stamps s_memtime / s_memrealtime at its start and after its month
# loop into a buffer of its own; bench.py prints the median clock (run with
# --hb-split 1 so the last launch owns every stamp)
CLK = [("constexpr int HB_DAY_BYTES = 12 * 1024;",
        "__device__ unsigned long long g_clk[4][8192];\nconstexpr int HB_DAY_BYTES = 12 * 1024;"),
       ("    WsLayout W = ws_layout(ws, n);\n    // battery-case bins",
        "    WsLayout W = ws_layout(ws, n);\n"
        "    if (threadIdx.x == 0 && blockIdx.x < 8192) { g_clk[0][blockIdx.x] = __builtin_amdgcn_s_memtime();"
        " g_clk[1][blockIdx.x] = __builtin_amdgcn_s_memrealtime(); }\n    // battery-case bins"),
       ("    if (m_hi < 12) {\n        W.carry[i] = soc;",
        "    if (threadIdx.x == 0 && blockIdx.x < 8192) { g_clk[2][blockIdx.x] = __builtin_amdgcn_s_memtime();"
        " g_clk[3][blockIdx.x] = __builtin_amdgcn_s_memrealtime(); }\n    if (m_hi < 12) {\n        W.carry[i] = soc;"),
       ('extern "C" {', 'extern "C" {\nint32_t dgen_clk_read(void* dst) { return (int32_t)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_clk), sizeof(g_clk)); }')]
VARIANTS["hb_clk"] = CLK
VARIANTS["hb_nostores_clk"] = VARIANTS["hb_nostores"] + CLK
VARIANTS["hb_notarget_clk"] = VARIANTS["hb_notarget"] + CLK

# the three plane stores kept but always to the launch's first hour-quad row
# (48 MB at 1M agents: cache-resident, no HBM write stream): store issue vs HBM
VARIANTS["hb_stores_l2"] = [("                        st_f32x4(ow + q16, off16, qw);\n                        q16 += row16;\n",
                             "                        st_f32x4(ow + q16, off16, qw);\n")]
VARIANTS["hb_stores_l2_clk"] = VARIANTS["hb_stores_l2"] + CLK

# day counters with slot 13 / 14 = lane-days / wave-days whose battery holds
# no deliverable energy at the day's first hour (avail = 0: the day's target
# cannot discharge anything, so its value does not matter)
VARIANTS["phase_empty"] = [("#define DGEN_PHASE_PROF 0", "#define DGEN_PHASE_PROF 1"),
                           ("#define DGEN_DAY_COUNTERS 0", "#define DGEN_DAY_COUNTERS 1"),
                           ("                    const bool fits = need <= avail;",
                            "                    const bool fits = !(avail > 0.0); (void)need;")]

# C3 k_size attribution by doubling (results unchanged, the time difference is
# one copy's cost): the NEM bins build twice per tariff / the objective twice
# per Brent evaluation
VARIANTS["ks_bins_x2"] = [("        PH_T0(tn);\n        wave_lds_sync();\n        yl_build_bins(t, c.lslots, c.gslots, c.load_scale, c.S, c.g);\n",
                           "        PH_T0(tn);\n        wave_lds_sync();\n        yl_build_bins(t, c.lslots, c.gslots, c.load_scale, c.S, c.g);\n"
                           "        yl_build_bins(t, c.lslots, c.gslots, c.load_scale, c.S, c.g);\n")]
VARIANTS["ks_nosys_x2"] = [("        c.wo1 = yl_bill_nem_nosys(t, c.S, c.yearend, c.g);\n",
                            "        c.wo1 = yl_bill_nem_nosys(t, c.S, c.yearend, c.g);\n"
                            "        c.wo1 = yl_bill_nem_nosys(t, c.S, c.yearend, c.g);\n")]
VARIANTS["ks_obj_x2"] = [("            return yl_objective<LPA, DC, NET, PK>(c, x);",
                          "            (void)yl_objective<LPA, DC, NET, PK>(c, x);\n            return yl_objective<LPA, DC, NET, PK>(c, x);")]

# k_size (bins-only and net-billing instantiations) at 4 waves per SIMD
VARIANTS["ks_occ4"] = [("amdgpu_waves_per_eu(DC ? 2 : 3)", "amdgpu_waves_per_eu(DC ? 2 : 4)")]
# the demand-charge instantiations at 3 waves per SIMD (168 VGPRs: spills)
VARIANTS["ks_dc3"] = [("amdgpu_waves_per_eu(DC ? 2 : 3)", "amdgpu_waves_per_eu(3)")]

# yl_build_bins: slot sums loaded 12 / 24 per row and batch (2 / 1 batches per
# day type instead of 3): C3 k_size 9.3 -> 9.7 / 14.5 ms (profiles/r05/s18)
VARIANTS["bins_b12"] = [("        constexpr int BB = 8;\n        const double* lm = lslots + m * 48;",
                         "        constexpr int BB = 12;\n        const double* lm = lslots + m * 48;")]
VARIANTS["bins_b24"] = [("        constexpr int BB = 8;\n        const double* lm = lslots + m * 48;",
                         "        constexpr int BB = 24;\n        const double* lm = lslots + m * 48;")]

# k_dc_env at 2 waves per SIMD (no spills) instead of 3
VARIANTS["dce_w2"] = [("__global__ void __launch_bounds__(WAVE * DCE_WPB) __attribute__((amdgpu_waves_per_eu(NQ <= 4 ? 3 : 2)))",
                       "__global__ void __launch_bounds__(WAVE * DCE_WPB) __attribute__((amdgpu_waves_per_eu(2)))")]

# the NEM-only k_size at 4 waves per SIMD (128 VGPRs: spills) now that its
# slimmer LDS layout would admit a fourth
VARIANTS["ks_nem_w4"] = [("amdgpu_waves_per_eu(DC ? 2 : 3)", "amdgpu_waves_per_eu(DC ? 2 : (NET ? 3 : 4))")]

# timing only (C3: mo 0, P <= PREG, so the NEM bills use no slot but the
# cash flow's two): NEM-only kernels with 2 slots per lane, k_batt_finance's
# NEM-only instantiation at 5 waves per SIMD -- C3 k_batt_finance 3.14 -> 3.14 /
# 3.35 ms (profiles/r05/s29), not kept
VARIANTS["kf_w5"] = [("__host__ __device__ inline int ylds_slots(int half, bool slim) { return slim ? 2 * half : 4 * half; }",
                      "__host__ __device__ inline int ylds_slots(int half, bool slim) { return slim ? 2 : 4 * half; }"),
                     ("template <int LPA, bool DC, bool NET, bool PK>\n__global__ void __launch_bounds__(WAVE)\nk_batt_finance_w(",
                      "template <int LPA, bool DC, bool NET, bool PK>\n__global__ void __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu((DC || NET) ? 1 : 5)))\nk_batt_finance_w(")]
VARIANTS["kf_s2"] = [("__host__ __device__ inline int ylds_slots(int half, bool slim) { return slim ? 2 * half : 4 * half; }",
                      "__host__ __device__ inline int ylds_slots(int half, bool slim) { return slim ? 2 : 4 * half; }")]

# yl_bill_nb: staged entries read per group ahead of the billed group
VARIANTS["nbu2"] = [("#define DGEN_NB_U 4", "#define DGEN_NB_U 2")]
VARIANTS["nbu8"] = [("#define DGEN_NB_U 4", "#define DGEN_NB_U 8")]


def main():
    os.makedirs(OUT, exist_ok=True)
    src = open(SRC).read().replace('#include "../../include/dgen_hip.h"',
                                   f'#include "{REPO}/include/dgen_hip.h"')
    names = sys.argv[1:] or list(VARIANTS)
    for name in names:
        s = src
        for a, b in VARIANTS[name]:
            assert a in s, (name, a[:60])
            s = s.replace(a, b)
        tmp = f"/tmp/ablate_{name}.hip"
        open(tmp, "w").write(s)
        out = os.path.join(OUT, f"libdgen_{name}.so")
        subprocess.run([hipcc(), *FLAGS, "-o", out, tmp], check=True)
        print("built", out, flush=True)


if __name__ == "__main__":
    main()
