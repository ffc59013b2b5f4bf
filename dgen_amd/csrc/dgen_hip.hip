// dgen_hip.hip -- gfx950 kernels + C-ABI for dGen's per-agent sizing & economics
// hot path (financial_functions.calc_system_size_and_performance and the PySAM
// Utilityrate5 / Cashloan / Battery work it drives).  See include/dgen_hip.h
// for the interface and DESIGN.md for the data layout and rooflines.
//
// Build (dgen_amd/build.py):
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared
// -ffp-contract=off keeps a*b+c as two roundings, like numpy / scipy / the
// oracle; the Brent search and the bracket are then bit-identical to scipy.
//
// Kernel map (one launch each per batch, all stream-ordered):
//   k_row_pairwise   once per table: numpy-order row sums (np.sum, elec.py:574;
//                    naep, ff:351)                          thread per row
//   k_row_slots      once per table: 576 (month, daytype, hour) slot sums
//                                                            thread per (row, slot)
//   k_size           Brent over PV kW (ff:440-447); each evaluation = sticky
//                    rate switch + 25-year bills + cash flow + NPV (ff:96-288),
//                    last-evaluation capture (ff:449-474)    thread per agent
//   k_hourly_batt    one sequential 8760 h scan per agent: baseline / PV-only
//                    hourly nets, battery sizing + storage rate switch +
//                    peak-shaving dispatch with SOC in registers (ff:130-164),
//                    per-(month, period) bins for the battery-case bill
//                                                            thread per agent
//   k_batt_finance   battery-case Utilityrate5 + Cashloan (ff:178-288)
//                                                            thread per agent
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <type_traits>

#include "../../include/dgen_hip.h"

// Two-agents-per-wave (32-lane) instantiations withdrawn by the build guard
// (dgen_amd/spill_guard.py): set to 1 by dgen_amd/build.py when the compiled
// kernel spills a live value ahead of a divergent branch's exec restore, so
// that its batches run one agent per wave (wave-uniform branches) instead.
#ifndef DGEN_NO2_SIZE
#define DGEN_NO2_SIZE 0
#endif
#ifndef DGEN_NO2_SIZE_DC
#define DGEN_NO2_SIZE_DC 0
#endif
#ifndef DGEN_NO2_FIN
#define DGEN_NO2_FIN 0
#endif
#ifndef DGEN_NO2_FIN_DC
#define DGEN_NO2_FIN_DC 0
#endif
#ifndef DGEN_NO2_SIZE_PK
#define DGEN_NO2_SIZE_PK 0
#endif
#ifndef DGEN_NO2_FIN_PK
#define DGEN_NO2_FIN_PK 0
#endif

namespace {

constexpr int NH = DGEN_NH;
constexpr int NSLOT = DGEN_NSLOT;
constexpr int MAXP = DGEN_MAXP;
constexpr int MAXT = DGEN_MAXT;
constexpr int MAXY = DGEN_MAXY;
constexpr int NBIN = 12 * MAXP;
constexpr int PREG = 4;   // periods whose NEM month recursion runs in registers
constexpr int DCP = DGEN_DCP;
constexpr int DCT = DGEN_DCT;
constexpr int BLOCK = 128;   // threads per block for the per-agent kernels
constexpr int HB_DAY_BYTES = 12 * 1024;   // k_hourly_batt day buffer per wave (LDS)
// hourly-plane stores every k_hourly_batt<true> day issues after its next-day
// DMA: 6 hour quads x 3 planes (the counted wait of the day pipeline)
constexpr int HB_STORES_AFTER_DMA = (24 / 4) * 3;
typedef __attribute__((address_space(3))) char* lds_ptr_t;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

// Metering options billed from hourly imports / exports (net billing: 2, and
// 3 = with $ carryover); 0 (NEM kWh), 1 (NEM $) and 4 (buy all / sell all)
// bill from the monthly (month, period) bins.  SAM's enumeration; the
// reference passes the tariff's value through (ff:586-588, 970-971).
__host__ __device__ __forceinline__ bool net_hourly(const dgen_tariff& t) { return t.mo == 2 || t.mo == 3; }

__constant__ int c_month_start_day[13] = {0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334, 365};
__constant__ int c_days_in_month[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};

thread_local char g_err[512] = {0};

void set_err(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

#define HIP_TRY(expr)                                                              \
    do {                                                                           \
        hipError_t _e = (expr);                                                    \
        if (_e != hipSuccess) {                                                    \
            set_err("%s failed: %s", #expr, hipGetErrorString(_e));                \
            return DGEN_E_HIP;                                                     \
        }                                                                          \
    } while (0)

// gen_per_kw = cf / 1e6 (ff:350) without the per-hour IEEE division: the
// reciprocal product corrected by one FMA residual step (Markstein) equals
// the correctly rounded quotient for every |cf| <= 2e7 (checked for each of
// those integers, tests/check_cf_div.c); larger values divide.
__device__ __forceinline__ double cf_per_kw(int32_t x) {
    const double a = (double)x;
    if (x > 20000000 || x < -20000000) return a / 1e6;
    constexpr double inv = 1.0 / 1e6;
    const double q = a * inv;
    const double r = __builtin_fma(-q, 1e6, a);
    return __builtin_fma(r, inv, q);
}

// cf_per_kw's common path (|x| <= 2e7, where it equals cf_per_kw); callers
// check the range
__device__ __forceinline__ double cf_per_kw_fast(int32_t x) {
    const double a = (double)x;
    constexpr double inv = 1.0 / 1e6;
    const double q = a * inv;
    const double r = __builtin_fma(-q, 1e6, a);
    return __builtin_fma(r, inv, q);
}

// ---------------------------------------------------------------------------
// numpy pairwise summation (loops_utils.h.src), chunked by the 8192-element
// reduction buffer; identical association order => bit-identical to np.sum.
// ---------------------------------------------------------------------------
template <class F>
__device__ double pw_leaf(const F& f, int off, int n) {
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; i++) res += f(off + i);
        return res;
    }
    double r0 = f(off + 0), r1 = f(off + 1), r2 = f(off + 2), r3 = f(off + 3);
    double r4 = f(off + 4), r5 = f(off + 5), r6 = f(off + 6), r7 = f(off + 7);
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
        r0 += f(off + i + 0); r1 += f(off + i + 1); r2 += f(off + i + 2); r3 += f(off + i + 3);
        r4 += f(off + i + 4); r5 += f(off + i + 5); r6 += f(off + i + 6); r7 += f(off + i + 7);
    }
    double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < n; i++) res += f(off + i);
    return res;
}

// Post-order walk of the pairwise split tree with an explicit stack.
template <class F>
__device__ double pw_sum(const F& f, int off, int n) {
    int so[16], sn[16], st[16];
    double sl[16];
    int sp = 0;
    so[0] = off; sn[0] = n; st[0] = 0; sp = 1;
    double ret = 0.0;
    bool have_ret = false;
    while (sp > 0) {
        int k = sp - 1;
        if (have_ret) {
            have_ret = false;
            if (st[k] == 1) {            // left child done -> run right child
                sl[k] = ret;
                st[k] = 2;
                int n2 = sn[k] / 2; n2 -= n2 % 8;
                so[sp] = so[k] + n2; sn[sp] = sn[k] - n2; st[sp] = 0; sp++;
            } else {                     // right child done -> combine
                ret = sl[k] + ret;
                sp--;
                have_ret = true;
            }
            continue;
        }
        if (sn[k] <= 128) {
            ret = pw_leaf(f, so[k], sn[k]);
            sp--;
            have_ret = true;
        } else {
            int n2 = sn[k] / 2; n2 -= n2 % 8;
            st[k] = 1;
            so[sp] = so[k]; sn[sp] = n2; st[sp] = 0; sp++;
        }
    }
    return ret;
}

template <class F>
__device__ double np_sum(const F& f, int n) {
    double res = 0.0;
    for (int s = 0; s < n; s += 8192) {
        int m = n - s < 8192 ? n - s : 8192;
        res += pw_sum(f, s, m);
    }
    return res;
}

struct ShapeVal {
    const float* p;
    __device__ double operator()(int i) const { return (double)p[i]; }
};
struct CfVal {
    const int32_t* p;
    __device__ double operator()(int i) const { return (double)p[i] / 1e6; }
};

__global__ void k_row_pairwise_shape(const float* __restrict__ rows, int64_t n_rows,
                                     double* __restrict__ out) {
    int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    ShapeVal f{rows + r * NH};
    out[r] = np_sum(f, NH);
}

__global__ void k_row_pairwise_cf(const int32_t* __restrict__ rows, int64_t n_rows,
                                  double* __restrict__ out) {
    int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    CfVal f{rows + r * NH};
    out[r] = np_sum(f, NH);
}

// slot = month * 48 + daytype * 24 + hour_of_day; day type from SSC's calendar
// (hour i is weekend iff (i % 168) >= 120: the year starts on a Monday).
template <class F>
__device__ double slot_sum(const F& f, int slot) {
    int m = slot / 48, dt = (slot / 24) % 2, hod = slot % 24;
    double acc = 0.0;
    for (int d = c_month_start_day[m]; d < c_month_start_day[m + 1]; d++) {
        int weekend = (d % 7) >= 5;
        if (weekend == dt) acc += f(d * 24 + hod);
    }
    return acc;
}

__global__ void k_row_slots_shape(const float* __restrict__ rows, int64_t n_rows,
                                  double* __restrict__ out) {
    int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_rows * NSLOT) return;
    int64_t r = g / NSLOT;
    int s = (int)(g % NSLOT);
    ShapeVal f{rows + r * NH};
    out[g] = slot_sum(f, s);
}

__global__ void k_row_slots_cf(const int32_t* __restrict__ rows, int64_t n_rows,
                               double* __restrict__ out) {
    int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_rows * NSLOT) return;
    int64_t r = g / NSLOT;
    int s = (int)(g % NSLOT);
    CfVal f{rows + r * NH};
    out[g] = slot_sum(f, s);
}

// ---------------------------------------------------------------------------
// Utilityrate5 subset (semantics: DESIGN.md "SSC subset"; oracle/orc.c)
// ---------------------------------------------------------------------------

// Dynamic LDS.  k_hourly_batt: per-lane (load, system) bin pairs [p][BLOCK];
// the year-lane kernels: YLds (below).
extern __shared__ double dyn_lds[];

// periods the LDS layouts are sized for (batch maximum, clamped to MAXP)
__host__ __device__ inline int lds_half(int max_periods) {
    return (max_periods > 0 && max_periods <= MAXP) ? max_periods : MAXP;
}

// ---------------------------------------------------------------------------
// Cashloan subset: one year's step of the after-tax cash flow
// ---------------------------------------------------------------------------
__device__ __forceinline__ double depr_frac(int type, int year, int sl) {
    if (type == 1) {   // MACRS 5-year half-year table (no local array: keeps it out of scratch)
        switch (year) {
            case 1: return 0.20;
            case 2: return 0.32;
            case 3: return 0.192;
            case 4: return 0.1152;
            case 5: return 0.1152;
            case 6: return 0.0576;
            default: return 0.0;
        }
    }
    if (type == 2) return (year >= 1 && year <= sl) ? 1.0 / (double)sl : 0.0;
    return 0.0;
}

// apply_rate_switch (elec.py:838-863): exactly one row with min <= size < max.
// the tariff's demand-charge record when demand charges are billed (extension mode)
__device__ __forceinline__ const dgen_demand* tariff_demand(const dgen_demand* table, int n_demand,
                                                            bool dc_on, const dgen_tariff& t) {
    const int dc = t.dc;
    return (dc_on && dc > 0 && dc <= n_demand) ? table + (dc - 1) : nullptr;
}
__device__ __forceinline__ const dgen_demand* tariff_demand(const dgen_tables& T, const dgen_cfg& cfg,
                                                            const dgen_tariff& t) {
    return tariff_demand(T.demand, T.n_demand, cfg.skip_demand_charges == 0, t);
}
// kWh/kW tier units (codes 1, 3): the caps scale with the month's peak import,
// which the demand machinery computes from the record `dc` points to (its flat
// peak), in either mode; its charges count only when demand charges are billed
__device__ __forceinline__ bool peak_unit(const dgen_tariff& t) { return t.unit == 1 || t.unit == 3; }
__device__ __forceinline__ const dgen_demand* tariff_peaks(const dgen_demand* table, int n_demand,
                                                           const dgen_tariff& t) {
    return peak_unit(t) ? tariff_demand(table, n_demand, true, t) : nullptr;
}

__device__ __forceinline__ double rate_switch(const dgen_switch* rows, int cnt, double size,
                                              int* new_tariff) {
    int hit = -1, k = 0;
    for (int r = 0; r < cnt; r++)
        if (rows[r].min_kw <= size && rows[r].max_kw > size) { k++; hit = r; }
    *new_tariff = -1;
    if (size > 0.0 && k == 1) {
        *new_tariff = rows[hit].tariff;
        return rows[hit].one_time_charge;
    }
    return 0.0;
}

__device__ __forceinline__ double np_sign(double v) {
    return (v > 0.0) ? 1.0 : ((v < 0.0) ? -1.0 : 0.0);
}

// scipy 1.15.3 _minimize_scalar_bounded, op for op (maxfun 500).  The
// objective is called from one site (the loop head), so the kernel carries one
// inlined copy of it: scipy's first evaluation and its loop evaluations run
// through the same call, the first one only seeding the state.
// trace (optional, one lane per agent): the objective value of evaluation k
// goes to trace[k] for k < BT_MAX -- the certified-path replay's input
// (k_brent_certify), whose x's are this loop's, recomputed from these values
constexpr int BT_MAX = 32;
template <class Obj>
__device__ __forceinline__ double brent_bounded(Obj&& f, double x1, double x2, double xatol, int* nfev,
                                double* x_last, double* trace = nullptr) {
    const double sqrt_eps = 1.4832396974191326e-08;     // sqrt(2.2e-16)
    const double golden_mean = 0.3819660112501051;      // 0.5 * (3 - sqrt(5))
    double a = x1, b = x2;
    double fulc = a + golden_mean * (b - a);
    double nfc = fulc, xf = fulc;
    double rat = 0.0, e = 0.0;
    double x = xf;
    double fx = 0.0, ffulc = 0.0, fnfc = 0.0;
    int num = 0;
    for (;;) {
        const double fu = f(x);
        *x_last = x;
        if (trace && num < BT_MAX) trace[num] = fu;
        num += 1;
        if (num == 1) {
            fx = fu;
            ffulc = fu;
            fnfc = fu;
        } else if (fu <= fx) {
            if (x >= xf) a = xf; else b = xf;
            fulc = nfc; ffulc = fnfc;
            nfc = xf; fnfc = fx;
            xf = x; fx = fu;
        } else {
            if (x < xf) a = x; else b = x;
            if ((fu <= fnfc) || (nfc == xf)) {
                fulc = nfc; ffulc = fnfc;
                nfc = x; fnfc = fu;
            } else if ((fu <= ffulc) || (fulc == xf) || (fulc == nfc)) {
                fulc = x; ffulc = fu;
            }
        }
        const double xm = 0.5 * (a + b);
        const double tol1 = sqrt_eps * fabs(xf) + xatol / 3.0;
        const double tol2 = 2.0 * tol1;
        if (num >= 500) break;
        if (!(fabs(xf - xm) > (tol2 - 0.5 * (b - a)))) break;
        bool golden = true;
        if (fabs(e) > tol1) {
            golden = false;
            double r = (xf - nfc) * (fx - ffulc);
            double q = (xf - fulc) * (fx - fnfc);
            double p = (xf - fulc) * q - (xf - nfc) * r;
            q = 2.0 * (q - r);
            if (q > 0.0) p = -p;
            q = fabs(q);
            r = e;
            e = rat;
            if ((fabs(p) < fabs(0.5 * q * r)) && (p > q * (a - xf)) && (p < q * (b - xf))) {
                rat = (p + 0.0) / q;
                x = xf + rat;
                if (((x - a) < tol2) || ((b - x) < tol2)) {
                    double si = np_sign(xm - xf) + (((xm - xf) == 0.0) ? 1.0 : 0.0);
                    rat = tol1 * si;
                }
            } else {
                golden = true;
            }
        }
        if (golden) {
            if (xf >= xm) e = a - xf; else e = b - xf;
            rat = golden_mean * e;
        }
        double si = np_sign(rat) + ((rat == 0.0) ? 1.0 : 0.0);
        double ar = fabs(rat);
        x = xf + si * (ar > tol1 ? ar : tol1);
    }
    *nfev = num;
    return xf;
}

struct WsLayout {
    // doubles, plane-major [k][n]
    double* carry;    // NBIN planes: [0] SOC, [1] annual PV kWh between month-segment launches
    double* aux;      // NBIN planes: [0] 1.0 where the storage switch changed the tariff
    double2* LGb;     // [n][NBIN] (load, system) bins, battery case, final tariff (2 NBIN planes)
    double* otc_b;    // 1 plane: storage one-time charge
    double* scratch;  // [8760][n_scratch] battery system output (mo 2)
    char* nb;         // [n_scratch][NB_BYTES] net-billing split records (k_size)
};

__host__ __device__ inline WsLayout ws_layout(void* base, int64_t n) {
    WsLayout w;
    double* p = (double*)base;
    w.carry = p; p += (int64_t)NBIN * n;
    w.aux = p; p += (int64_t)NBIN * n;
    w.LGb = reinterpret_cast<double2*>(p); p += (int64_t)2 * NBIN * n;
    w.otc_b = p; p += n;
    w.scratch = p;
    return w;
}
__host__ __device__ inline char* ws_nb(void* base, int64_t n, int64_t n_scratch) {
    return reinterpret_cast<char*>(base) + sizeof(double) * ((size_t)4 * NBIN * (size_t)n + (size_t)n +
                                                            (size_t)NH * (size_t)n_scratch);
}

// Phase timers (DGEN_PHASE_PROF=1 ablation builds only): per-segment shader
// cycles spent in a phase, summed over segments, read by dgen_phase_read.
// Slots 0-15: year-lane kernels -- 0 k_size, 1 set_tariff's net-billing split
// build or demand envelopes (build + stage), 2 / 3 net-billing evaluation
// (split / hourly) or 3 the demand-charge evaluation, 4 k_batt_finance, 5 / 6
// its split build / evaluation or 5 its staged demand pass, 7 / 8 split builds
// / evaluations counted (or envelope builds / demand evaluations), 9 Brent evaluations, 10 / 11 split entries visited /
// their loop, 12-15 NEM set_tariff, NEM bill, cash flow, prologue.  With
// DGEN_DAY_COUNTERS, 12-15 count k_hourly_batt day targets instead.
#ifndef DGEN_PHASE_PROF
#define DGEN_PHASE_PROF 0
#endif
#ifndef DGEN_DAY_COUNTERS          // k_hourly_batt day-target counters (slots 12-15)
#define DGEN_DAY_COUNTERS 0
#endif
// k_size's NEM phase timers use slots 12-15 unless the day counters do
#if DGEN_DAY_COUNTERS
#define PH_ADD_KS(k, v, lead) do {} while (0)
#else
#define PH_ADD_KS(k, v, lead) PH_ADD(k, v, lead)
#endif
#if DGEN_PHASE_PROF
__device__ unsigned long long g_phase[16];
#define PH_T0(v) const unsigned long long v = __builtin_readcyclecounter()
#define PH_ADD(k, v, lead) \
    do { if (lead) atomicAdd(&g_phase[k], __builtin_readcyclecounter() - (v)); } while (0)
#define PH_CNT(k, n, lead) \
    do { if (lead) atomicAdd(&g_phase[k], (unsigned long long)(n)); } while (0)
#else
#define PH_T0(v) do {} while (0)
#define PH_ADD(k, v, lead) do {} while (0)
#define PH_CNT(k, n, lead) do {} while (0)
#endif

__device__ __forceinline__ double pow_seq(double b, int e) {   // 1 * b * b ... (e times)
    double r = 1.0;
    for (int k = 0; k < e; k++) r = r * b;
    return r;
}

// Net-billing split records (see the net-billing split section below): per
// scratch slot, per (month, period) four sums linear in the generation scale
// and the month's mixed hours.
// NB_SYS_ZERO_IMPORT: in the battery case the hours where the battery takes
// the whole PV surplus have system output = load up to an ulp, i.e. an import
// of ~0 at s = 1 and a small one below; counted as mixed they overflowed the
// record for a third of the CA-like agents.  The battery-case splits (scan and
// plane build alike) put an hour whose import is above -slack at both ends of
// [s_lo, s_hi] on the import side: its linear term then bills at most the
// slack (1e-10 of the hour's load + generation) of export as negative import.
constexpr int NB_CAPM = DGEN_NB_CAPM;
// an M entry carries the hour's own inputs, so an evaluation reads one
// contiguous record instead of gathering the shape / cf (or system-output) /
// TS rows at scattered hours: load L, generation term g (cf / 1e6 per kW in
// the search, the system output in the battery case), the float32 sell
// weight w and the period
struct NbEnt {
    double L, g;
    float w;
    int p;
};
static_assert(sizeof(NbEnt) == 24, "24-B mixed-hour entries");
// The scan's compact form (k_hourly_batt, battery case, sell weight 1): the
// generation term, the hour's float32 shape value (the load is that x the
// load scale, exactly as the scan formed it, re-derived when the entry is
// fetched) and the period -- one 16-B store per mixed hour instead of 24 B in
// two stores.
struct NbEntC {
    double g;
    float sh;
    int p;
};
static_assert(sizeof(NbEntC) == 16, "16-B compact mixed-hour entries");
constexpr size_t NB_SUMS_BYTES = (size_t)12 * MAXP * 4 * sizeof(double);
constexpr size_t NB_BYTES = NB_SUMS_BYTES + 64 + (size_t)12 * NB_CAPM * sizeof(NbEnt);
static_assert(NB_BYTES % 16 == 0, "per-slot net-billing records stay 16-B aligned");
static_assert(NB_BYTES == DGEN_NB_BYTES, "include/dgen_hip.h DGEN_NB_BYTES");

struct NbRec {
    double* sums;        // [12][MAXP][4]: SA_L, SA_g, SX_gw, SX_Lw
    int* cnt;            // [12] M hours per month
    NbEnt* ent;          // [12][NB_CAPM]
};
// cnt[12]: 1 when k_hourly_batt built the battery case's split into the record
__device__ __forceinline__ int& nbr_flag(char* p) { return reinterpret_cast<int*>(p + NB_SUMS_BYTES)[12]; }
// cnt[13]: 1 + the tariff k_nb_env built the PV-only search's split for (0: none)
__device__ __forceinline__ int& nbr_tag(char* p) { return reinterpret_cast<int*>(p + NB_SUMS_BYTES)[13]; }
__device__ __forceinline__ NbRec nb_rec(char* p) {
    NbRec r;
    r.sums = reinterpret_cast<double*>(p);
    r.cnt = reinterpret_cast<int*>(p + NB_SUMS_BYTES);
    r.ent = reinterpret_cast<NbEnt*>(p + NB_SUMS_BYTES + 64);
    return r;
}


// Battery-case demand records (k_hourly_batt<.., DCR = true> -> k_batt_finance):
// per scratch slot, what the battery-case demand pass needs from the hours,
// built in the scan as the system output is produced.  Per (month, demand
// period): mxl = the max load (the no-system peak, exact) and lb = the running
// max over the hours of min(import at s_lo, import at s_hi) -- every year
// lane's import is between those two (fl(L - fl(sys s)) is monotone in s), so
// lb bounds every lane's peak from below; and in hour order the hours whose
// max(import at s_lo, import at s_hi) exceeds lb as it stood before them
// (16-B entries: system output, float32 shape value, period).  An hour not
// kept is at or below an earlier hour's import on every lane, so the lanes'
// peaks over the kept hours from 0 equal their peaks over all hours (maxima:
// bit-identical), and they may start from lb.  ~49 kept hours per agent-month
// on the C4 population (of 730; a study on the oracle's dispatch), against the
// staged pass's 8760 hours per lane group.  Entries of all months share one
// list (off[m] .. off[m + 1]); a list beyond DCR_CAP sets flag 2 and the
// finance kernel takes the staged pass over the system-output plane.
constexpr int DCR_CAP = DGEN_DCR_CAP;
struct DcrRec {
    double* lb;      // [12][DCP]
    double* mxl;     // [12][DCP]
    int* off;        // [13] entry offsets per month (running count)
    int* flag;       // 1: this step's scan built the record, 2: overflow, 0: none
    NbEntC* ent;     // [DCR_CAP]
};
constexpr size_t DCR_HEAD = (size_t)2 * 12 * DCP * sizeof(double) + 64;
constexpr size_t DCR_BYTES = DCR_HEAD + (size_t)DCR_CAP * sizeof(NbEntC);
static_assert(DCR_BYTES % 16 == 0, "per-slot demand records stay 16-B aligned");
__device__ __forceinline__ DcrRec dcr_rec(char* base, int64_t slot) {
    char* p = base + (size_t)slot * DCR_BYTES;
    DcrRec r;
    r.lb = reinterpret_cast<double*>(p);
    r.mxl = r.lb + 12 * DCP;
    r.off = reinterpret_cast<int*>(p + (size_t)2 * 12 * DCP * sizeof(double));
    r.flag = r.off + 13;
    r.ent = reinterpret_cast<NbEntC*>(p + DCR_HEAD);
    return r;
}

// ---------------------------------------------------------------------------
// k_hourly_batt: one sequential scan over the year per agent
// ---------------------------------------------------------------------------
// BatteryTools.battery_model_sizing restated (ff:140-147).
__device__ __forceinline__ void batt_size(double desired_kw, double desired_kwh, double v,
                                          const dgen_cfg& cfg, double* bank, double* power) {
    if (!(desired_kwh > 0.0)) { *bank = 0.0; *power = 0.0; return; }
    double series = ceil(v / cfg.batt_v_nom);
    double strings = floor(desired_kwh * 1000.0 / (cfg.batt_q_full * cfg.batt_v_nom * series) + 0.5);
    if (strings < 1.0) strings = 1.0;
    double b = cfg.batt_q_full * cfg.batt_v_nom * series * strings * 0.001;
    *bank = b;
    *power = b * (desired_kw / desired_kwh);
}

// Daily peak-shaving target (same algorithm as the oracle's day_target):
// smallest T >= 0 with f(T) = sum_h min(max(d_h - T, 0), P) <= E on the day's
// deficits d_h = max(load_h - pv_h, 0), sorted descending (s[0] = max).
// No saturated hour (s[0] <= P): f(T) = max_k (S_k - k T) with S_k the sum of
// the k largest, so T = (S_K - E) / K for the largest K with
// f(s[K-1]) = S_K - K s[K-1] <= E -- exact, one pass over the sorted day
// instead of the 4-5 Newton passes a wave ran before.  Otherwise bisection
// until no breakpoint (s_k, s_k - P) is inside the bracket, then the exact
// linear piece.  Every sum runs over the sorted order.
__device__ __forceinline__ void cswap_desc(double& a, double& b) {
    const double hi = fmax(a, b), lo = fmin(a, b);
    a = hi;
    b = lo;
}

// 132-comparator network (Batcher odd-even merge for 32 restricted to 24
// inputs), verified on all 2^24 binary inputs by scripts/gen_sortnet.py
__device__ __forceinline__ void sort24_desc(double (&v)[24]) {
    constexpr uint8_t net[132][2] = {
        {0, 1}, {2, 3}, {0, 2}, {1, 3}, {1, 2}, {4, 5}, {6, 7}, {4, 6}, {5, 7}, {5, 6}, {0, 4},
        {2, 6}, {2, 4}, {1, 5}, {3, 7}, {3, 5}, {1, 2}, {3, 4}, {5, 6}, {8, 9}, {10, 11}, {8, 10},
        {9, 11}, {9, 10}, {12, 13}, {14, 15}, {12, 14}, {13, 15}, {13, 14}, {8, 12}, {10, 14},
        {10, 12}, {9, 13}, {11, 15}, {11, 13}, {9, 10}, {11, 12}, {13, 14}, {0, 8}, {4, 12},
        {4, 8}, {2, 10}, {6, 14}, {6, 10}, {2, 4}, {6, 8}, {10, 12}, {1, 9}, {5, 13}, {5, 9},
        {3, 11}, {7, 15}, {7, 11}, {3, 5}, {7, 9}, {11, 13}, {1, 2}, {3, 4}, {5, 6}, {7, 8},
        {9, 10}, {11, 12}, {13, 14}, {16, 17}, {18, 19}, {16, 18}, {17, 19}, {17, 18}, {20, 21},
        {22, 23}, {20, 22}, {21, 23}, {21, 22}, {16, 20}, {18, 22}, {18, 20}, {17, 21}, {19, 23},
        {19, 21}, {17, 18}, {19, 20}, {21, 22}, {18, 20}, {19, 21}, {17, 18}, {19, 20}, {21, 22},
        {0, 16}, {8, 16}, {4, 20}, {12, 20}, {4, 8}, {12, 16}, {2, 18}, {10, 18}, {6, 22},
        {14, 22}, {6, 10}, {14, 18}, {2, 4}, {6, 8}, {10, 12}, {14, 16}, {18, 20}, {1, 17},
        {9, 17}, {5, 21}, {13, 21}, {5, 9}, {13, 17}, {3, 19}, {11, 19}, {7, 23}, {15, 23},
        {7, 11}, {15, 19}, {3, 5}, {7, 9}, {11, 13}, {15, 17}, {19, 21}, {1, 2}, {3, 4}, {5, 6},
        {7, 8}, {9, 10}, {11, 12}, {13, 14}, {15, 16}, {17, 18}, {19, 20}, {21, 22}};
#pragma unroll
    for (int c = 0; c < 132; c++) cswap_desc(v[net[c][0]], v[net[c][1]]);
}

__device__ __forceinline__ double day_target_sorted(const double (&s)[24], double power,
                                                    double avail, int* its = nullptr) {
    if (s[0] <= power) {
        // no hour above the power limit: need0 = sum_k min(s_k, P) is the
        // scan's total S_24 (the same additions in the same order), so one
        // pass decides the early-out and the target
        double S = 0.0, SK = s[0];
        int K = 1;
#pragma unroll
        for (int k = 1; k <= 24; k++) {
            S += s[k - 1];
            const bool ok = S - (double)k * s[k - 1] <= avail;
            K = ok ? k : K;
            SK = ok ? S : SK;
        }
        if (S <= avail) return 0.0;
        return (SK - avail) / (double)K;
    }
    double need0 = 0.0;
#pragma unroll
    for (int k = 0; k < 24; k++) need0 += fmin(s[k], power);
    if (need0 <= avail) return 0.0;
    int a_lo = 0, b_lo = 0;
#pragma unroll
    for (int k = 0; k < 24; k++) {
        a_lo += s[k] > 0.0;
        b_lo += (s[k] - power) >= 0.0;
    }
    double lo = 0.0, hi = s[0], f_hi = 0.0;
    int a_hi = 0, b_hi = 0;
    for (int it = 0; it < 48; it++) {
        if (a_lo == a_hi && b_lo == b_hi) break;
        if (its) ++*its;                 // phase-counter builds only
        const double mid = 0.5 * (lo + hi);
        double f = 0.0;
        int am = 0, bm = 0;
#pragma unroll
        for (int k = 0; k < 24; k++) {
            const double e = s[k] - mid;
            am += e > 0.0;
            bm += (e - power) >= 0.0;
            f += fmin(fmax(e, 0.0), power);
        }
        if (f <= avail) { hi = mid; f_hi = f; a_hi = am; b_hi = bm; }
        else { lo = mid; a_lo = am; b_lo = bm; }
    }
    const int k = a_hi - b_hi;
    if (k <= 0) return hi;
    double t = hi - (avail - f_hi) / (double)k;
    if (t < lo) t = lo;
    if (t > hi) t = hi;
    return t;
}

struct DayRaw {
    float s[24];
    int32_t c[24];
};

__device__ __forceinline__ double opaque(double x) {
    asm volatile("" : "+v"(x));
    return x;
}
__device__ __forceinline__ float opaque_f(float x) {
    asm volatile("" : "+v"(x));
    return x;
}
__device__ __forceinline__ int32_t opaque_i(int32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}

// Store of one lane's hour quad into a tile row, in the scalar-base form
// (global_store v_off, v_data, s[base]): the wave-uniform row base stays in
// SGPRs, the lane's 32-bit offset zero-extends, no per-store 64-bit vector
// address arithmetic.  The hourly output planes (105 KB per agent, read by
// nobody in the step) go out non-temporal so they do not evict the
// profile-row slices the resident waves share from L2 / MALL (1M agents:
// 33.2 -> 31.8 ms).  The store is invisible to the compiler's vmcnt
// bookkeeping, which only makes its waits stricter (vmcnt retires in order).
__device__ __forceinline__ void st_f32x4(char* row, uint32_t off, const float (&q)[4]) {
    const f32x4 v = {q[0], q[1], q[2], q[3]};
    asm volatile("global_store_dwordx4 %0, %1, %2 nt" :: "v"(off), "v"(v), "s"(row) : "memory");
}
// The fp64 planes' form (dgen_outputs.hourly_f64): the lane's 4 hours as 32 B,
// two stores
typedef double f64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st_f32x4(char* row, uint32_t off, const double (&q)[4]) {
    const f64x2 a = {q[0], q[1]}, b = {q[2], q[3]};
    asm volatile("global_store_dwordx4 %0, %1, %2 nt\n\t"
                 "global_store_dwordx4 %0, %3, %2 offset:16 nt"
                 :: "v"(off), "v"(a), "s"(row), "v"(b) : "memory");
}

// One hour of the dispatch (same arithmetic as the oracle's branchy
// orc_batt_dispatch, written without divergence): charge when the net load is
// negative, discharge towards the day's target otherwise.  With no battery
// (bank = power = 0) every clamp is 0 and sys = pv, g2l = max(nn, 0).
struct HourStep {
    double sys, g2l;
};
__device__ __forceinline__ HourStep batt_hour(double nn, double pv, double target, double power,
                                              double bank, double& soc, const dgen_cfg& cfg,
                                              double inv_eta_in, double in_per_bank,
                                              double out_per_bank) {
    const bool chg = nn < 0.0;
    // clamps as v_min/v_max (they can differ from the oracle's ternaries only in
    // the sign of a zero result, which no later sum or product can see)
    const double room = fmax((cfg.batt_max_soc - soc) * bank * inv_eta_in, 0.0);
    const double avail = fmax((soc - cfg.batt_min_soc) * bank * cfg.batt_eta_out, 0.0);
    const double cc = fmin(fmin(-nn, power), room);
    const double dd = fmin(fmin(fmax(nn - target, 0.0), power), avail);
    // f: the battery's flow to the load (-cc charging, dd discharging).
    // dsoc = -(f x k) is cc x k_in or -(dd x k_out) bit for bit (negation is
    // exact); g2l = max(nn - f, 0) is 0 charging (cc <= -nn) and nn - dd >= 0
    // discharging (dd <= nn) -- one select and one product fewer per hour
    const double f = chg ? -cc : dd;
    const double dsoc = -(f * (chg ? in_per_bank : out_per_bank));
    soc = soc + dsoc;
    HourStep r;
    r.sys = pv + f;
    r.g2l = fmax(nn - f, 0.0);
    return r;
}

// The same hour under the Li-ion loss model (dgen_cfg.batt_loss_model = 1;
// the oracle's orc_batt_dispatch loss branch, operation for operation):
// converters of efficiency eta each way and the cells' I^2 R at the bank's
// open-circuit voltage, k = r q v_nom / (bank v(soc)^2) at the hour's
// starting SOC (rqv = (r q) v_nom); the limits are the quadratics' roots.
__device__ __forceinline__ HourStep batt_hour_loss(double nn, double pv, double target, double power,
                                                   double bank, double& soc, const dgen_cfg& cfg,
                                                   double rqv, double eta) {
    const double v = cfg.batt_v_cell_empty + (cfg.batt_v_cell_full - cfg.batt_v_cell_empty) * soc;
    const double k = rqv / (bank * (v * v));
    HourStep r;
    if (nn < 0.0) {
        const double e_room = fmax((cfg.batt_max_soc - soc) * bank, 0.0);
        const double disc = 1.0 - 4.0 * k * e_room;
        const double x_max = disc > 0.0 ? 2.0 * e_room / (1.0 + sqrt(disc)) : 0.5 / k;
        double c = -nn;
        if (c > power) c = power;
        if (c > x_max / eta) c = x_max / eta;
        const double x = c * eta;
        soc = soc + (x - k * (x * x)) / bank;
        r.sys = pv - c;
        r.g2l = 0.0;
    } else {
        const double e_av = fmax((soc - cfg.batt_min_soc) * bank, 0.0);
        const double y_max = 2.0 * e_av / (1.0 + sqrt(1.0 + 4.0 * k * e_av));
        double d = nn - target;
        if (d < 0.0) d = 0.0;
        if (d > power) d = power;
        if (d > y_max * eta) d = y_max * eta;
        const double y = d / eta;
        soc = soc - (y + k * (y * y)) / bank;
        r.sys = pv + d;
        r.g2l = nn - d;
    }
    return r;
}

// 16 B per lane global -> LDS at lds + lane * 16 (m0 = wave-uniform base)
__device__ __forceinline__ void lds_dma16(const void* g, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off"
                 :: "v"(g), "s"(lds) : "memory", "m0");
}

// Read back a day buffer (lane's 12 chunks) after vmcnt(VM): chunk q of the
// shape row at +q KB, of the cf row at +(6 + q) KB.
template <int VM>
__device__ __forceinline__ void day_read(uint32_t a, DayRaw& r) {
    f32x4 s0, s1, s2, s3, s4, s5;
    i32x4 c0, c1, c2, c3, c4, c5;
    asm volatile("s_waitcnt vmcnt(%12)\n\t"
                 "ds_read_b128 %0, %13\n\t"
                 "ds_read_b128 %1, %13 offset:1024\n\t"
                 "ds_read_b128 %2, %13 offset:2048\n\t"
                 "ds_read_b128 %3, %13 offset:3072\n\t"
                 "ds_read_b128 %4, %13 offset:4096\n\t"
                 "ds_read_b128 %5, %13 offset:5120\n\t"
                 "ds_read_b128 %6, %13 offset:6144\n\t"
                 "ds_read_b128 %7, %13 offset:7168\n\t"
                 "ds_read_b128 %8, %13 offset:8192\n\t"
                 "ds_read_b128 %9, %13 offset:9216\n\t"
                 "ds_read_b128 %10, %13 offset:10240\n\t"
                 "ds_read_b128 %11, %13 offset:11264\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(s0), "=&v"(s1), "=&v"(s2), "=&v"(s3), "=&v"(s4), "=&v"(s5),
                   "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3), "=&v"(c4), "=&v"(c5)
                 : "n"(VM), "v"(a)
                 : "memory");
    const f32x4 sv[6] = {s0, s1, s2, s3, s4, s5};
    const i32x4 cv[6] = {c0, c1, c2, c3, c4, c5};
#pragma unroll
    for (int q = 0; q < 6; q++) {
        r.s[4 * q + 0] = sv[q].x; r.s[4 * q + 1] = sv[q].y; r.s[4 * q + 2] = sv[q].z; r.s[4 * q + 3] = sv[q].w;
        r.c[4 * q + 0] = cv[q].x; r.c[4 * q + 1] = cv[q].y; r.c[4 * q + 2] = cv[q].z; r.c[4 * q + 3] = cv[q].w;
    }
}

// One hour of the day buffer (ROLL: tomorrow's hour hh, after its DMA landed):
// shape at chunk hh / 4, cf at chunk 6 + hh / 4 (compile-time offsets).
__device__ __forceinline__ void day_hour(uint32_t a, int hh, float& s, int32_t& c) {
    const uint32_t o = (uint32_t)(hh >> 2) * 1024u + (uint32_t)(hh & 3) * 4u;
    asm volatile("ds_read_b32 %0, %2\n\t"
                 "ds_read_b32 %1, %3\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(s), "=&v"(c)
                 : "v"(a + o), "v"(a + o + 6144u)
                 : "memory");
}

// Read the day buffer again (no vmcnt wait: it already landed).
__device__ __forceinline__ void day_reread(uint32_t a, DayRaw& r) {
    f32x4 s0, s1, s2, s3, s4, s5;
    i32x4 c0, c1, c2, c3, c4, c5;
    asm volatile("ds_read_b128 %0, %12\n\t"
                 "ds_read_b128 %1, %12 offset:1024\n\t"
                 "ds_read_b128 %2, %12 offset:2048\n\t"
                 "ds_read_b128 %3, %12 offset:3072\n\t"
                 "ds_read_b128 %4, %12 offset:4096\n\t"
                 "ds_read_b128 %5, %12 offset:5120\n\t"
                 "ds_read_b128 %6, %12 offset:6144\n\t"
                 "ds_read_b128 %7, %12 offset:7168\n\t"
                 "ds_read_b128 %8, %12 offset:8192\n\t"
                 "ds_read_b128 %9, %12 offset:9216\n\t"
                 "ds_read_b128 %10, %12 offset:10240\n\t"
                 "ds_read_b128 %11, %12 offset:11264\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(s0), "=&v"(s1), "=&v"(s2), "=&v"(s3), "=&v"(s4), "=&v"(s5),
                   "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3), "=&v"(c4), "=&v"(c5)
                 : "v"(a)
                 : "memory");
    const f32x4 sv[6] = {s0, s1, s2, s3, s4, s5};
    const i32x4 cv[6] = {c0, c1, c2, c3, c4, c5};
#pragma unroll
    for (int q = 0; q < 6; q++) {
        r.s[4 * q + 0] = sv[q].x; r.s[4 * q + 1] = sv[q].y; r.s[4 * q + 2] = sv[q].z; r.s[4 * q + 3] = sv[q].w;
        r.c[4 * q + 0] = cv[q].x; r.c[4 * q + 1] = cv[q].y; r.c[4 * q + 2] = cv[q].z; r.c[4 * q + 3] = cv[q].w;
    }
}

// F64: the hourly planes as doubles (the reference's fp64 lists) instead of
// floats: the same values the scan computes, 32 B per lane per hour quad.
// NB: the batch has net-billing scratch slots; the scan then also builds the
// battery case's net-billing split (below) for the agents that bill net
// without a TS sell rate, so k_batt_finance bills them without a pass over
// the system-output plane.
// ROLL: the peak-shaving target is re-planned every hour over the next 24
// hours (dgen_cfg.batt_update_hours = 1) instead of once per calendar day.
// The window's deficits live in 24 registers (win) indexed by hour of day: at a
// day's start they are that day's; after hour hh is dispatched, slot hh takes
// tomorrow's hour hh (the window is a set, its order does not matter), read
// from the LDS day buffer, which in this form holds TOMORROW during the day
// (its DMA is waited for at the day's start).  In an hour where some lane can
// discharge, the wave sorts a copy of the window and runs the same target
// rule as the daily form -- the oracle's day_target over hours h .. h + 23,
// wrapping past December 31 to January 1.  The hour loop is unrolled like the
// daily form's (a rolled loop indexes the hour's registers dynamically, and
// the compiler then keeps the window and both days in scratch: 592 B per
// lane), so the network appears once per hour of the day (~27k instructions),
// and the form runs one wave per SIMD: the window, its sorted copy and both
// days' raw values need ~400 registers.
// DCR: the batch bills demand charges (or kWh/kW tier peaks) and has room for
// the battery-case demand records (dcr: DCR_BYTES per scratch slot, dc_nq the
// batch's demand periods, which size the scan's per-period LDS maxima).
// LOSS: the Li-ion loss model (dgen_cfg.batt_loss_model = 1, batt_hour_loss);
// instantiated without the scan-built records (NB, DCR), whose finance
// kernels then take the plane passes (equal results).
// NEM: the batch has no scratch slot (dgen_size_agents' n_scratch == 0), so no
// agent bills hourly imports: the bins path only, no system-output plane and
// no per-hour net-billing branch (an agent that would need one is flagged
// DGEN_ST_SCRATCH, as in every form).
// TS (with NB): the scan also builds the split of the agents billed net with
// the hourly TS sell rate (non-CA, metering option 2): their exported kWh are
// weighted by the hour's float32 sell rate, so the wave DMAs the agents' TS
// rows day by day next to the profile rows (12 KB more LDS per wave: this form
// runs one wave per SIMD and is launched for those agents alone, ts_mode 2,
// beside the NB form over the rest, ts_mode 1) and the record holds full
// 24-B entries (load, generation, weight, period; flag 4).
// ts_mode: 0 every agent; 1 the agents that can bill the TS rate (a scratch
// slot and a wholesale row, non-CA: engine.path_class 2) skipped; 2 only those.
// XP (with HOURLY, f32 semantics): the per-state export's combined plane
// instead of the three planes: per agent-hour the f64 value k_state_hourly
// adds, ((double)pvo x w_pvo + (double)wbt x w_batt) + (double)base x w_non of
// the float32-rounded plane values, in hour-quad tiles [h / 4][n][4] (8 B per
// agent-hour instead of 12, and k_state_hourly reads one plane, bit-identical)
// WO (with HOURLY, f32, daily plan): the with-battery plane alone (the
// model-year loop's per-state export recomputes the load and PV-only net load
// from the profile rows, dgen_state_hourly_rows): 4 B per agent-hour written
// instead of 12.
template <bool HOURLY, bool F64, bool NB, bool ROLL, bool DCR, bool LOSS = false, bool NEM = false, bool TS = false,
          bool XP = false, bool WO = false>
__global__ void __launch_bounds__(BLOCK, (ROLL || TS) ? 1 : 2)
k_hourly_batt(dgen_tables T, dgen_agents A, dgen_outputs O, dgen_cfg cfg, int64_t n, void* ws,
              int64_t n_scratch, int64_t i0, int64_t i1, int m_lo, int m_hi, int batt_on, int nb_cap,
              int repair, char* dcr, int dc_nq, int dcr_cap, int ts_mode = 0,
              const double* xw_pvo = nullptr, const double* xw_batt = nullptr, const double* xw_non = nullptr,
              double* xplane = nullptr) {
    // agents [i0, i1) of a batch of n (row stride of every plane stays n),
    // months [m_lo, m_hi) of the year: the year is swept in month segments,
    // one launch each, so that every resident wave works on the same weeks
    // and the profile-row slices they read stay in L2 / MALL (SOC and the
    // running annual PV sum carry between launches in W.carry)
    int64_t i = i0 + (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= i1) return;
    // the TS agents' scan runs one wave per SIMD beside the other parts' waves
    // and is the national step's critical path: its waves issue first
    // (national 200k k_hourly_batt 8.5 -> 8.2 ms, profiles/r05/ts_prio)
    if constexpr (TS) __builtin_amdgcn_s_setprio(3);
    if (O.status[i] & (DGEN_ST_BOUNDS | DGEN_ST_TARIFF | DGEN_ST_YEARS)) return;
    if (ts_mode) {
        const bool ts_cap = A.scratch_slot[i] >= 0 && A.wholesale_row[i] >= 0 && (A.flags[i] & 2) == 0 &&
                            T.wholesale != nullptr;
        if (ts_cap != (ts_mode == 2)) return;
    }
    // repair pass: only the agents whose scan-built split (repair bit 1) or
    // demand record (bit 2) overflowed and whose system-output plane was
    // therefore not written (flag 2) run again, with the plane; every other
    // output it writes is the same value again
    if (repair) {
        const int sl = A.scratch_slot[i];
        const bool need = sl >= 0 &&
            (((repair & 1) && nbr_flag(ws_nb(ws, n, n_scratch) + (size_t)sl * NB_BYTES) == 2) ||
             ((repair & 2) && dcr && *dcr_rec(dcr, sl).flag == 2));
        if (!need) return;
    }
    WsLayout W = ws_layout(ws, n);
    // battery-case bins: (load, system output) pairs per period, [p][BLOCK]
    double2* bins = reinterpret_cast<double2*>(dyn_lds) + threadIdx.x;
    const bool is_res = (A.flags[i] & 1) != 0;
    const int lr = A.load_row[i], cr = A.cf_row[i];
    const double kwh = A.load_kwh[i];
    const double ls = kwh / T.shape_sum[lr];                     // load = shape * ls
    // an agent k_size left unsized (kWh/kW tier units) keeps its no-system
    // hourly planes (load as is), so per-state and chunk sums stay finite
    const bool unsized = (O.status[i] & DGEN_ST_UNIT) != 0;
    const double kw_star = unsized ? 0.0 : O.system_kw[i];
    const double x_last = unsized ? 0.0 : O.x_last[i];
    // pv = cf * (c / 1e6), c = ((kW * 1000) * 0.96) / 1000   (ff:118-120)
    const double cl6 = (((x_last * 1000.0) * 0.96) / 1000.0) / 1e6;
    const double cs6 = (((kw_star * 1000.0) * 0.96) / 1000.0) / 1e6;
    const float* __restrict__ shp = T.shapes + (int64_t)lr * NH;
    const int32_t* __restrict__ cfp = T.cfs + (int64_t)cr * NH;

    // battery sizing at kW* (ff:140-147) and the storage rate switch (ff:167-175)
    double desired_kwh = kw_star / 0.8, desired_kw = desired_kwh / 2.0;
    double bank = 0.0, power = 0.0;
    if (batt_on) batt_size(desired_kw, desired_kwh, is_res ? 240.0 : 500.0, cfg, &bank, &power);
    int tariff = O.tariff_final[i];
    int switched = O.switched[i];
    double otc = 0.0;
    if (bank > 0.0) {
        const dgen_switch* rows = T.switches + A.sw_storage_off[i];
        int cnt = A.sw_storage_cnt[i], hit = -1, k = 0;
        for (int r = 0; r < cnt; r++)
            if (rows[r].min_kw <= bank && rows[r].max_kw > bank) { k++; hit = r; }
        if (k == 1) { tariff = rows[hit].tariff; switched = 1; otc = rows[hit].one_time_charge; }
    }
    const dgen_tariff& t = T.tariffs[tariff];
    const int P = t.P;
    const bool mo2 = !NEM && net_hourly(t);     // hourly imports (net billing 2 / 3), else bins
    const int slot = A.scratch_slot[i];
    // the battery-case bill reads the hourly system output for net billing and
    // for demand charges (both need hourly imports, not bins)
    const bool has_dc = tariff_demand(T, cfg, t) != nullptr ||
                        tariff_peaks(T.demand, T.n_demand, t) != nullptr;   // kWh/kW tiers: peaks
    const bool need_sys = net_hourly(t) || has_dc;
    const bool put_sys = !NEM && need_sys && slot >= 0 && batt_on;
    int status = O.status[i] | t.flags;
    if (need_sys && slot < 0 && batt_on) status |= DGEN_ST_SCRATCH;
    // The battery case's net-billing split over the agent's degradation range
    // [s_lo, s_hi] (what k_batt_finance's yl_nb_build<true> builds from the
    // plane), classified hour by hour as the scan produces the system output:
    // import at both ends (import load / generation sums), export at both
    // ends (export generation / load sums, sell weight 1: no TS rate), else a
    // mixed entry in hour order.  Sums per (month, period) in the LDS bins
    // (import) and bins2 (export), the current period's in registers.
    bool put_nb = false;
    bool nb_over = false;        // a month's mixed hours exceeded nb_cap
    bool nb_full = false;        // TS: full entries with the hour's sell weight
    double nb_lo = 0.0, nb_hi = 0.0;
    NbRec nbr{nullptr, nullptr, nullptr};
    if constexpr (NB) {
        const bool is_ca = (A.flags[i] & 2) != 0;
        const bool ts_on = t.mo == 2 && !is_ca && A.wholesale_row[i] >= 0 && T.wholesale != nullptr;
        put_nb = put_sys && mo2 && (TS || !ts_on) && nb_cap > 0;
        nb_full = TS && ts_on && put_nb;
        if (put_nb) {
            const int N = A.econ_life[i];
            const double sys_base = 1.0 - (A.pv_deg[i] * 100.0) * 0.01;
            const double sN = pow_seq(sys_base, (N >= 1 && N <= MAXY) ? N - 1 : 0);
            nb_lo = sN < 1.0 ? sN : 1.0;
            nb_hi = sN > 1.0 ? sN : 1.0;
            nbr = nb_rec(ws_nb(ws, n, n_scratch) + (size_t)slot * NB_BYTES);
        }
    }
    // battery-case demand record (DcrRec) over the schedule the finance kernel
    // bills with: the kWh/kW tier peaks' record where the batch bills those,
    // else the tariff's demand charges; the year lanes' degradation range
    // [dc_lo, dc_hi] as in the finance kernel (s_y for y = 1 .. N)
    bool put_dcr = false;
    DcrRec dr{nullptr, nullptr, nullptr, nullptr, nullptr};
    const dgen_demand* dcd = nullptr;
    double dc_lo = 1.0, dc_hi = 1.0;
    int n_d = 0;
    if constexpr (DCR) {
        if (dcr && slot >= 0 && !repair) {
            dr = dcr_rec(dcr, slot);
            const dgen_demand* pkd = T.peak_units ? tariff_peaks(T.demand, T.n_demand, t) : nullptr;
            dcd = pkd ? pkd : tariff_demand(T, cfg, t);
            put_dcr = put_sys && dcd != nullptr;
            if (m_lo == 0) { *dr.flag = 0; dr.off[0] = 0; }
            if (put_dcr) {
                const int N = A.econ_life[i];
                const double sys_base = 1.0 - (A.pv_deg[i] * 100.0) * 0.01;
                const double sN = pow_seq(sys_base, (N >= 1 && N <= MAXY) ? N - 1 : 0);
                dc_lo = sN < 1.0 ? sN : 1.0;
                dc_hi = sN > 1.0 ? sN : 1.0;
                n_d = m_lo == 0 ? 0 : dr.off[m_lo];
            }
        }
    }
    // the split replaces the system-output plane for the energy bill; demand
    // charges still read the plane, and an overflowing split gets it from the
    // repair pass.  A demand record replaces it for an agent billed from bins
    // (NEM: the energy bill does not read hours), the same way.
    const bool skip_plane = (put_nb && !has_dc) || (DCR && put_dcr && !mo2);

    const double inv_eta_in = 1.0 / cfg.batt_eta_in;
    const double in_per_bank = bank > 0.0 ? cfg.batt_eta_in / bank : 0.0;
    const double out_per_bank = bank > 0.0 ? 1.0 / (cfg.batt_eta_out * bank) : 0.0;
    const bool has_batt = bank > 0.0;
    if (!has_batt) power = 0.0;
    const double rqv = LOSS ? cfg.batt_r_cell * cfg.batt_q_full * cfg.batt_v_nom : 0.0;   // loss model: r q v_nom
    double soc = m_lo == 0 ? cfg.batt_init_soc : W.carry[i];
    double annual = m_lo == 0 ? 0.0 : W.carry[n + i];
    const int d_lo = c_month_start_day[m_lo];
    // hour rows: wave-uniform bases advanced per row; per-lane 32-bit byte
    // offsets (host guarantees n < 2^28, n_scratch < 2^28)
    // system-output scratch plane in day tiles [365][n_scratch][24] f64
    // (sys_index): a lane stores each hour quad as 32 contiguous bytes of its
    // 192-B day, a reader loads a quad as two 16-B loads (sys_quad)
    const size_t off192 = (size_t)(put_sys ? slot : 0) * 192u;
    const size_t row192 = (size_t)n_scratch * 192u;
    char* const ob = reinterpret_cast<char*>(O.baseline);
    char* const op = reinterpret_cast<char*>(O.net_pvonly);
    char* const ow = reinterpret_cast<char*>(O.net_with_batt);
    char* const osc = reinterpret_cast<char*>(W.scratch);
    size_t hd192 = (size_t)d_lo * row192;                // the current day's tile
    double qs[4] = {0.0, 0.0, 0.0, 0.0};
    // hourly planes in hour-quad tiles (include/dgen_hip.h): (hour h, agent i)
    // at ((h / 4) * n + i) * 4 + h % 4, so a lane stores 16 B and a wave 1 KB
    // contiguous per plane every 4 hours (measured 29.3 -> 27.9 ms vs one
    // 4-B store per lane-hour)
    using PT = typename std::conditional<F64, double, float>::type;
    constexpr uint32_t QB = (XP ? 8 : sizeof(PT)) * 4;   // bytes per lane per hour quad
    const uint32_t off16 = (uint32_t)i * QB;
    const size_t row16 = (size_t)n * QB;
    size_t q16 = (size_t)d_lo * 6 * row16;
    PT qb[4], qp[4], qw[4];
    // XP: the agent's export weights and the combined plane
    const double xa = XP ? xw_pvo[i] : 0.0, xb = XP ? xw_batt[i] : 0.0, xd = XP ? xw_non[i] : 0.0;
    char* const ox = reinterpret_cast<char*>(xplane);
    (void)ox;

    // Software pipeline over days through LDS: the next day's raw profile
    // values (96 B of the shape row + 96 B of the cf row per lane) are DMA'd
    // global -> LDS (global_load_lds_dwordx4: no VGPRs held in flight) at the
    // start of the current day, BEFORE the day's hourly stores.  vmcnt is
    // shared by loads and stores and retires in issue order, so at the next
    // day start vmcnt(HB_STORES_AFTER_DMA) implies the DMA landed while the
    // day's last stores may still be in flight: every day issues at least
    // HB_STORES_AFTER_DMA = 6 hour quads x 3 planes asm stores after its DMA
    // (plus 12 scratch stores with put_sys, which only make the wait
    // stricter).  The day loop issues no compiler-visible load (the period
    // schedule is loaded per month, below): the compiler's own waits count
    // only the ops it sees, so a load pending in the loop would get a
    // vmcnt(0) at its first use that drains every store of the day.  DMA and
    // read-back are inline asm: the compiler would otherwise order every LDS
    // access of the kernel (the bins) behind a vmcnt(0).  Per wave: 12 chunks
    // x 64 lanes x 16 B = HB_DAY_BYTES.  (ISA check: DESIGN.md section 5.)
    // DCR: per-period (max load, lb) pairs [dc_nq][BLOCK] after the bins
    double2* const dcb = reinterpret_cast<double2*>(reinterpret_cast<char*>(dyn_lds) +
                         (size_t)(NB ? 32 : 16) * lds_half(T.max_periods) * BLOCK) + threadIdx.x;
    const uint32_t dbase = (uint32_t)(size_t)(lds_ptr_t)(reinterpret_cast<char*>(dyn_lds) +
                           (size_t)(NB ? 32 : 16) * lds_half(T.max_periods) * BLOCK +
                           (DCR ? (size_t)16 * dc_nq * BLOCK : 0) +
                           (size_t)(threadIdx.x / 64) * HB_DAY_BYTES * (TS ? 2 : 1));
    const uint32_t dbase_s = __builtin_amdgcn_readfirstlane(dbase);
    const uint32_t dlane = dbase_s + (threadIdx.x & 63u) * 16u;
    // TS: the lane's chunks of the TS day (a pointer into dyn_lds: ds_read)
    const char* const tsl = reinterpret_cast<const char*>(dyn_lds) + (size_t)(NB ? 32 : 16) * lds_half(T.max_periods) * BLOCK +
                            (DCR ? (size_t)16 * dc_nq * BLOCK : 0) +
                            (size_t)(threadIdx.x / 64) * HB_DAY_BYTES * 2 + HB_DAY_BYTES + (threadIdx.x & 63u) * 16u;
    (void)tsl;
    // TS: the agent's TS row (a path-2 agent always has one), its day in 12
    // more chunks after the profile rows' (2 hours each)
    const double* __restrict__ tsp = TS ? T.wholesale + (int64_t)(A.wholesale_row[i] >= 0 ? A.wholesale_row[i] : 0) * NH
                                        : nullptr;
    const double ts_mult = TS ? A.price_mult[i] : 1.0;
    auto day_dma = [&](int dd) {
#pragma unroll
        for (int q = 0; q < 6; q++) {
            lds_dma16(shp + dd * 24 + 4 * q, dbase_s + q * 1024u);
            lds_dma16(cfp + dd * 24 + 4 * q, dbase_s + (6 + q) * 1024u);
        }
        if constexpr (TS) {
#pragma unroll
            for (int q = 0; q < 12; q++) lds_dma16(tsp + dd * 24 + 2 * q, dbase_s + HB_DAY_BYTES + q * 1024u);
        }
    };
    float tw[24];                  // TS: the day's sell weights (float)(rate x price multiplier)
    (void)tw;
    // settle every load before the day loop: the waitcnt pass merges the
    // loop entry with the back edge, and a pending entry load would put a
    // vmcnt wait (which also drains the in-flight day DMA) into hour 0
    __builtin_amdgcn_s_waitcnt(0x0f70);                  // vmcnt(0)
    day_dma(d_lo);
    const int d_last = c_month_start_day[m_hi] - 1;
    DayRaw r;
    double win[24];                // ROLL: the 24-hour window's deficits by hour of day
    (void)win;
    double2* const bins2 = bins + (size_t)lds_half(T.max_periods) * BLOCK;   // NB: export sums
    for (int m = m_lo; m < m_hi; m++) {
        for (int p = 0; p < P; p++) bins[p * BLOCK] = make_double2(0.0, 0.0);
        if (NB && put_nb)
            for (int p = 0; p < P; p++) bins2[p * BLOCK] = make_double2(0.0, 0.0);
        double2 xacc = make_double2(0.0, 0.0);
        int n_m = 0;
        NbEntC* const nb_ent = (NB && put_nb) ? reinterpret_cast<NbEntC*>(nbr.ent) + m * NB_CAPM : nullptr;
        // monthly target floor (dgen_cfg.batt_month_floor): the largest target
        // planned so far this month (a month-segment launch starts at a month)
        double mfloor = 0.0;
        // the current period's bin in registers (the same additions in the same
        // order as a per-hour LDS read-modify-write), written back when the
        // period changes and at the month's end
        int bcur = 0;
        double2 bacc = make_double2(0.0, 0.0);
        // the month's weekday / weekend period rows (24 bytes each, 8-aligned)
        // in 6 registers, loaded once per month: the day loop below then
        // issues no compiler-visible load (see the pipeline note above); the
        // compiler's wait for these lands in the month's first hour
        uint64_t swd[3], swe[3];
        {
            const uint64_t* a = reinterpret_cast<const uint64_t*>(t.wkday[m]);
            const uint64_t* b = reinterpret_cast<const uint64_t*>(t.wkend[m]);
            swd[0] = a[0]; swd[1] = a[1]; swd[2] = a[2];
            swe[0] = b[0]; swe[1] = b[1]; swe[2] = b[2];
        }
        // DCR: the month's demand-period rows, loaded with the energy rows; the
        // current period's (max load, lb) in registers like the bins
        uint64_t dsd[3] = {0, 0, 0}, dse[3] = {0, 0, 0};
        int dq = 0;
        double2 dacc = make_double2(0.0, 0.0);
        const int d_first = n_d;                      // the month's first kept hour
        (void)d_first;
        if (DCR && put_dcr) {
            const uint64_t* a = reinterpret_cast<const uint64_t*>(dcd->wkday[m]);
            const uint64_t* b = reinterpret_cast<const uint64_t*>(dcd->wkend[m]);
            dsd[0] = a[0]; dsd[1] = a[1]; dsd[2] = a[2];
            dse[0] = b[0]; dse[1] = b[1]; dse[2] = b[2];
            for (int q = 0; q < dc_nq; q++) dcb[q * BLOCK] = make_double2(0.0, 0.0);
        }
        // the month's schedule rows land here, once per month: left pending,
        // the compiler's wait for them can fall inside the day loop, where
        // (loop-carried) it drains every day's stores and the next-day DMA
        __builtin_amdgcn_s_waitcnt(0x0f70);                  // vmcnt(0)
        for (int d = c_month_start_day[m]; d < c_month_start_day[m + 1]; d++) {
            if (ROLL && d > d_lo) day_reread(dlane, r);    // the DMA was waited for yesterday
            else if (HOURLY && d > d_lo) day_read<XP ? 12 : (WO ? 6 : HB_STORES_AFTER_DMA * (F64 ? 2 : 1))>(dlane, r);
            else day_read<0>(dlane, r);
            const bool wkend = (d % 7) >= 5;
            const uint64_t sched[3] = {wkend ? swe[0] : swd[0], wkend ? swe[1] : swd[1],
                                       wkend ? swe[2] : swd[2]};
            const uint64_t dsch[3] = {wkend ? dse[0] : dsd[0], wkend ? dse[1] : dsd[1],
                                      wkend ? dse[2] : dsd[2]};
            (void)dsch;
            double target = 0.0;
            if constexpr (ROLL) {
                // the window at the day's first hour is the day itself; then the
                // day after (January 1 after December 31) comes in as it is read
#pragma unroll
                for (int hh = 0; hh < 24; hh++)
                    win[hh] = fmax((double)r.s[hh] * ls - (double)r.c[hh] * cs6, 0.0);
                day_dma(d + 1 < 365 ? d + 1 : 0);
                // tomorrow's values are read from the buffer hour by hour
                // (below): wait here until its DMA has landed
                __builtin_amdgcn_s_waitcnt(0x0f70);        // vmcnt(0)
            } else if (has_batt) {
                // the day's deficits d_h = max(load_h - pv_h, 0), sorted; the raw
                // registers are dead meanwhile and re-read from the LDS buffer
                double dv[24];
#pragma unroll
                for (int hh = 0; hh < 24; hh++)
                    dv[hh] = fmax((double)r.s[hh] * ls - (double)r.c[hh] * cs6, 0.0);
                sort24_desc(dv);
                // deliverable energy of the plan (the loss model's without the
                // cell losses: the oracle's e_av x eta)
                const double avail = LOSS ? fmax((soc - cfg.batt_min_soc) * bank, 0.0) * cfg.batt_conv_eff
                                          : fmax((soc - cfg.batt_min_soc) * bank * cfg.batt_eta_out, 0.0);
#if DGEN_PHASE_PROF && DGEN_DAY_COUNTERS
                int its = 0;
                target = day_target_sorted(dv, power, avail, &its);
                {   // 12: battery lane-days, 13: lane-days whose whole need fits
                    // (target 0), 14: wave-days where it fits for every lane,
                    // 15: saturated lane-days (an hour above the power limit)
                    double need = 0.0;
                    for (int k = 0; k < 24; k++) need += fmin(dv[k], power);
                    const bool fits = need <= avail;
                    const unsigned long long act = __ballot(1), fit = __ballot(fits),
                                             sat = __ballot(dv[0] > power);
                    const bool lead = (int)(threadIdx.x & 63u) == __ffsll((long long)act) - 1;
                    PH_CNT(12, __popcll(act), lead);
                    PH_CNT(13, __popcll(fit), lead);
                    PH_CNT(14, fit == act, lead);
                    PH_CNT(15, __popcll(sat), lead);
                    (void)its;
                }
#else
                target = day_target_sorted(dv, power, avail);
#endif
                if (cfg.batt_month_floor) {           // the month's target never falls
                    if (target < mfloor) target = mfloor;
                    else mfloor = target;
                }
                day_reread(dlane, r);
            }
            if constexpr (TS) {   // the day's weights, before the next-day DMA reuses the buffer
                f64x2 tv[12];
#pragma unroll
                for (int q = 0; q < 12; q++) tv[q] = *reinterpret_cast<const f64x2*>(tsl + q * 1024u);
#pragma unroll
                for (int q = 0; q < 12; q++) {
                    tw[2 * q] = (float)(tv[q].x * ts_mult);
                    tw[2 * q + 1] = (float)(tv[q].y * ts_mult);
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);           // lgkmcnt(0): the reads are done
            }
            if (!ROLL && d < d_last) day_dma(d + 1);            // after the last read of the buffer
            const double ls2 = opaque(ls), cs2 = opaque(cs6), cl2 = opaque(cl6);
#pragma unroll
            for (int hh = 0; hh < 24; hh++) {
                const double ld = (double)opaque_f(r.s[hh]) * ls2;
                const double cfv = (double)opaque_i(r.c[hh]);
                const double pl = cfv * cl2;                 // PV-only run (x_last)
                annual += pl;
                const double pv = cfv * cs2;                 // battery run (kW*)
                const double nn = ld - pv;
                if constexpr (ROLL) {
                    // this hour's plan over hours h .. h + 23, from the energy
                    // stored now; only an hour that can discharge needs one
                    // (elsewhere the dispatch is the same for any target)
                    const double av = LOSS ? fmax((soc - cfg.batt_min_soc) * bank, 0.0) * cfg.batt_conv_eff
                                           : fmax((soc - cfg.batt_min_soc) * bank * cfg.batt_eta_out, 0.0);
                    const bool need = has_batt && nn > 0.0 && av > 0.0;
                    target = 0.0;
                    if (__ballot(need)) {
                        double dv[24];
#pragma unroll
                        for (int k = 0; k < 24; k++) dv[k] = win[k];
                        sort24_desc(dv);
                        double t = day_target_sorted(dv, power, av);
                        if (cfg.batt_month_floor && need) {
                            if (t < mfloor) t = mfloor;
                            else mfloor = t;
                        }
                        target = need ? t : 0.0;
                    }
                }
                HourStep st;
                if constexpr (LOSS) {
                    if (has_batt) st = batt_hour_loss(nn, pv, target, power, bank, soc, cfg, rqv, cfg.batt_conv_eff);
                    else { st.sys = pv; st.g2l = fmax(nn, 0.0); }
                } else {
                    st = batt_hour(nn, pv, target, power, bank, soc, cfg, inv_eta_in, in_per_bank, out_per_bank);
                }
                if constexpr (ROLL) {   // the window moves on: tomorrow's hour hh comes in
                    float ts;
                    int32_t tc;
                    day_hour(dlane, hh, ts, tc);
                    win[hh] = fmax((double)ts * ls - (double)tc * cs6, 0.0);
                }
                if constexpr (HOURLY) {
                    const double dn = ld - pl;
                    qb[hh & 3] = (PT)ld;
                    qp[hh & 3] = (PT)fmax(dn, 0.0);
                    qw[hh & 3] = (PT)st.g2l;
                    if ((hh & 3) == 3) {
                        if constexpr (XP) {
                            double xv[4];
#pragma unroll
                            for (int u = 0; u < 4; u++)
                                xv[u] = ((double)qp[u] * xa + (double)qw[u] * xb) + (double)qb[u] * xd;
                            st_f32x4(ox + q16, off16, xv);
                        } else if constexpr (WO) {
                            st_f32x4(ow + q16, off16, qw);
                        } else {
                            st_f32x4(ob + q16, off16, qb);
                            st_f32x4(op + q16, off16, qp);
                            st_f32x4(ow + q16, off16, qw);
                        }
                        q16 += row16;
                    }
                }
                if constexpr (DCR) {
                    if (put_dcr) {
                        int q = (int)((dsch[hh >> 3] >> (8 * (hh & 7))) & 0xffu);
                        // dc_nq (dgen_tables.max_dc_periods) sizes the per-period
                        // LDS maxima: a schedule beyond it is a malformed table
                        // (flagged, never written past the region)
                        if (q >= dc_nq) { status |= DGEN_ST_DEMAND; q = 0; }
                        if (q != dq) {
                            dcb[dq * BLOCK] = dacc;
                            dq = q;
                            dacc = dcb[q * BLOCK];
                        }
                        const double i_lo = ld - st.sys * dc_lo, i_hi = ld - st.sys * dc_hi;
                        if (fmax(i_lo, i_hi) > dacc.y) {       // may raise some lane's peak
                            if (n_d < dcr_cap) {
                                NbEntC e;
                                e.g = st.sys;
                                e.sh = r.s[hh];
                                e.p = q;
                                dr.ent[n_d] = e;
                            }
                            n_d++;
                        }
                        dacc.x = fmax(dacc.x, ld);
                        dacc.y = fmax(dacc.y, fmin(i_lo, i_hi));
                    }
                }
                qs[hh & 3] = st.sys;
                if ((hh & 3) == 3) {
                    if (put_sys && !skip_plane) {               // tile [d][slot][24], quad hh / 4
                        double2* q = reinterpret_cast<double2*>(osc + hd192 + off192 + (size_t)(hh >> 2) * 32u);
                        q[0] = make_double2(qs[0], qs[1]);
                        q[1] = make_double2(qs[2], qs[3]);
                    }
                    if (hh == 23) hd192 += row192;
                }
                if (!mo2) {   // NEM energy bill from bins (demand charges also read the plane)
                    const int p = (int)((sched[hh >> 3] >> (8 * (hh & 7))) & 0xffu);
                    if (p != bcur) {
                        bins[bcur * BLOCK] = bacc;
                        bcur = p;
                        bacc = bins[p * BLOCK];
                    }
                    bacc.x += ld;
                    bacc.y += st.sys;
                } else if (NB && put_nb) {   // battery-case net-billing split
                    const int p = (int)((sched[hh >> 3] >> (8 * (hh & 7))) & 0xffu);
                    if (p != bcur) {
                        bins[bcur * BLOCK] = bacc;
                        bins2[bcur * BLOCK] = xacc;
                        bcur = p;
                        bacc = bins[p * BLOCK];
                        xacc = bins2[p * BLOCK];
                    }
                    const double gk = st.sys;
                    const double vlo = ld - gk * nb_lo, vhi = ld - gk * nb_hi;
                    const double slack = 1e-10 * (fabs(ld) + fabs(gk) * nb_hi);
                    const bool imp = fmin(vlo, vhi) > -slack;              // imports (or ~0) at every s
                    const bool exq = !imp && fmax(vlo, vhi) < -slack;      // exports at every s
                    bacc.x += imp ? ld : 0.0;
                    bacc.y += imp ? gk : 0.0;
                    // the export side x the hour's sell weight (yl_nb_build<true>'s
                    // products; 1 without a TS rate: gk x 1.0 is gk)
                    const double wd = nb_full ? (double)tw[hh] : 1.0;
                    xacc.x += exq ? gk * wd : 0.0;
                    xacc.y += exq ? ld * wd : 0.0;
                    if (!imp && !exq) {
                        if (n_m < nb_cap) {
                            if (TS && nb_full) {
                                NbEnt e;
                                e.L = ld;
                                e.g = gk;
                                e.w = tw[hh];
                                e.p = p;
                                nbr.ent[m * NB_CAPM + n_m] = e;
                            } else {
                                NbEntC e;
                                e.g = gk;
                                e.sh = r.s[hh];
                                e.p = p;
                                nb_ent[n_m] = e;
                            }
                        }
                        n_m++;
                    }
                }
            }
        }
        if (NB && put_nb) {
            bins[bcur * BLOCK] = bacc;
            bins2[bcur * BLOCK] = xacc;
            for (int p = 0; p < P; p++) {
                const double2 a = bins[p * BLOCK], x = bins2[p * BLOCK];
                double* q = nbr.sums + (m * MAXP + p) * 4;
                q[0] = a.x; q[1] = a.y; q[2] = x.x; q[3] = x.y;
            }
            nbr.cnt[m] = n_m <= nb_cap ? n_m : NB_CAPM + 1;     // > NB_CAPM: overflow
        }
        if (DCR && put_dcr) {
            dcb[dq * BLOCK] = dacc;
            for (int q = 0; q < dc_nq; q++) {
                const double2 v = dcb[q * BLOCK];
                dr.mxl[m * DCP + q] = v.x;
                dr.lb[m * DCP + q] = v.y;
            }
            // the month's kept hours against its final lower bounds: an hour at
            // or below lb on both ends is at or below every lane's peak (~1.5 %
            // of the month's hours stay, of ~7 % kept while lb was rising)
            if (n_d <= dcr_cap) {
                int w = d_first;
                for (int k = d_first; k < n_d; k++) {
                    const NbEntC e = dr.ent[k];
                    const double L = (double)e.sh * ls;
                    const double a = L - e.g * dc_lo, b = L - e.g * dc_hi;
                    if (fmax(a, b) > dcb[e.p * BLOCK].y) {
                        if (w != k) dr.ent[w] = e;
                        w++;
                    }
                }
                n_d = w;
            }
            dr.off[m + 1] = n_d;
        }
        if (!mo2) bins[bcur * BLOCK] = bacc;
        if (!mo2) {
            // agent-major (load, system) pairs: k_batt_finance's lanes read the
            // agent's 12 P cells as one contiguous run
            double2* lg = W.LGb + (int64_t)i * NBIN + m * P;
            for (int p = 0; p < P; p++) lg[p] = bins[p * BLOCK];
        }
    }
    if (m_hi < 12) {
        W.carry[i] = soc;
        W.carry[n + i] = annual;
        if (DCR && (status & DGEN_ST_DEMAND)) O.status[i] = status;   // the next segment reloads it
        return;
    }
    // 1: the record holds every kept hour; 2: it overflowed and the plane was
    // not written (the repair pass writes it); 3: overflowed, plane written
    if (DCR && put_dcr) *dr.flag = n_d <= dcr_cap ? 1 : (skip_plane ? 2 : 3);
    // the record holds this scan's battery-case split (1: k_batt_finance skips
    // its build), or it overflowed without a plane (2: the repair pass writes
    // the plane, k_batt_finance builds from it), or neither (0)
    if (NB && mo2 && slot >= 0) {
        int fl = 0;
        if (put_nb) {
            for (int k = 0; k < 12; k++) nb_over = nb_over || nbr.cnt[k] > NB_CAPM;
            fl = !nb_over ? (nb_full ? 4 : 1) : (skip_plane ? 2 : 0);
        }
        nbr_flag(ws_nb(ws, n, n_scratch) + (size_t)slot * NB_BYTES) = fl;
    }
    O.annual_kwh[i] = annual;
    double den = kw_star > 1e-9 ? kw_star : 1e-9;
    double naep = annual / den;
    O.naep[i] = naep;
    O.capacity_factor[i] = naep / 8760.0;
    O.batt_kw[i] = has_batt ? power : 0.0;
    O.batt_kwh[i] = bank;
    if (!batt_on || unsized) O.npv_pv_batt[i] = NAN;   // k_batt_finance does not run
    // battery run on the PV run's tariff: k_batt_finance reuses its no-system
    // bill (same load, same tariff -> the same bill, as in the oracle)
    if (!repair) {   // the repair pass starts from the already switched tariff
        const bool same = tariff == O.tariff_final[i];
        W.aux[i] = same ? 0.0 : 1.0;
        O.tariff_final[i] = tariff;
        O.switched[i] = switched;
    }
    O.status[i] = status;
    W.otc_b[i] = otc;
}

// ===========================================================================
// Year-lane engine: one 64-lane wave per agent, lane = analysis year.
// Every per-agent quantity (tariff state, Brent state, cost, bins) is
// wave-uniform, so it lives in scalar registers / LDS; each lane owns one
// year's bill and cash-flow line; NPV is a deterministic wave sum and the
// payback year a wave prefix scan + ballot.
// ===========================================================================
constexpr int WAVE = 64;

// An agent's lanes: LPA = 64 (one agent per wave, analysis periods up to
// DGEN_MAXY years) or 32 (two agents per wave, periods up to 32 years -- the
// reference's 25-year life fills 25 of 32 lanes instead of 25 of 64).  Every
// per-agent quantity is uniform over its segment; reductions stay inside it.
template <int LPA>
struct Seg {
    int lane;   // 0..63
    int sl;     // lane within the segment (year - 1)
    int base;   // first lane of the segment
    __device__ explicit Seg(int l)
        : lane(l), sl(LPA == WAVE ? l : (l & (LPA - 1))), base(LPA == WAVE ? 0 : (l & ~(LPA - 1))) {}
    // fixed butterfly, then the segment's first lane's value (segment-uniform);
    // lanes past the analysis period hold 0, so the result does not depend on LPA
    __device__ __forceinline__ double sum(double v) const {
#pragma unroll
        for (int o = LPA / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
        return __shfl(v, base, WAVE);
    }
    __device__ __forceinline__ double incl_scan(double v) const {
#pragma unroll
        for (int o = 1; o < LPA; o <<= 1) {
            double t = __shfl_up(v, o, WAVE);
            if (sl >= o) v += t;
        }
        return v;
    }
    // first segment lane where pred holds, or -1
    __device__ __forceinline__ int first(bool pred) const {
        unsigned long long m = __ballot(pred);
        if (LPA < WAVE) m = (m >> base) & ((1ull << LPA) - 1ull);
        return m ? __ffsll((long long)m) - 1 : -1;
    }
    __device__ __forceinline__ double bcast(double v, int k) const { return __shfl(v, base + k, WAVE); }
};


// LDS hand-off between the lanes of one wave (every year-lane block is one
// wave): orders the LDS stores before the loads without s_barrier, so it is
// also correct where the two agents of a wave have diverged.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}


// Per-block LDS (one wave):
//   tariff [WAVE / LPA][dgen_tariff]                 (LPA < WAVE: staged copy, see stage_tariff)
//   bins  [WAVE / LPA][L[12 * half], G[12 * half]]  (segment-uniform, broadcast reads)
//   lane  [4 * half][WAVE]                          (per-lane per-period state)
//   peaks [12][WAVE]                                (dgen_tables.peak_units only:
//                                                   the lane's month peaks, kWh/kW tiers)
struct YLds {
    dgen_tariff* trf;   // the segment's staged tariff (LPA < WAVE only)
    double* L;
    double* G;
    double* lane;   // lane column base (already offset by lane)
    double* pk;     // the lane's month peak imports (stride WAVE), or nullptr
    int half;
    __device__ double& at(int k) const { return lane[k * WAVE]; }
};
constexpr int PK_SLOTS = 12;

static_assert(sizeof(dgen_tariff) % sizeof(double) == 0, "tariff staging copies qwords");
constexpr int TRF_QW = (int)(sizeof(dgen_tariff) / sizeof(double));

// LDS slots per lane (layout modes): YL_FULL 4 half (the net-billing bill
// stages entries and month sums after its 2 half accumulators); YL_NEM 2 half
// for the bins-only kernels (yl_bill_mo0's credits and billed kWh; the cash
// flow's two rows); YL_DC max(2 half, DCP) for the demand-charge kernels
// without net billing (the demand passes' per-period peaks).  The smaller
// layouts let k_batt_finance run one more wave per SIMD.
constexpr int YL_FULL = 0, YL_NEM = 1, YL_DC = 2;
__host__ __device__ inline int ylds_slots(int half, int mode) {
    return mode == YL_NEM ? 2 * half : mode == YL_DC ? (2 * half > DCP ? 2 * half : DCP) : 4 * half;
}
template <bool DC, bool NET>
constexpr int yl_mode() { return NET ? YL_FULL : (DC ? YL_DC : YL_NEM); }

__host__ __device__ inline size_t ylds_bytes(int half, int lpa, bool pk, int mode = YL_FULL) {
    const size_t trf = lpa < WAVE ? (size_t)(WAVE / lpa) * sizeof(dgen_tariff) : 0;
    return trf + sizeof(double) * ((size_t)24 * half * (WAVE / lpa) +
                                   (size_t)(ylds_slots(half, mode) + (pk ? PK_SLOTS : 0)) * WAVE);
}

template <int LPA>
__device__ __forceinline__ YLds ylds_make(double* base, int half, const Seg<LPA>& g, bool pk, int mode = YL_FULL) {
    YLds y;
    y.trf = nullptr;
    if (LPA < WAVE) {
        y.trf = reinterpret_cast<dgen_tariff*>(base) + g.lane / LPA;
        base += (WAVE / LPA) * TRF_QW;
    }
    y.L = base + (LPA == WAVE ? 0 : (g.lane / LPA) * 24 * half);
    y.G = y.L + 12 * half;
    y.lane = base + (WAVE / LPA) * 24 * half + g.lane;
    y.pk = pk ? y.lane + ylds_slots(half, mode) * WAVE : nullptr;
    y.half = half;
    return y;
}

// The tariff a year-lane agent bills with.  With one agent per wave the
// global record is wave-uniform and read through the scalar cache; with two
// agents per wave its address is per-lane, so every field read would be a
// vector load waited on in the middle of the month recursion -- the segment
// copies the record (1808 B) into its LDS slot once and reads it from there.
template <int LPA>
__device__ __forceinline__ const dgen_tariff* stage_tariff(const dgen_tariff* src, const YLds& S,
                                                          const Seg<LPA>& g) {
    if constexpr (LPA == WAVE) {
        return src;
    } else {
        wave_lds_sync();
        const double* s = reinterpret_cast<const double*>(src);
        double* d = reinterpret_cast<double*>(S.trf);
        // every load of the lane issued before the first store (one latency)
        constexpr int PER = (TRF_QW + LPA - 1) / LPA;
        double v[PER];
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const int k = g.sl + j * LPA;
            v[j] = k < TRF_QW ? s[k] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const int k = g.sl + j * LPA;
            if (k < TRF_QW) d[k] = v[j];
        }
        wave_lds_sync();
        return S.trf;
    }
}

// Tier-cap scale of month m by usage unit (oracle/orc.c month_energy_charge):
// 0 kWh: 1, 2 kWh daily: days, 1 kWh/kW: the month's peak import (kW), 3 kWh/kW
// daily: peak x days -- pk: the lane's month peaks (stride WAVE), written by
// the demand pass ahead of the bill (units 1 / 3 only).
__device__ __forceinline__ double tier_scale(const dgen_tariff& t, int m, const double* pk) {
    // the kernels without peak slots (pk a constant nullptr) keep units 0 / 2
    // only: a kWh/kW tariff never bills there (DGEN_ST_UNIT)
    if (!pk) return (t.unit == 2) ? (double)c_days_in_month[m] : 1.0;
    const double a = (t.unit & 1) ? pk[m * WAVE] : 1.0;
    const double b = (t.unit & 2) ? (double)c_days_in_month[m] : 1.0;
    return a * b;
}

// month energy charge from the lane's billed kWh u_p = at(uoff + p)
__device__ __forceinline__ double yl_month_charge(const dgen_tariff& t, int m, const YLds& S, int uoff) {
    const int P = t.P, T = t.T;
    double U = 0.0;
    for (int p = 0; p < P; p++) U += S.at(uoff + p);
    if (!(U > 0.0)) return 0.0;
    if (T == 1) {                       // one tier: sum_p u_p * buy_p (oracle order)
        double charge = 0.0;
        for (int p = 0; p < P; p++) charge += S.at(uoff + p) * t.buy[p][0];
        return charge;
    }
    double scale = tier_scale(t, m, S.pk);
    double charge = 0.0, prev = 0.0;
    for (int k = 0; k < T; k++) {
        double hi = (k == T - 1) ? INFINITY : t.cap[k] * scale;
        double top = U < hi ? U : hi;
        double amt = top - prev;
        if (amt < 0.0) amt = 0.0;
        if (hi > prev) prev = hi;
        for (int p = 0; p < P; p++) charge += (S.at(uoff + p) / U) * amt * t.buy[p][k];
    }
    return charge;
}

// A net-billing month's bill: fixed + energy charge - export credit; option 3
// floors the energy part at 0 and carries the excess credit to the next month
// (lost at year end).  oracle/orc.c year_bill, same order.
__device__ __forceinline__ double nb_month(const dgen_tariff& t, double charge, double cr, double& carry) {
    if (t.mo == 3) {
        const double e = charge - cr - carry;
        carry = e < 0.0 ? -e : 0.0;
        return t.fixed + (e < 0.0 ? 0.0 : e);
    }
    return t.fixed + charge - cr;
}

// Bill of metering options 1 (NEM with $ credits: per-period monthly net,
// imports billed, surplus kWh credited at the period's tier-1 sell rate, the
// energy part floored at 0 with the excess carried) and 4 (buy all / sell
// all: the whole load billed, all generation credited at the tier-1 sell
// rate) from the lane's bins; oracle/orc.c year_bill, same order.  Parity
// unpinned (SSC restatement).
__device__ double yl_bill_bins_ext(const dgen_tariff& t, const YLds& S, double gscale) {
    const int P = t.P, half = S.half;
    double total = 0.0, carry = 0.0;
    for (int m = 0; m < 12; m++) {
        double cr = 0.0;
        for (int p = 0; p < P; p++) {
            const double L = S.L[m * half + p], G = S.G[m * half + p];
            if (t.mo == 1) {
                const double nn = L - gscale * G;
                S.at(p) = nn > 0.0 ? nn : 0.0;
                cr += (nn < 0.0 ? -nn : 0.0) * t.sell[p][0];
            } else {
                S.at(p) = L;
                cr += (gscale * G) * t.sell[p][0];
            }
        }
        const double charge = yl_month_charge(t, m, S, 0);
        if (t.mo == 1) {
            const double e = charge - cr - carry;
            carry = e < 0.0 ? -e : 0.0;
            total += t.fixed + (e < 0.0 ? 0.0 : e);
        } else {
            total += t.fixed + (charge - cr);
        }
    }
    return total;
}

// NEM (mo 0) bill of the lane's year: net = L - gscale * G per (month, period)
// from the LDS bins; per-period kWh credits; December true-up.
__device__ __forceinline__ double yl_bill_mo0(const dgen_tariff& t, const YLds& S, double gscale,
                                              double yearend) {
    const int P = t.P, half = S.half;
    const int cr = 0, uo = half;
    for (int p = 0; p < P; p++) S.at(cr + p) = 0.0;
    double total = 0.0;
    for (int m = 0; m < 12; m++) {
        for (int p = 0; p < P; p++) {
            double nn = S.L[m * half + p] - gscale * S.G[m * half + p];
            double credit = S.at(cr + p);
            double u = 0.0;
            if (nn >= 0.0) {
                double use = nn < credit ? nn : credit;
                u = nn - use;
                credit -= use;
            } else {
                credit += -nn;
            }
            S.at(cr + p) = credit;
            S.at(uo + p) = u;
        }
        double bill = t.fixed + yl_month_charge(t, m, S, uo);
        if (m == 11) {
            double cc = 0.0;
            for (int p = 0; p < P; p++) cc += S.at(cr + p);
            bill -= cc * yearend;
        }
        total += bill;
    }
    return total;
}

// Same bill with the per-period credits and billed kWh in registers (P <= 4,
// the common case): loops run to the compile-time bound under the uniform
// guard p < P, so the order of every sum is the LDS version's.
__device__ __forceinline__ double yl_bill_mo0_reg(const dgen_tariff& t, const YLds& S, double gscale,
                                                  double yearend) {
    const int P = t.P, T = t.T, half = S.half;
    const double fixed = t.fixed;
    // first-tier prices in registers (every month reads them)
    double b0[PREG];
#pragma unroll
    for (int p = 0; p < PREG; p++) b0[p] = p < P ? t.buy[p][0] : 0.0;
    double credit[PREG], u[PREG];
#pragma unroll
    for (int p = 0; p < PREG; p++) { credit[p] = 0.0; u[p] = 0.0; }
    double total = 0.0;
    for (int m = 0; m < 12; m++) {
#pragma unroll
        for (int p = 0; p < PREG; p++) {
            if (p < P) {
                double nn = S.L[m * half + p] - gscale * S.G[m * half + p];
                double use = nn < credit[p] ? nn : credit[p];
                double un = nn - use;
                double cn = credit[p] - use;
                const bool pos = nn >= 0.0;
                u[p] = pos ? un : 0.0;
                credit[p] = pos ? cn : credit[p] + -nn;
            }
        }
        double U = 0.0;
#pragma unroll
        for (int p = 0; p < PREG; p++)
            if (p < P) U += u[p];
        double charge = 0.0;
        if (U > 0.0) {
            if (T == 1) {
                // one tier: every period's kWh at its own price (the oracle's
                // month_energy_charge; no share / re-multiplication)
#pragma unroll
                for (int p = 0; p < PREG; p++)
                    if (p < P) charge += u[p] * b0[p];
            } else {
                // each period's share of the month, once per month (the same
                // quotient the tier loop used to recompute per tier)
                double fr[PREG];
#pragma unroll
                for (int p = 0; p < PREG; p++) fr[p] = p < P ? u[p] / U : 0.0;
                const double scale = tier_scale(t, m, S.pk);
                double prev = 0.0;
                for (int k = 0; k < T; k++) {
                    double hi = (k == T - 1) ? INFINITY : t.cap[k] * scale;
                    double top = U < hi ? U : hi;
                    double amt = top - prev;
                    if (amt < 0.0) amt = 0.0;
                    if (hi > prev) prev = hi;
#pragma unroll
                    for (int p = 0; p < PREG; p++)
                        if (p < P) charge += fr[p] * amt * (k == 0 ? b0[p] : t.buy[p][k]);
                }
            }
        }
        double bill = fixed + charge;
        if (m == 11) {
            double cc = 0.0;
#pragma unroll
            for (int p = 0; p < PREG; p++)
                if (p < P) cc += credit[p];
            bill -= cc * yearend;
        }
        total += bill;
    }
    return total;
}

__device__ __forceinline__ double yl_bill_nem(const dgen_tariff& t, const YLds& S, double gscale,
                                              double yearend) {
    if (t.mo != 0) return yl_bill_bins_ext(t, S, gscale);                 // options 1 and 4
    return (t.P <= PREG) ? yl_bill_mo0_reg(t, S, gscale, yearend) : yl_bill_mo0(t, S, gscale, yearend);
}

// The no-system NEM bill (gscale 0): every month nets its load (>= 0), so no
// kWh credit ever accrues and the months are independent -- lane m < 12 of
// the segment bills month m with yl_bill_mo0_reg's arithmetic (credit 0),
// then the months are added in order, the serial loop's sum.  A negative
// bin (months then depend on each other) or P > PREG takes the serial bill.
template <int LPA>
__device__ __forceinline__ double yl_bill_nem_nosys(const dgen_tariff& t, const YLds& S, double yearend,
                                                    const Seg<LPA>& g) {
    if (t.mo != 0 || t.P > PREG) return yl_bill_nem(t, S, 0.0, yearend);
    const int P = t.P, T = t.T, half = S.half;
    const int m = g.sl < 12 ? g.sl : 11;
    double b0[PREG], u[PREG], credit[PREG];
    bool neg = false;
#pragma unroll
    for (int p = 0; p < PREG; p++) {
        b0[p] = p < P ? t.buy[p][0] : 0.0;
        u[p] = 0.0;
        credit[p] = 0.0;
        if (p < P) {
            const double nn = S.L[m * half + p] - 0.0 * S.G[m * half + p];
            const double use = nn < 0.0 ? nn : 0.0;
            const double un = nn - use;
            const double cn = 0.0 - use;
            const bool pos = nn >= 0.0;
            u[p] = pos ? un : 0.0;
            credit[p] = pos ? cn : 0.0 + -nn;
            neg = neg || !pos;
        }
    }
    if (g.first(neg) >= 0) return yl_bill_nem(t, S, 0.0, yearend);
    double U = 0.0;
#pragma unroll
    for (int p = 0; p < PREG; p++)
        if (p < P) U += u[p];
    double charge = 0.0;
    if (U > 0.0) {
        if (T == 1) {
#pragma unroll
            for (int p = 0; p < PREG; p++)
                if (p < P) charge += u[p] * b0[p];
        } else {
            double fr[PREG];
#pragma unroll
            for (int p = 0; p < PREG; p++) fr[p] = p < P ? u[p] / U : 0.0;
            const double scale = tier_scale(t, m, S.pk);
            double prev = 0.0;
            for (int k = 0; k < T; k++) {
                double hi = (k == T - 1) ? INFINITY : t.cap[k] * scale;
                double top = U < hi ? U : hi;
                double amt = top - prev;
                if (amt < 0.0) amt = 0.0;
                if (hi > prev) prev = hi;
#pragma unroll
                for (int p = 0; p < PREG; p++)
                    if (p < P) charge += fr[p] * amt * (k == 0 ? b0[p] : t.buy[p][k]);
            }
        }
    }
    double bill = t.fixed + charge;
    if (m == 11) {
        double cc = 0.0;
#pragma unroll
        for (int p = 0; p < PREG; p++)
            if (p < P) cc += credit[p];
        bill -= cc * yearend;
    }
    double total = 0.0;
    for (int mm = 0; mm < 12; mm++) total += __shfl(bill, g.base + mm, WAVE);
    return total;
}

// Wave-uniform hourly source for net billing.
struct YSrc {
    const float* shape;
    const int32_t* cf;        // PV-only (or nullptr)
    const double* sysgen;     // battery scratch [h * stride] (or nullptr)
    int64_t sys_stride;
    double load_scale, gen_scale;
    const double* ts;
    double ts_mult;
};

// The battery case's system-output plane in day tiles [365][n_scratch][24] f64
// (src.sysgen = scratch + 24 x slot, stride n_scratch): an agent's day is 192
// contiguous bytes, so the finance kernel's hour lanes read a day as 1.5 cache
// lines (the hour-quad tiles [2190][n_scratch][4] cost them a line per 4 hours,
// each shared with 3 other agents: ~3.4x the plane in L2 fills on the national
// TS sell-rate agents), while a scan wave's 6 quad stores of a day still cover
// one contiguous 12 KB run.
__device__ __forceinline__ int64_t sys_index(const YSrc& src, int h) {
    const int d = h / 24;
    return (int64_t)d * src.sys_stride * 24 + (h - d * 24);
}
__device__ __forceinline__ double sys_at(const YSrc& src, int h) { return src.sysgen[sys_index(src, h)]; }

// The 4 system-output values of hours h .. h + 3 (h % 4 == 0; a quad never
// straddles a day)
__device__ __forceinline__ void sys_quad(const YSrc& src, int h, double* g) {
    const double2* q = reinterpret_cast<const double2*>(src.sysgen + sys_index(src, h));
    const double2 a = q[0], b = q[1];
    g[0] = a.x; g[1] = a.y; g[2] = b.x; g[3] = b.y;
}

// Month energy charge from register-held billed kWh (P <= PREG), the same
// arithmetic and order as yl_month_charge.
__device__ __forceinline__ double reg_month_charge(const dgen_tariff& t, int m, const double (&u)[PREG],
                                                   const double* pk) {
    const int P = t.P, T = t.T;
    double U = 0.0;
#pragma unroll
    for (int p = 0; p < PREG; p++)
        if (p < P) U += u[p];
    if (!(U > 0.0)) return 0.0;
    double charge = 0.0;
    if (T == 1) {
#pragma unroll
        for (int p = 0; p < PREG; p++)
            if (p < P) charge += u[p] * t.buy[p][0];
        return charge;
    }
    double fr[PREG];
#pragma unroll
    for (int p = 0; p < PREG; p++) fr[p] = p < P ? u[p] / U : 0.0;
    const double scale = tier_scale(t, m, pk);
    double prev = 0.0;
    for (int k = 0; k < T; k++) {
        double hi = (k == T - 1) ? INFINITY : t.cap[k] * scale;
        double top = U < hi ? U : hi;
        double amt = top - prev;
        if (amt < 0.0) amt = 0.0;
        if (hi > prev) prev = hi;
#pragma unroll
        for (int p = 0; p < PREG; p++)
            if (p < P) charge += fr[p] * amt * t.buy[p][k];
    }
    return charge;
}

// Net-billing (mo 2) bill with the per-period import / export sums in
// registers (P <= PREG).  The hour loop of yl_bill_mo2 waited on two loads
// and an LDS read-modify-write per hour; here each 8-hour chunk's profile
// (and system output / sell-rate) values are loaded together before use, and
// each hour adds dd (or the export credit) into its period's register, the
// others adding an exact +0.0 -- the same sums in the same hour order.
constexpr int MO2_CH = 8;
__device__ __forceinline__ double yl_bill_mo2_reg(const dgen_tariff& t, const YSrc& src, double s,
                                                  bool with_gen, const double* pk) {
    const int P = t.P;
    double total = 0.0, carry = 0.0;
    int h = 0;
    for (int m = 0; m < 12; m++) {
        double imp[PREG], exv[PREG];
#pragma unroll
        for (int p = 0; p < PREG; p++) { imp[p] = 0.0; exv[p] = 0.0; }
        for (int d = c_month_start_day[m]; d < c_month_start_day[m + 1]; d++, h += 24) {
            const uint32_t* sr = reinterpret_cast<const uint32_t*>(((d % 7) >= 5) ? t.wkend[m] : t.wkday[m]);
#pragma unroll 1
            for (int c0 = 0; c0 < 24; c0 += MO2_CH) {
                uint32_t pq[MO2_CH / 4];
#pragma unroll
                for (int j = 0; j < MO2_CH / 4; j++) pq[j] = sr[c0 / 4 + j];
                float sh[MO2_CH];
                double g[MO2_CH], tsv[MO2_CH];
#pragma unroll
                for (int k = 0; k < MO2_CH; k += 4) {
                    const float4 a = *reinterpret_cast<const float4*>(src.shape + h + c0 + k);
                    sh[k] = a.x; sh[k + 1] = a.y; sh[k + 2] = a.z; sh[k + 3] = a.w;
                }
#pragma unroll
                for (int k = 0; k < MO2_CH; k++) g[k] = 0.0;
                if (with_gen) {
                    if (src.sysgen) {
#pragma unroll
                        for (int k = 0; k < MO2_CH; k += 4) sys_quad(src, h + c0 + k, g + k);
                    } else {
#pragma unroll
                        for (int k = 0; k < MO2_CH; k += 4) {
                            const int4 a = *reinterpret_cast<const int4*>(src.cf + h + c0 + k);
                            g[k] = cf_per_kw(a.x) * src.gen_scale;
                            g[k + 1] = cf_per_kw(a.y) * src.gen_scale;
                            g[k + 2] = cf_per_kw(a.z) * src.gen_scale;
                            g[k + 3] = cf_per_kw(a.w) * src.gen_scale;
                        }
                    }
                }
                if (src.ts) {
#pragma unroll
                    for (int k = 0; k < MO2_CH; k++) tsv[k] = src.ts[h + c0 + k];
                }
#pragma unroll
                for (int k = 0; k < MO2_CH; k++) {
                    const double load = (double)sh[k] * src.load_scale;
                    const double dd = load - g[k] * s;
                    const int p = (int)((pq[k >> 2] >> (8 * (k & 3))) & 0xffu);
                    const bool pos = dd > 0.0;
                    double e = -dd;
                    if (src.ts) e *= (double)(float)(tsv[k] * src.ts_mult);
#pragma unroll
                    for (int q = 0; q < PREG; q++) {
                        imp[q] += (pos && p == q) ? dd : 0.0;
                        exv[q] += (!pos && p == q) ? e : 0.0;
                    }
                }
            }
        }
        double cr = 0.0;
#pragma unroll
        for (int p = 0; p < PREG; p++)
            if (p < P) cr += src.ts ? exv[p] : exv[p] * t.sell[p][0];
        total += nb_month(t, reg_month_charge(t, m, imp, pk), cr, carry);
    }
    return total;
}

// Net-billing (mo 2) bill of the lane's year (system output x s).
__device__ __forceinline__ double yl_bill_mo2(const dgen_tariff& t, const YSrc& src, double s,
                                              bool with_gen, const YLds& S) {
    const int P = t.P, half = S.half;
    double total = 0.0, carry = 0.0;
    int h = 0;
    for (int m = 0; m < 12; m++) {
        for (int p = 0; p < P; p++) { S.at(p) = 0.0; S.at(half + p) = 0.0; }
        // the running import / export sums of the current period live in
        // registers (cur, ci, ce) and go through LDS only when the period
        // changes: the same additions in the same hour order, without an LDS
        // read-modify-write round trip per hour
        int cur = 0;
        double ci = 0.0, ce = 0.0;
        for (int d = c_month_start_day[m]; d < c_month_start_day[m + 1]; d++) {
            const uint8_t* sched = ((d % 7) >= 5) ? t.wkend[m] : t.wkday[m];
#pragma unroll 1
            for (int c0 = 0; c0 < 24; c0 += 4, h += 4) {
                // the 4 hours' inputs loaded together (one latency, not four)
                const float4 sv = *reinterpret_cast<const float4*>(src.shape + h);
                const uint32_t pq = *reinterpret_cast<const uint32_t*>(sched + c0);
                const float shv[4] = {sv.x, sv.y, sv.z, sv.w};
                double g[4] = {0.0, 0.0, 0.0, 0.0}, tsv[4] = {0.0, 0.0, 0.0, 0.0};
                int4 cv = make_int4(0, 0, 0, 0);
                if (with_gen && !src.sysgen) cv = *reinterpret_cast<const int4*>(src.cf + h);
                if ((!with_gen || !src.sysgen) && (cv.x | cv.y | cv.z | cv.w) == 0) {
                    // no PV in these 4 hours (night, or the no-system bill): the
                    // import is the load itself (load - 0 * s == load) and a zero
                    // load adds a signed zero to the export sum -- the general
                    // path's result, without its generation / sell-rate work
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const double load = (double)shv[k] * src.load_scale;
                        const int p = (int)((pq >> (8 * k)) & 0xffu);
                        if (p != cur) {
                            S.at(cur) = ci;
                            S.at(half + cur) = ce;
                            cur = p;
                            ci = S.at(p);
                            ce = S.at(half + p);
                        }
                        if (load > 0.0) ci += load;
                    }
                    continue;
                }
                if (with_gen) {
                    if (src.sysgen) {
                        sys_quad(src, h, g);
                    } else {
                        g[0] = cf_per_kw(cv.x) * src.gen_scale;
                        g[1] = cf_per_kw(cv.y) * src.gen_scale;
                        g[2] = cf_per_kw(cv.z) * src.gen_scale;
                        g[3] = cf_per_kw(cv.w) * src.gen_scale;
                    }
                }
                if (src.ts) {
#pragma unroll
                    for (int k = 0; k < 4; k++) tsv[k] = src.ts[h + k];
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    double load = (double)shv[k] * src.load_scale;
                    double dd = load - g[k] * s;
                    int p = (int)((pq >> (8 * k)) & 0xffu);
                    if (p != cur) {
                        S.at(cur) = ci;
                        S.at(half + cur) = ce;
                        cur = p;
                        ci = S.at(p);
                        ce = S.at(half + p);
                    }
                    if (dd > 0.0) {
                        ci += dd;
                    } else {
                        double e = -dd;
                        if (src.ts) e *= (double)(float)(tsv[k] * src.ts_mult);
                        ce += e;
                    }
                }
            }
        }
        S.at(cur) = ci;
        S.at(half + cur) = ce;
        double cr = 0.0;
        for (int p = 0; p < P; p++) {
            double e = S.at(half + p);
            cr += src.ts ? e : e * t.sell[p][0];
        }
        total += nb_month(t, yl_month_charge(t, m, S, 0), cr, carry);
    }
    return total;
}

// k_batt_finance's net-billing bills (k_size keeps the LDS version: the register
// version's chunk buffers push its 168-VGPR budget into spills, measured slower)
__device__ __forceinline__ double yl_bill_net(const dgen_tariff& t, const YSrc& src, double s,
                                              bool with_gen, const YLds& S) {
    return (t.P <= PREG) ? yl_bill_mo2_reg(t, src, s, with_gen, S.pk) : yl_bill_mo2(t, src, s, with_gen, S);
}

// ---------------------------------------------------------------------------
// Demand charges (extension mode; the reference keeps them off, ff:35):
// monthly flat + TOU peaks of hourly grid import, tiered (oracle/orc.c
// year_demand, same order: flat tiers, then periods 0..DCP-1).
// ---------------------------------------------------------------------------
__device__ __forceinline__ double dc_tier_charge(double peak, const double* cap, const double* price,
                                                 int nt) {
    double charge = 0.0, prev = 0.0;
    for (int k = 0; k < nt; k++) {
        double hi = (k == nt - 1) ? INFINITY : cap[k];
        double top = peak < hi ? peak : hi;
        double amt = top - prev;
        if (amt < 0.0) amt = 0.0;
        if (hi > prev) prev = hi;
        charge += amt * price[k];
    }
    return charge;
}

// The reference's per-hour PV output at kW (ff:117-119, dc -> ac -> kWh), in
// its own operation order: demand charges bill maxima, where a last-bit
// difference can move a Brent comparison at a kink, so the demand passes form
// each hour's generation exactly as the reference (and the oracle) does.
__device__ __forceinline__ double ref_gen(double gpk, double kw) {
    return (((gpk * kw) * 1000.0) * 0.96) / 1000.0;
}

// One lane's year of demand charges (system output x s; no system when
// !with_gen).  Peaks are maxima, so they are exact whatever the hour order;
// only the imports' own rounding differs from the oracle.  The TOU peaks live
// in the lane's LDS column (S.at(0 .. DCP-1); the host sizes it, see
// dgen_size_agents): held in registers they pushed k_size into spills.
// kw: the search's system kW (PV-only case; the battery case reads the
// system-output plane, src.sysgen)
__device__ __forceinline__ double yl_demand(const dgen_demand* D, const YSrc& src, double kw, double s,
                                           bool with_gen, const YLds& S) {
    double total = 0.0;
    int h = 0;
    for (int m = 0; m < 12; m++) {
        double flat = 0.0;
        for (int q = 0; q < DCP; q++) S.at(q) = 0.0;
        // half a day per step: the 12 hours of every input are loaded
        // together (one memory latency per 12 hours, not one per 4)
        for (int d = c_month_start_day[m]; d < c_month_start_day[m + 1]; d++) {
            const uint32_t* sq = reinterpret_cast<const uint32_t*>(((d % 7) >= 5) ? D->wkend[m] : D->wkday[m]);
#pragma unroll 1
            for (int half12 = 0; half12 < 2; half12++, h += 12) {
                uint32_t pq[3];
                float sh[12];
                double g[12];
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    pq[k] = sq[3 * half12 + k];
                    const float4 a = *reinterpret_cast<const float4*>(src.shape + h + 4 * k);
                    sh[4 * k] = a.x; sh[4 * k + 1] = a.y; sh[4 * k + 2] = a.z; sh[4 * k + 3] = a.w;
                }
                if (with_gen && src.sysgen) {
#pragma unroll
                    for (int k = 0; k < 12; k += 4) sys_quad(src, h + k, g + k);
                } else if (with_gen) {
#pragma unroll
                    for (int k = 0; k < 3; k++) {
                        const int4 cv = *reinterpret_cast<const int4*>(src.cf + h + 4 * k);
                        g[4 * k] = ref_gen(cf_per_kw(cv.x), kw);
                        g[4 * k + 1] = ref_gen(cf_per_kw(cv.y), kw);
                        g[4 * k + 2] = ref_gen(cf_per_kw(cv.z), kw);
                        g[4 * k + 3] = ref_gen(cf_per_kw(cv.w), kw);
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < 12; k++) g[k] = 0.0;
                }
#pragma unroll
                for (int k = 0; k < 12; k++) {
                    const double imp = (double)sh[k] * src.load_scale - g[k] * s;
                    const int p = (int)((pq[k >> 2] >> (8 * (k & 3))) & 0xffu);
                    flat = imp > flat ? imp : flat;
                    double& pk = S.at(p < DCP ? p : 0);
                    pk = imp > pk ? imp : pk;
                }
            }
        }
        if (S.pk) S.pk[m * WAVE] = flat;          // the month's peak import (kWh/kW tiers)
        double c = dc_tier_charge(flat, D->flat_cap[m], D->flat_price[m], D->flat_nt[m]);
        for (int q = 0; q < DCP; q++) c += dc_tier_charge(S.at(q), D->tou_cap[q], D->tou_price[q], D->tou_nt[q]);
        total += c;
    }
    return total;
}

// Battery-case demand charges with the hours staged through LDS: every year
// lane of a segment bills the same hours (only its degradation factor s
// differs), so the segment loads each batch of DEM_BATCH hours once --
// lane k takes DEM_BATCH / LPA of them (load L = shape x load_scale, system
// output, demand period) -- and stores them grouped by demand period
// (a counting sort by ballots), with the group offsets.  Every lane then
// scans each period's run from LDS (broadcast reads) with a plain running max:
// no per-hour branch or LDS write in the scan.  The same imports as yl_demand
// (L - sys x s) and the same maxima (a max does not depend on the order).
constexpr int DEM_BATCH = 64;
struct DemStage {
    double2 lg[DEM_BATCH];       // (L, system output) of the batch's hours, grouped by period
    int off[DCP + 1];            // period q's hours: [off[q], off[q + 1])
    int pad[(16 - (DCP + 1) % 16) % 16];
};
constexpr size_t DEM_STAGE_BYTES = sizeof(DemStage);
static_assert(DEM_STAGE_BYTES % 16 == 0, "stage keeps 16-B alignment");

// R: the same pass over the agent's battery-case demand record (DcrRec, built
// by k_hourly_batt) instead of the system-output plane: each month's lanes
// start from the record's lower bounds lb and stage only its kept hours
// (entries off[m] .. off[m + 1], segment-specific trip counts: the ballots and
// the stage are per segment), with the filter below.  The no-system pass
// (with_gen false) is the record's max loads, no hours at all.
template <int LPA>
__device__ __forceinline__ double yl_demand_staged(const dgen_demand* D, const YSrc& src, double s, bool with_gen,
                                   const YLds& S, DemStage* st, const Seg<LPA>& g,
                                   bool REC = false, const DcrRec& R = DcrRec{}, int nq = DCP) {
    constexpr int HPL = DEM_BATCH / LPA;              // hours each lane stages (1 or 2)
    const uint64_t segmask = LPA == WAVE ? ~0ull : (((1ull << LPA) - 1ull) << g.base);
    const uint64_t below = ((1ull << g.lane) - 1ull) & segmask;   // segment lanes before this one
    const int k0 = g.sl * HPL;
    // Filter: an hour whose import cannot exceed the lowest running peak of
    // its period among the segment's lanes changes no lane's peak, so it is
    // not staged.  Its largest import over the lanes' factors is at the
    // smallest or largest s of the segment (a line in s).
    double s_mn = s, s_mx = s;
#pragma unroll
    for (int o = LPA / 2; o > 0; o >>= 1) {
        const double a = __shfl_xor(s_mn, o, WAVE), b = __shfl_xor(s_mx, o, WAVE);
        s_mn = a < s_mn ? a : s_mn;
        s_mx = b > s_mx ? b : s_mx;
    }
    double total = 0.0;
    for (int m = 0; m < 12; m++) {
        double flat = 0.0;
        for (int q = 0; q < DCP; q++) S.at(q) = 0.0;
        if (REC) {
            const double* from = with_gen ? R.lb + m * DCP : R.mxl + m * DCP;
            for (int q = 0; q < nq; q++) {
                const double v = from[q];
                S.at(q) = v;
                flat = v > flat ? v : flat;
            }
            if (!with_gen) {                      // the no-system peaks: exact from the record
                if (S.pk) S.pk[m * WAVE] = flat;
                double c = dc_tier_charge(flat, D->flat_cap[m], D->flat_price[m], D->flat_nt[m]);
                for (int q = 0; q < nq; q++) c += dc_tier_charge(S.at(q), D->tou_cap[q], D->tou_price[q], D->tou_nt[q]);
                total += c;
                continue;
            }
        }
        const int h_lo = REC ? R.off[m] : c_month_start_day[m] * 24;
        const int h_hi = REC ? R.off[m + 1] : c_month_start_day[m + 1] * 24;
        // the batch's hours (load, system output, period), the next batch's
        // loads issued before the current batch is processed
        auto fetch = [&](int hb, double (&Lq)[HPL], double (&gq)[HPL], int (&pq)[HPL])
            __attribute__((always_inline)) {
            const int nb = (h_hi - hb) < DEM_BATCH ? (h_hi - hb) : DEM_BATCH;
#pragma unroll
            for (int u = 0; u < HPL; u++) {
                const bool valid = hb < h_hi && k0 + u < nb;
                if (REC) {                        // a kept hour: its entry
                    const NbEntC e = R.ent[valid ? hb + k0 + u : 0];
                    pq[u] = valid ? e.p : -1;
                    Lq[u] = (double)e.sh * src.load_scale;
                    gq[u] = e.g;
                } else {
                    const int hu = valid ? hb + k0 + u : h_lo;
                    const int d = hu / 24, hod = hu - d * 24;
                    const int pp = ((d % 7) >= 5) ? D->wkend[m][hod] : D->wkday[m][hod];
                    pq[u] = valid ? (pp < DCP ? pp : 0) : -1;
                    Lq[u] = (double)src.shape[hu] * src.load_scale;
                    gq[u] = with_gen ? src.sysgen[(int64_t)d * src.sys_stride * 24 + hod] : 0.0;
                }
            }
        };
        double nL[HPL], ng[HPL];
        int np[HPL];
        fetch(h_lo, nL, ng, np);
#pragma unroll 1
        for (int hb = h_lo; hb < h_hi; hb += DEM_BATCH) {
            double Lv[HPL], gv[HPL];
            int pv[HPL];
#pragma unroll
            for (int u = 0; u < HPL; u++) {
                Lv[u] = nL[u];
                gv[u] = ng[u];
                pv[u] = np[u];
            }
            fetch(hb + DEM_BATCH, nL, ng, np);
            // the segment's lowest running peak per period; drop hours below it
            double thr[DCP];
#pragma unroll
            for (int q = 0; q < DCP; q++) {
                double v = S.at(q);
                if (!REC) {
#pragma unroll
                    for (int o = LPA / 2; o > 0; o >>= 1) {
                        const double w = __shfl_xor(v, o, WAVE);
                        v = w < v ? w : v;
                    }
                }
                thr[q] = v;
            }
#pragma unroll
            for (int u = 0; u < HPL; u++) {
                if (pv[u] >= 0 && !REC) {        // a record's kept hours passed this against lb
                    double t_u = thr[0];
#pragma unroll
                    for (int q = 1; q < DCP; q++) t_u = pv[u] == q ? thr[q] : t_u;
                    const double a = Lv[u] - gv[u] * s_mn, b = Lv[u] - gv[u] * s_mx;
                    if (!((a > b ? a : b) > t_u)) pv[u] = -1;
                }
            }
            wave_lds_sync();                          // previous batch fully read
            int base_q = 0;
#pragma unroll 1
            for (int q = 0; q < nq; q++) {
                uint64_t b[HPL];
                int cnt = 0;
#pragma unroll
                for (int u = 0; u < HPL; u++) {
                    b[u] = __ballot(pv[u] == q) & segmask;
                    cnt += __popcll(b[u]);
                }
                int pos = base_q;
#pragma unroll
                for (int u = 0; u < HPL; u++) pos += __popcll(b[u] & below);
#pragma unroll
                for (int u = 0; u < HPL; u++) {
                    if (pv[u] == q) st->lg[pos++] = make_double2(Lv[u], gv[u]);
                }
                if (g.sl == 0) st->off[q] = base_q;
                base_q += cnt;
            }
            if (g.sl == 0) st->off[nq] = base_q;
            wave_lds_sync();
            for (int q = 0; q < nq; q++) {
                const int lo = st->off[q], hi = st->off[q + 1];
                if (lo == hi) continue;
                double mx = -INFINITY;
#pragma unroll 4
                for (int k = lo; k < hi; k++) {
                    const double2 v = st->lg[k];           // one ds_read_b128 per hour
                    const double imp = v.x - v.y * s;
                    mx = imp > mx ? imp : mx;
                }
                flat = mx > flat ? mx : flat;
                double& pk = S.at(q);
                pk = mx > pk ? mx : pk;
            }
        }
        if (S.pk) S.pk[m * WAVE] = flat;          // the month's peak import (kWh/kW tiers)
        double c = dc_tier_charge(flat, D->flat_cap[m], D->flat_price[m], D->flat_nt[m]);
        for (int q = 0; q < nq; q++) c += dc_tier_charge(S.at(q), D->tou_cap[q], D->tou_price[q], D->tou_nt[q]);
        total += c;
    }
    return total;
}

// ---------------------------------------------------------------------------
// Demand-charge envelopes (PV-only search).  Within one (month, demand
// period) group the import of hour h at generation scale t is the line
// L_h - g_h t, and the group's peak is max(0, max_h line).  The search only
// evaluates t in [t_lo, t_hi] (the Brent bracket's kW x the analysis years'
// degradation factors), where a line can reach the max only if it beats
// M(t) = max(A(t), B(t)) -- A, B the maxima at t_lo and t_hi -- at the point
// t* where A and B cross (M is their convex hull: a line below M at t_lo, t*
// and t_hi is below it on the whole interval).  So each group keeps A, B and
// the lines above M(t*) (a relative slack of 1e-10 keeps the set a superset
// under rounding); an evaluation then takes the max over <= DC_NL lines per
// group instead of re-scanning 8760 hours, with the hourly pass's arithmetic
// per line (L = shape x load_scale, g = cf / 1e6, import = L - ref_gen(g, kW) x s),
// so the peaks are the hourly pass's peaks.  A group that needs more lines
// sends the agent back to the hourly pass (yl_demand).
// ---------------------------------------------------------------------------
constexpr int DC_NL = 8;
struct DcEnv {
    double2* lines;   // [12][DCP][DC_NL] (L, g)
    double* maxl;     // [12][DCP] max load (the no-system peak)
    int* cnt;         // [12][DCP] lines kept (0 = period absent from the month)
    int* tag;         // k_dc_env: 1 + the tariff built for, -(1 + it) when a group overflowed, 0 none
};
constexpr size_t DCW_BYTES = (size_t)12 * DCP * (DC_NL * sizeof(double2) + sizeof(double) + sizeof(int)) + 16;

__device__ __forceinline__ DcEnv dc_env_at(void* base, int64_t i) {
    char* b = reinterpret_cast<char*>(base) + (size_t)i * DCW_BYTES;
    DcEnv e;
    e.lines = reinterpret_cast<double2*>(b);
    e.maxl = reinterpret_cast<double*>(b + (size_t)12 * DCP * DC_NL * sizeof(double2));
    e.cnt = reinterpret_cast<int*>(b + (size_t)12 * DCP * (DC_NL * sizeof(double2) + sizeof(double)));
    e.tag = reinterpret_cast<int*>(b + (size_t)12 * DCP * (DC_NL * sizeof(double2) + sizeof(double) + sizeof(int)));
    return e;
}

// Build the agent's envelopes: segment lane m < 12 takes month m (two passes
// over the month per demand period present).  Returns true when every group
// fit in DC_NL lines (segment-uniform).
template <int LPA>
__device__ __forceinline__ bool yl_dc_build(const dgen_demand* D, const YSrc& src, double tlo, double thi,
                            const DcEnv& E, const Seg<LPA>& g) {
    bool ok = true;
    const int m = g.sl;
    if (m < 12) {
        uint32_t mask = 0;
        for (int h = 0; h < 24; h++) mask |= (1u << D->wkday[m][h]) | (1u << D->wkend[m][h]);
        const int d0 = c_month_start_day[m], d1 = c_month_start_day[m + 1];
        for (int p = 0; p < DCP; p++) {
            int n_l = 0;
            double mL = 0.0;
            if ((mask >> p) & 1u) {
                double aL = 0.0, ag = 0.0, av = -INFINITY, bL = 0.0, bg = 0.0, bv = -INFINITY;
                int ah = -1, bh = -1;
                for (int pass = 0; pass < 2; pass++) {
                    double ts = tlo, Ms = 0.0, slack = 0.0;
                    if (pass == 1) {
                        if (ag > bg) {
                            ts = (aL - bL) / (ag - bg);
                            ts = ts < tlo ? tlo : (ts > thi ? thi : ts);
                        }
                        const double va = aL - ag * ts, vb = bL - bg * ts;
                        Ms = va > vb ? va : vb;
                        slack = 1e-10 * (fabs(aL) + fabs(bL) + 1.0);
                        E.lines[(m * DCP + p) * DC_NL] = make_double2(aL, ag);
                        E.lines[(m * DCP + p) * DC_NL + 1] = make_double2(bL, bg);
                        n_l = 2;
                    }
                    for (int d = d0; d < d1; d++) {
                        const uint8_t* sc = ((d % 7) >= 5) ? D->wkend[m] : D->wkday[m];
#pragma unroll 1
                        for (int c0 = 0; c0 < 24; c0 += 4) {
                            const int h0 = d * 24 + c0;
                            const uint32_t pq = *reinterpret_cast<const uint32_t*>(sc + c0);
                            const float4 sv = *reinterpret_cast<const float4*>(src.shape + h0);
                            const int4 cv = *reinterpret_cast<const int4*>(src.cf + h0);
                            const float shv[4] = {sv.x, sv.y, sv.z, sv.w};
                            const int cfv[4] = {cv.x, cv.y, cv.z, cv.w};
#pragma unroll
                            for (int k = 0; k < 4; k++) {
                                if ((int)((pq >> (8 * k)) & 0xffu) != p) continue;
                                const double L = (double)shv[k] * src.load_scale;
                                const double gp = cf_per_kw(cfv[k]);
                                if (pass == 0) {
                                    mL = L > mL ? L : mL;
                                    const double vlo = L - gp * tlo, vhi = L - gp * thi;
                                    if (vlo > av) { av = vlo; aL = L; ag = gp; ah = h0 + k; }
                                    if (vhi > bv) { bv = vhi; bL = L; bg = gp; bh = h0 + k; }
                                } else if (h0 + k != ah && h0 + k != bh && L - gp * ts > Ms - slack) {
                                    if (n_l < DC_NL) E.lines[(m * DCP + p) * DC_NL + n_l++] = make_double2(L, gp);
                                    else ok = false;
                                }
                            }
                        }
                    }
                }
            }
            E.cnt[m * DCP + p] = n_l;
            E.maxl[m * DCP + p] = mL;
        }
    }
    // the other lanes of the wave read these groups.  A work-group-scope
    // release emits no vmcnt wait for a one-wave work-group (checked in the
    // ISA: the loads could overtake the stores), so: wait for every store
    // to complete, then drop the CU's L1 lines (a rebuild after a rate switch
    // rewrites lines the evaluations have cached) -- s_waitcnt vmcnt(0) +
    // buffer_inv sc1, once per build.
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    return g.first(!ok) < 0;
}

// The agent's envelope lines staged in the wave's LDS (k_size): an evaluation
// reads every present group's few lines, and from global memory each read was
// a dependent L2 round trip inside the month / group loops (the C4 k_size was
// latency-bound: SQ_WAIT_ANY ~4.6x its VALU instructions).  The groups' lines
// are packed in group order, off[k] .. off[k + 1] for group k = m x DCP + p.
constexpr int DCS_CAP = 128;                       // lines per agent (else the global path)
constexpr int DCS_NG = 12 * DCP;
struct DcStage {
    double2 lines[DCS_CAP];
    double gen[DCS_CAP];     // the lines' generation at the current evaluation's kW (yl_dc_gen)
    uint16_t off[DCS_NG + 1];
    uint16_t pad[(8 - (DCS_NG + 1) % 8) % 8];
};
constexpr size_t DCS_BYTES = sizeof(DcStage);
static_assert(DCS_BYTES % 16 == 0, "stage keeps 16-B alignment");

// Stage the envelope the segment just built (yl_dc_build's global record):
// lane sl takes groups sl, sl + LPA, ...; offsets by a segment scan in group
// order.  Segment-uniform result: false when the lines exceed DCS_CAP.
template <int LPA>
__device__ __forceinline__ bool yl_dc_stage(const DcEnv& E, DcStage* st, const Seg<LPA>& g) {
    constexpr int PER = (DCS_NG + LPA - 1) / LPA;
    int cnt[PER], off[PER];
    int base = 0;
#pragma unroll
    for (int j = 0; j < PER; j++) {
        const int k = g.sl + j * LPA;
        const int v = k < DCS_NG ? E.cnt[k] : 0;
        int incl = v;
#pragma unroll
        for (int o = 1; o < LPA; o <<= 1) {
            const int t = __shfl_up(incl, o, WAVE);
            if (g.sl >= o) incl += t;
        }
        cnt[j] = v;
        off[j] = base + incl - v;
        base += __shfl(incl, g.base + LPA - 1, WAVE);
    }
    if (base > DCS_CAP) return false;
    wave_lds_sync();                                   // the previous stage is no longer read
#pragma unroll
    for (int j = 0; j < PER; j++) {
        const int k = g.sl + j * LPA;
        if (k < DCS_NG) {
            st->off[k] = (uint16_t)off[j];
            const double2* src = E.lines + (size_t)k * DC_NL;
            for (int l = 0; l < cnt[j]; l++) st->lines[off[j] + l] = src[l];
        }
    }
    if (g.sl == 0) st->off[DCS_NG] = (uint16_t)base;
    wave_lds_sync();
    return true;
}

// Each staged line's generation term at this evaluation's kW, ref_gen(g, kW):
// the same for every year lane of the agent, so the segment's lanes form it
// once per line (a division each) instead of every lane for every line.
template <int LPA>
__device__ __forceinline__ void yl_dc_gen(DcStage* st, double kw, const Seg<LPA>& g) {
    const int n = st->off[DCS_NG];
    wave_lds_sync();                                   // the previous evaluation's reads
    for (int k = g.sl; k < n; k += LPA) st->gen[k] = ref_gen(st->lines[k].y, kw);
    wave_lds_sync();
}

// The same envelopes built by the segment's hour lanes (k_size: the serial
// month-lane build above was 60 % of the C4 search's cycles, each month lane
// walking its 730 hours twice per demand period).  Lane hd < 24 takes hour of
// day hd of every day, whose demand period is fixed per day type, so one walk
// over the year serves every period: pass 1 keeps, per day type, the lane's
// first maximiser of the import at tlo and at thi and its max load; the
// segment merges the 48 partials per (month, period) through LDS (ties to the
// earlier hour: the serial build's first maximiser); pass 2 appends the lines
// above the crossing bound (an LDS counter per period hands out positions:
// the envelope is a set, evaluations take its max).  Same lines kept, same
// overflow rule as yl_dc_build.  Loads run DCB_DAYS days ahead (the serial
// build waited on an L2 round trip per 4 hours).  `st`: the segment's stage,
// free while the envelope is rebuilt, holds the partials (240 doubles), the
// per-period bounds (16) and the counters.
// Per-day-type running maximisers of one hour lane (pass 1)
struct DcPart {
    double av, aL, ag, bv, bL, bg, mL;
    int ah, bh;
};
__device__ __forceinline__ void dc_part_init(DcPart& q) {
    q.av = -INFINITY; q.aL = 0.0; q.ag = 0.0; q.bv = -INFINITY; q.bL = 0.0; q.bg = 0.0; q.mL = 0.0;
    q.ah = 0x7fffffff; q.bh = 0x7fffffff;
}
__device__ __forceinline__ void dc_part_add(DcPart& q, double L, double gp, int h, double tlo, double thi) {
    q.mL = L > q.mL ? L : q.mL;
    const double vlo = L - gp * tlo, vhi = L - gp * thi;
    if (vlo > q.av) { q.av = vlo; q.aL = L; q.ag = gp; q.ah = h; }
    if (vhi > q.bv) { q.bv = vhi; q.bL = L; q.bg = gp; q.bh = h; }
}
constexpr int DCB_DAYS = 8;          // days of loads in flight per hour lane

template <int LPA>
__device__ __forceinline__ bool yl_dc_build_coop(const dgen_demand* D, const YSrc& src, double tlo, double thi,
                                                 const DcEnv& E, DcStage* st, const Seg<LPA>& g) {
    static_assert(sizeof(DcStage) >= 256 * sizeof(double), "stage holds the build's partials");
    double* const part = reinterpret_cast<double*>(st);          // [10][24]: 9 fields + the lane's period
    double* const prm = part + 240;                               // [2][DCP]: ts, Ms (pass 2)
    int* const ctr = reinterpret_cast<int*>(part);                // [DCP] (pass 2: partials are dead)
    const int hd = g.sl;
    const bool act = hd < 24;
    const int hq = act ? hd : 23;                                 // in-range loads for idle lanes
    bool ok = true;
    for (int m = 0; m < 12; m++) {
        const int d0 = c_month_start_day[m], d1 = c_month_start_day[m + 1];
        const int pd = (int)D->wkday[m][hq], pe = (int)D->wkend[m][hq];
        uint32_t mask = act ? (1u << pd) | (1u << pe) : 0u;
#pragma unroll
        for (int o = 1; o < LPA; o <<= 1) mask |= (uint32_t)__shfl_xor((int)mask, o, WAVE);
        // pass 1: the month's days in batches, both day types at once (the
        // day type is segment-uniform, so the branch picks one partial)
        DcPart qw, qe;
        dc_part_init(qw);
        dc_part_init(qe);
        for (int db = d0; db < d1; db += DCB_DAYS) {
            float sv[DCB_DAYS];
            int32_t cv[DCB_DAYS];
#pragma unroll
            for (int k = 0; k < DCB_DAYS; k++) {
                const int d = db + k < d1 ? db + k : d1 - 1;
                sv[k] = src.shape[d * 24 + hq];
                cv[k] = src.cf[d * 24 + hq];
            }
#pragma unroll
            for (int k = 0; k < DCB_DAYS; k++) {
                const int d = db + k;
                if (d >= d1) break;
                const double L = (double)sv[k] * src.load_scale;
                const double gp = cf_per_kw(cv[k]);
                if ((d % 7) >= 5) dc_part_add(qe, L, gp, d * 24 + hd, tlo, thi);
                else dc_part_add(qw, L, gp, d * 24 + hd, tlo, thi);
            }
        }
        // merge the 24 lanes' partials per period: reduction lane r = period r
        const bool red = hd < DCP && ((mask >> hd) & 1u);
        double A = -INFINITY, AL = 0.0, Ag = 0.0, B = -INFINITY, BL = 0.0, Bg = 0.0, ML = 0.0;
        int AH = 0x7fffffff, BH = 0x7fffffff;
        for (int dt = 0; dt < 2; dt++) {
            const DcPart& q = dt ? qe : qw;
            wave_lds_sync();
            if (act) {
                part[0 * 24 + hd] = q.av; part[1 * 24 + hd] = q.aL; part[2 * 24 + hd] = q.ag;
                part[3 * 24 + hd] = (double)q.ah;
                part[4 * 24 + hd] = q.bv; part[5 * 24 + hd] = q.bL; part[6 * 24 + hd] = q.bg;
                part[7 * 24 + hd] = (double)q.bh; part[8 * 24 + hd] = q.mL;
                part[9 * 24 + hd] = (double)(dt ? pe : pd);
            }
            wave_lds_sync();
            if (red) {
                for (int k = 0; k < 24; k++) {
                    if ((int)part[9 * 24 + k] != hd) continue;
                    const double v = part[0 * 24 + k], w = part[4 * 24 + k];
                    const int kh = (int)part[3 * 24 + k], kb = (int)part[7 * 24 + k];
                    if (v > A || (v == A && kh < AH)) { A = v; AL = part[1 * 24 + k]; Ag = part[2 * 24 + k]; AH = kh; }
                    if (w > B || (w == B && kb < BH)) { B = w; BL = part[5 * 24 + k]; Bg = part[6 * 24 + k]; BH = kb; }
                    const double ml = part[8 * 24 + k];
                    ML = ml > ML ? ml : ML;
                }
            }
        }
        // the period's crossing bound (yl_dc_build's pass-1 hand-over)
        double ts = tlo, Ms = 0.0;
        if (red) {
            if (Ag > Bg) {
                ts = (AL - BL) / (Ag - Bg);
                ts = ts < tlo ? tlo : (ts > thi ? thi : ts);
            }
            const double va = AL - Ag * ts, vb = BL - Bg * ts;
            Ms = va > vb ? va : vb;
            Ms -= 1e-10 * (fabs(AL) + fabs(BL) + 1.0);               // the slack
            E.lines[(m * DCP + hd) * DC_NL] = make_double2(AL, Ag);
            E.lines[(m * DCP + hd) * DC_NL + 1] = make_double2(BL, Bg);
        }
        wave_lds_sync();
        if (red) { prm[hd] = ts; prm[DCP + hd] = Ms; }
        wave_lds_sync();
        // each lane's two periods' bounds and excluded hours
        const double tw = prm[pd], mw = prm[DCP + pd], te = prm[pe], me = prm[DCP + pe];
        const int aw = __shfl((int)AH, g.base + pd, WAVE), bw = __shfl((int)BH, g.base + pd, WAVE);
        const int ae = __shfl((int)AH, g.base + pe, WAVE), be = __shfl((int)BH, g.base + pe, WAVE);
        wave_lds_sync();
        if (hd < DCP) ctr[hd] = 2;
        wave_lds_sync();
        // pass 2: the lines above the bound
        for (int db = d0; db < d1; db += DCB_DAYS) {
            float sv[DCB_DAYS];
            int32_t cv[DCB_DAYS];
#pragma unroll
            for (int k = 0; k < DCB_DAYS; k++) {
                const int d = db + k < d1 ? db + k : d1 - 1;
                sv[k] = src.shape[d * 24 + hq];
                cv[k] = src.cf[d * 24 + hq];
            }
#pragma unroll
            for (int k = 0; k < DCB_DAYS; k++) {
                const int d = db + k;
                if (d >= d1) break;
                const bool we = (d % 7) >= 5;
                const int h = d * 24 + hd;
                const double L = (double)sv[k] * src.load_scale;
                const double gp = cf_per_kw(cv[k]);
                const double t_ = we ? te : tw, M_ = we ? me : mw;
                const int a_ = we ? ae : aw, b_ = we ? be : bw, pp = we ? pe : pd;
                if (act && h != a_ && h != b_ && L - gp * t_ > M_) {
                    const int pos = atomicAdd(&ctr[pp], 1);
                    if (pos < DC_NL) E.lines[(m * DCP + pp) * DC_NL + pos] = make_double2(L, gp);
                    else ok = false;
                }
            }
        }
        wave_lds_sync();
        if (hd < DCP) {
            const bool here = (mask >> hd) & 1u;
            const int n_l = here ? ctr[hd] : 0;
            E.cnt[m * DCP + hd] = n_l < DC_NL ? n_l : DC_NL;
            E.maxl[m * DCP + hd] = here ? ML : 0.0;
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    return g.first(!ok) < 0;
}

// k_size's build: the hour-lane form when the segment has its stage
template <int LPA>
__device__ __forceinline__ bool yl_dc_build_any(const dgen_demand* D, const YSrc& src, double tlo, double thi,
                                                const DcEnv& E, DcStage* st, const Seg<LPA>& g) {
    if (st) return yl_dc_build_coop(D, src, tlo, thi, E, st, g);
    return yl_dc_build(D, src, tlo, thi, E, g);
}

// One lane's year of demand charges from the envelopes (same month / period /
// tier order as yl_demand): system output x s at system kW kw (ref_gen, the
// reference's operation order), or the no-system peaks (max load) when !with_gen.
// st: the agent's staged lines (or nullptr: the global record).
__device__ __forceinline__ double yl_dc_eval(const dgen_demand* D, const DcEnv& E, double kw, double s,
                                             bool with_gen, const YLds& S, const DcStage* st = nullptr,
                                             int nq = DCP) {
    // nq: the batch's demand periods (dgen_tables.max_dc_periods): a period no
    // schedule uses has no hours, a zero peak and a zero charge
    double total = 0.0;
    for (int m = 0; m < 12; m++) {
        double flat = 0.0;
        for (int q = 0; q < nq; q++) {
            const int gk = m * DCP + q;
            const int o0 = (st && with_gen) ? st->off[gk] : 0;
            const int n_l = (st && with_gen) ? st->off[gk + 1] - o0 : E.cnt[gk];
            double pk = 0.0;
            if (n_l > 0) {
                if (with_gen) {
                    if (st) {                  // the stage: generation formed by yl_dc_gen
                        for (int k = 0; k < n_l; k++) {
                            const double imp = st->lines[o0 + k].x - st->gen[o0 + k] * s;
                            pk = imp > pk ? imp : pk;
                        }
                    } else {
                        const double2* ln = E.lines + gk * DC_NL;
                        for (int k = 0; k < n_l; k++) {
                            const double2 v = ln[k];
                            const double imp = v.x - ref_gen(v.y, kw) * s;
                            pk = imp > pk ? imp : pk;
                        }
                    }
                } else {
                    pk = E.maxl[gk];
                }
            }
            S.at(q) = pk;
            flat = pk > flat ? pk : flat;
        }
        if (S.pk) S.pk[m * WAVE] = flat;          // the month's peak import (kWh/kW tiers)
        double c = dc_tier_charge(flat, D->flat_cap[m], D->flat_price[m], D->flat_nt[m]);
        for (int q = 0; q < nq; q++) c += dc_tier_charge(S.at(q), D->tou_cap[q], D->tou_price[q], D->tou_nt[q]);
        total += c;
    }
    return total;
}

// ---------------------------------------------------------------------------
// Net-billing split (PV-only search, mo 2).  The hourly pass of yl_bill_mo2
// bills max(L_h - g_h t, 0) as import and the rest as export, with t the
// generation scale (kW' x the year's degradation factor).  The search only
// evaluates t in [tlo, thi] (bracket x degradation range), and over that
// interval most hours never change side: an hour whose import is positive at
// both ends (beyond a 1e-10 relative slack that covers the rounding of the
// per-hour product) imports at every evaluated t, one negative at both ends
// always exports.  Their contributions are linear in t, so per (month,
// period) the build keeps four sums -- import load and generation, export
// generation x sell weight and load x sell weight -- and the M hours in
// between as a list.  An evaluation then bills
//     import_p = SA_L - (SA_g kW') s + sum over the period's M hours
//     export_p = (SX_gw kW') s - SX_Lw + sum over the period's M hours
// with the hourly pass's own per-hour arithmetic on the M hours: the same
// quantities as the hourly pass up to rounding (re-associated sums), on
// ~700 of 8760 hours for the synthetic CA population.  Month lane m builds
// month m once per tariff; a month with more than NB_CAPM M hours sends the
// agent back to the hourly pass.  Storage per scratch slot: NB_BYTES in the
// caller's workspace.
// ---------------------------------------------------------------------------
// The sell weight of an exported kWh: the float32-rounded TS sell rate
// (ff:756) when the reference enables it, else 1 (the period's sell column is
// applied per month).
__device__ __forceinline__ float nb_weight_f(const YSrc& src, int h) {
    return src.ts ? (float)(src.ts[h] * src.ts_mult) : 1.0f;
}
__device__ __forceinline__ double nb_weight(const YSrc& src, int h) { return (double)nb_weight_f(src, h); }

// (hour, day type) partials -> (period, quantity) sums at a month's end:
// lane r = 4 p + q (and r + LPA when 4 MAXP > LPA) adds the hour lanes'
// partials (their LDS columns) whose period is p, hours in order, weekdays
// first -- a fixed order, a re-association of the serial hour sums.
// k_nb_env's form: the month's two 24-hour schedules are read into registers
// once (6 words each) instead of a byte load per hour, each of which waited
// for its own round trip (yl_nb_build keeps those loads: inside k_size and
// k_batt_finance the registers are short, and the register form measured
// slower there).
template <int LPA>
__device__ __forceinline__ void nb_month_sums(const dgen_tariff& t, int m, int P, const Seg<LPA>& g, const YLds& S,
                                              const double* col0, const double (&a0)[4], const double (&a1)[4],
                                              const NbRec& R) {
    constexpr int NR = (4 * MAXP + LPA - 1) / LPA;
    uint32_t sw[2][6];
    {
        const uint32_t* d4 = reinterpret_cast<const uint32_t*>(t.wkday[m]);
        const uint32_t* e4 = reinterpret_cast<const uint32_t*>(t.wkend[m]);
#pragma unroll
        for (int k = 0; k < 6; k++) { sw[0][k] = d4[k]; sw[1][k] = e4[k]; }
    }
    double v[NR];
#pragma unroll
    for (int k = 0; k < NR; k++) v[k] = 0.0;
#pragma unroll
    for (int dt = 0; dt < 2; dt++) {
        wave_lds_sync();
#pragma unroll
        for (int q = 0; q < 4; q++) S.at(q) = dt ? a1[q] : a0[q];
        wave_lds_sync();
#pragma unroll
        for (int k = 0; k < NR; k++) {
            const int r = g.sl + k * LPA;
            const bool on = r < 4 * P;
            const int p = r >> 2;
            const double* cq = col0 + (on ? (r & 3) : 0) * WAVE;
#pragma unroll
            for (int hh = 0; hh < 24; hh++) {
                const int ph = (int)((sw[dt][hh >> 2] >> (8 * (hh & 3))) & 0xffu);
                const double x = cq[hh];
                v[k] = (on && ph == p) ? v[k] + x : v[k];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < NR; k++) {
        const int r = g.sl + k * LPA;
        if (r < 4 * P) R.sums[(m * MAXP + (r >> 2)) * 4 + (r & 3)] = v[k];
    }
}

// The segment builds the split cooperatively: lane k < 24 of the segment
// takes hour k of every day (all days of a month share one period per hour
// and day type), so a month is ~30 steps of 24 hours in parallel instead of
// 730 serial hours on one lane.  Each hour lane sums its own import / export
// terms per day type in registers (day order); at the month's end the lanes
// hand them over through their LDS columns and lane r = 4 p + q adds the
// (hour, day type) partials whose period is p, hours in order, weekdays
// first -- a fixed order, a re-association of the serial hour sums.  The
// mixed hours are appended in hour order (ballot rank within the day).
// Returns true when every month's M hours fit (segment-uniform).
// days per load batch: the battery case's f64 system output takes twice the
// registers of the cf row, and k_batt_finance stays at 3 waves with 4; the
// search's cf build measured 2 / 3 / 4 / 6 / 8 / 12 days: 21.2 / 20.3 / 20.0 /
// 19.8 / 20.6 / 29.4 ms of C2 k_size at 200k (12 spills); sys 2 / 3 / 4 / 8:
// 16.5 / 15.6 / 15.2 / 18.1 ms of k_batt_finance
#ifndef DGEN_NB_DB_CF
#define DGEN_NB_DB_CF 6
#endif
#ifndef DGEN_NB_DB_SYS
#define DGEN_NB_DB_SYS 4
#endif
template <bool SYS>
struct NbDays {
    static constexpr int D = SYS ? DGEN_NB_DB_SYS : DGEN_NB_DB_CF;
    float sh[D], w[D];
    int32_t cf[SYS ? 1 : D];
    double sg[SYS ? D : 1];
};
template <bool SYS>
__device__ __forceinline__ void nb_load_days(const YSrc& src, int d0, int hd, bool act, NbDays<SYS>& b) {
#pragma unroll
    for (int k = 0; k < NbDays<SYS>::D; k++) {
        const int h = (d0 + k) * 24 + hd;
        const bool v = act && d0 + k < 365;
        b.sh[k] = v ? src.shape[h] : 0.0f;
        b.w[k] = (v && src.ts) ? (float)(src.ts[h] * src.ts_mult) : 1.0f;
        if constexpr (SYS) b.sg[k] = v ? src.sysgen[(int64_t)(d0 + k) * src.sys_stride * 24 + hd] : 0.0;
        else b.cf[k] = v ? src.cf[h] : 0;
    }
}

// The segment builds the split cooperatively: lane k < 24 of the segment
// takes hour k of every day (all days of a month share one period per hour
// and day type), so a month is ~30 steps of 24 hours in parallel instead of
// 730 serial hours on one lane; the loads of the next batch of days are issued
// before the current ones are classified.  Each hour lane sums its own
// import / export terms per day type in registers (day order); at the month's
// end the lanes hand them over through their LDS columns and lane r = 4 p + q
// adds the (hour, day type) partials whose period is p, hours in order,
// weekdays first -- a fixed order, a re-association of the serial hour sums.
// The mixed hours are appended in hour order (ballot rank within the day).
// Returns true when every month's M hours fit (segment-uniform).  SYS: the
// battery case's system output (k_batt_finance), else the per-kW cf row.
template <bool SYS, int LPA>
__device__ __forceinline__ bool yl_nb_build(const dgen_tariff& t, const YSrc& src, double tlo, double thi,
                                            char* nbp, const YLds& S, const Seg<LPA>& g) {
    const NbRec R = nb_rec(nbp);
    const int P = t.P;
    const int hd = g.sl;
    const bool act = hd < 24;
    const unsigned long long segm = (LPA == WAVE) ? ~0ull : (((1ull << LPA) - 1ull) << g.base);
    const unsigned long long below = (1ull << g.lane) - 1ull;
    double* col0 = S.lane - g.sl;          // the segment's first lane's LDS column
    bool ok = true;
    constexpr int DB = NbDays<SYS>::D;
    NbDays<SYS> cur, nxt;
    nb_load_days<SYS>(src, 0, hd, act, cur);
    for (int m = 0; m < 12; m++) {
        const int pd = act ? (int)t.wkday[m][hd] : 0, pe = act ? (int)t.wkend[m][hd] : 0;
        double a0[4] = {0.0, 0.0, 0.0, 0.0}, a1[4] = {0.0, 0.0, 0.0, 0.0};
        int n_m = 0;
        NbEnt* ent = R.ent + m * NB_CAPM;
        const int de = c_month_start_day[m + 1];
#pragma unroll 1
        for (int d0 = c_month_start_day[m]; d0 < de; d0 += DB) {
            nb_load_days<SYS>(src, d0 + DB < de ? d0 + DB : de, hd, act, nxt);
#pragma unroll
            for (int k = 0; k < DB; k++) {
                const int d = d0 + k;
                if (d >= de) break;
                const bool we = (d % 7) >= 5;
                const double L = (double)cur.sh[k] * src.load_scale;
                double gk;
                if constexpr (SYS) gk = cur.sg[k];
                else gk = cf_per_kw(cur.cf[k]);
                const float w = cur.w[k];
                const double vlo = L - gk * tlo, vhi = L - gk * thi;
                const double slack = 1e-10 * (fabs(L) + fabs(gk) * thi);
                // battery case (SYS): an hour within the slack of zero joins the
                // import side (NB_SYS_ZERO_IMPORT below)
                const bool imp = act && fmin(vlo, vhi) > (SYS ? -slack : slack);   // imports at every t
                const bool exq = act && !imp && fmax(vlo, vhi) < -slack;   // exports at every t
                const double wd = (double)w;
                const double i0 = imp ? L : 0.0, i1 = imp ? gk : 0.0;
                const double x0 = exq ? gk * wd : 0.0, x1 = exq ? L * wd : 0.0;
                if (we) {
                    a1[0] += i0; a1[1] += i1; a1[2] += x0; a1[3] += x1;
                } else {
                    a0[0] += i0; a0[1] += i1; a0[2] += x0; a0[3] += x1;
                }
                const bool mx = act && !imp && !exq;
                const unsigned long long bm = __ballot(mx) & segm;
                if (mx) {
                    const int pos = n_m + __popcll(bm & below);
                    if (pos < NB_CAPM) {
                        NbEnt e;
                        e.L = L;
                        e.g = gk;
                        e.w = w;
                        e.p = we ? pe : pd;
                        ent[pos] = e;
                    }
                }
                n_m += __popcll(bm);
            }
            cur = nxt;
        }
        ok = ok && n_m <= NB_CAPM;
        if (g.sl == 0) R.cnt[m] = n_m;
        // (hour, day type) partials -> (period, quantity) sums
        // lane r and (4 MAXP > LPA) lane r + LPA (k_nb_env: nb_month_sums, the
        // same order)
        constexpr int NR = (4 * MAXP + LPA - 1) / LPA;
        double v[NR];
#pragma unroll
        for (int k = 0; k < NR; k++) v[k] = 0.0;
        for (int dt = 0; dt < 2; dt++) {
            wave_lds_sync();
#pragma unroll
            for (int q = 0; q < 4; q++) S.at(q) = dt ? a1[q] : a0[q];
            wave_lds_sync();
            const uint8_t* sc = dt ? t.wkend[m] : t.wkday[m];
#pragma unroll
            for (int k = 0; k < NR; k++) {
                const int r = g.sl + k * LPA;
                if (r < 4 * P) {
                    const int p = r >> 2, q = r & 3;
                    for (int hh = 0; hh < 24; hh++)
                        if ((int)sc[hh] == p) v[k] += col0[q * WAVE + hh];
                }
            }
        }
#pragma unroll
        for (int k = 0; k < NR; k++) {
            const int r = g.sl + k * LPA;
            if (r < 4 * P) R.sums[(m * MAXP + (r >> 2)) * 4 + (r & 3)] = v[k];
        }
    }
    // hand-off to the other lanes through global memory, as yl_dc_build
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    wave_lds_sync();
    return ok;
}

// k_nb_env's form of yl_nb_build<false>: the same hour-lane classification,
// sums and entry order (so the same split, bit for bit), but the rows come
// through an LDS stage of NBS_DAYS days per agent, filled by coalesced 16-B
// loads (segment lane k < 16: day k's 96 B of shape and of cf; lane 16 + k:
// day k's 24 float32 sell weights from the 192 B of its TS row) instead of
// one 4-B load per hour lane and day (C2 200k: k_nb_env was 7.5 ms of the
// 18.6 ms search, waiting on those loads).  Two agents per wave (LPA 32),
// each segment staging its own agent.
constexpr int NBS_DAYS = 16;
struct NbStage {                 // one segment's (agent's) days
    float sh[NBS_DAYS * 24];
    int32_t cf[NBS_DAYS * 24];
    float w[NBS_DAYS * 24];
};
constexpr size_t NBS_BYTES = sizeof(NbStage);
static_assert(NBS_BYTES % 16 == 0, "stage keeps 16-B alignment");

__device__ __forceinline__ bool cf_slow(int32_t x) { return (uint32_t)x + 20000000u > 40000000u; }

// One staged batch of nd days on the segment's hour lanes: the classification,
// sums and entries of yl_nb_build<false>'s day loop, bit for bit, with the
// batch's days formed four at a time (branch-free) ahead of their sums, and
// the sums as a += v x {0, 1} in one fma each (exact: v + a or a; a is never
// -0).  FAST: every cf value of the batch is in cf_per_kw's fast range.
template <bool FAST>
__device__ __forceinline__ void nbs_days(const NbStage* st, int hq, bool act, int nd, int d0, double ls, double tlo,
                                         double thi, bool ts, int pd, int pe, double (&a0)[4], double (&a1)[4],
                                         int& n_m, NbEnt* ent, unsigned long long segm, unsigned long long below) {
    const int dow0 = d0 % 7;
#pragma unroll 1
    for (int k0 = 0; k0 < nd; k0 += 4) {
        double L[4], G[4], mi[4], me[4];
        float W[4];
        bool mx[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int o = (k0 + j) * 24 + hq;       // k0 + j < NBS_DAYS: a day past nd is stale, unused
            const double Lj = (double)st->sh[o] * ls;
            const double gk = FAST ? cf_per_kw_fast(st->cf[o]) : cf_per_kw(st->cf[o]);
            const float w = ts ? st->w[o] : 1.0f;
            const double vlo = Lj - gk * tlo, vhi = Lj - gk * thi;
            const double slack = 1e-10 * (fabs(Lj) + fabs(gk) * thi);
            const bool imp = act && fmin(vlo, vhi) > slack;              // imports at every t
            const bool exq = act && !imp && fmax(vlo, vhi) < -slack;     // exports at every t
            L[j] = Lj;
            G[j] = gk;
            W[j] = w;
            mi[j] = imp ? 1.0 : 0.0;
            me[j] = exq ? 1.0 : 0.0;
            mx[j] = act && !imp && !exq;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (k0 + j >= nd) break;                 // uniform
            const bool we = ((dow0 + k0 + j) % 7) >= 5;
            const double wd = (double)W[j];
            const double x0 = G[j] * wd, x1 = L[j] * wd;
            if (we) {
                a1[0] = __builtin_fma(L[j], mi[j], a1[0]); a1[1] = __builtin_fma(G[j], mi[j], a1[1]);
                a1[2] = __builtin_fma(x0, me[j], a1[2]);   a1[3] = __builtin_fma(x1, me[j], a1[3]);
            } else {
                a0[0] = __builtin_fma(L[j], mi[j], a0[0]); a0[1] = __builtin_fma(G[j], mi[j], a0[1]);
                a0[2] = __builtin_fma(x0, me[j], a0[2]);   a0[3] = __builtin_fma(x1, me[j], a0[3]);
            }
            const unsigned long long bm = __ballot(mx[j]) & segm;
            if (mx[j]) {
                const int pos = n_m + __popcll(bm & below);
                if (pos < NB_CAPM) {
                    NbEnt e;
                    e.L = L[j];
                    e.g = G[j];
                    e.w = W[j];
                    e.p = we ? pe : pd;
                    ent[pos] = e;
                }
            }
            n_m += __popcll(bm);
        }
    }
}

template <int LPA>
__device__ __forceinline__ bool yl_nb_build_stg(const dgen_tariff& t, const YSrc& src, double tlo, double thi,
                                                char* nbp, const YLds& S, const Seg<LPA>& g, NbStage* st) {
    static_assert(LPA == 32, "k_nb_env runs two agents per wave");
    const NbRec R = nb_rec(nbp);
    const int P = t.P;
    const int hd = g.sl;
    const bool act = hd < 24;
    const int hq = act ? hd : 0;
    const unsigned long long segm = ((1ull << LPA) - 1ull) << g.base;
    const unsigned long long below = (1ull << g.lane) - 1ull;
    double* col0 = S.lane - g.sl;          // the segment's first lane's LDS column
    bool ok = true;
    // the next batch's rows in flight during the current batch's days: lane
    // sl < NBS_DAYS holds day sl's 24 shape values, lane NBS_DAYS + k day k's
    // 24 cf values (16-B loads; a day past the batch repeats its last day)
    const int kf = g.sl & (NBS_DAYS - 1);
    const bool pf_cf = g.sl >= NBS_DAYS;
    uint4 pf[6];
    auto fetch = [&](int b0, int bn) {
        const int d = b0 + (kf < bn ? kf : bn - 1);
        const uint4* p4 = pf_cf ? reinterpret_cast<const uint4*>(src.cf + d * 24)
                                : reinterpret_cast<const uint4*>(src.shape + d * 24);
#pragma unroll
        for (int q = 0; q < 6; q++) pf[q] = p4[q];
    };
    fetch(0, NBS_DAYS);
    for (int m = 0; m < 12; m++) {
        const int pd = act ? (int)t.wkday[m][hd] : 0, pe = act ? (int)t.wkend[m][hd] : 0;
        double a0[4] = {0.0, 0.0, 0.0, 0.0}, a1[4] = {0.0, 0.0, 0.0, 0.0};
        int n_m = 0;
        NbEnt* ent = R.ent + m * NB_CAPM;
        const int ds = c_month_start_day[m], de = c_month_start_day[m + 1];
#pragma unroll 1
        for (int d0 = ds; d0 < de; d0 += NBS_DAYS) {
            const int nd = de - d0 < NBS_DAYS ? de - d0 : NBS_DAYS;
            wave_lds_sync();                              // the previous batch's reads
            bool bad = false;                             // a cf value outside cf_per_kw's fast range
            {
                uint4* dst = reinterpret_cast<uint4*>(pf_cf ? reinterpret_cast<char*>(st->cf + kf * 24)
                                                            : reinterpret_cast<char*>(st->sh + kf * 24));
#pragma unroll
                for (int q = 0; q < 6; q++) {
                    dst[q] = pf[q];
                    bad = bad | (pf_cf & (cf_slow((int32_t)pf[q].x) | cf_slow((int32_t)pf[q].y) |
                                          cf_slow((int32_t)pf[q].z) | cf_slow((int32_t)pf[q].w)));
                }
            }
            if (src.ts) {                                 // sell weights: lane sl = day sl / 2, half sl % 2
                const int k = g.sl >> 1, hf = g.sl & 1;
                const int d = d0 + (k < nd ? k : nd - 1);
                const double2* t2 = reinterpret_cast<const double2*>(src.ts + d * 24 + hf * 12);
                double2 tv[6];
#pragma unroll
                for (int q = 0; q < 6; q++) tv[q] = t2[q];
#pragma unroll
                for (int q = 0; q < 3; q++)
                    reinterpret_cast<float4*>(st->w + k * 24 + hf * 12)[q] =
                        make_float4((float)(tv[2 * q].x * src.ts_mult), (float)(tv[2 * q].y * src.ts_mult),
                                    (float)(tv[2 * q + 1].x * src.ts_mult), (float)(tv[2 * q + 1].y * src.ts_mult));
            }
            {                                             // the next batch (maybe next month's first)
                // drain what is pending (this month's pd / pe bytes): the day
                // loop uses them, and a value pending at the loop's entry
                // makes the compiler drain vmcnt there -- the prefetch with it
                __builtin_amdgcn_s_waitcnt(0x0F70);       // vmcnt(0)
                const int nx = d0 + nd;
                if (nx < 365) {
                    const int me = c_month_start_day[(nx < de ? m : m + 1) + 1];
                    fetch(nx, me - nx < NBS_DAYS ? me - nx : NBS_DAYS);
                }
            }
            wave_lds_sync();
            // wave-uniform: every staged cf value of both segments takes
            // cf_per_kw's fast form, so the days run without its branch
            if (__ballot(bad) == 0)
                nbs_days<true>(st, hq, act, nd, d0, src.load_scale, tlo, thi, src.ts != nullptr, pd, pe, a0, a1,
                               n_m, ent, segm, below);
            else
                nbs_days<false>(st, hq, act, nd, d0, src.load_scale, tlo, thi, src.ts != nullptr, pd, pe, a0, a1,
                                n_m, ent, segm, below);
        }
        ok = ok && n_m <= NB_CAPM;
        if (g.sl == 0) R.cnt[m] = n_m;
        nb_month_sums<LPA>(t, m, P, g, S, col0, a0, a1, R);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    wave_lds_sync();
    return ok;
}

// Net-billing bill of the lane's year from the split (generation kW' =
// src.gen_scale, degradation factor s; battery case: src.sysgen with
// gen_scale 1): yl_bill_mo2's result up to the rounding of the re-associated
// import / export sums.
// max of a segment-uniform count in [0, LPA] over the wave's segments
// (wave-uniform).  A segment whose lanes are inactive here (the wave's other
// agent on another path) contributes a stale value, so the result is clamped
// to LPA: extra trips are predicated off by the caller.
template <int LPA>
__device__ __forceinline__ int nb_wave_max(int v) {
    int r;
    if constexpr (LPA == WAVE) {
        r = __builtin_amdgcn_readfirstlane(v);
    } else {
        const int a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, LPA);
        r = a > b ? a : b;
    }
    return r < LPA ? r : LPA;
}

// The M entries reach the lanes through LDS in chunks of LPA: lane k loads
// entry j0 + k of the next chunk (one coalesced 24-B record per lane) while
// the segment bills the current chunk out of the lanes' LDS columns (slots
// 2 half .. 2 half + 2, broadcast reads), so the record's load latency is
// paid about once per evaluation instead of once per 4 entries; the month's
// four sums per period are staged the same way (slots 2 half + 3 ..), fetched
// one month ahead.  Needs 4 half >= 2 half + 3 + NR (dgen_size_agents raises
// max_periods to 3 for net-billing batches).  Same per-entry arithmetic and
// order as the hourly pass on the M hours.
template <int LPA>
__device__ __forceinline__ double yl_bill_nb(const dgen_tariff& t, const YSrc& src, double s, char* nbp,
                                             const YLds& S, const Seg<LPA>& g, bool compact = false) {
    const NbRec R = nb_rec(nbp);
    const int P = t.P, half = S.half;
    const double kws = src.gen_scale;
    const bool sysg = src.sysgen != nullptr, tsw = src.ts != nullptr;
    double* col0 = S.lane - g.sl;
    const int E = 2 * half;                      // staged entry: L, g, (w, p)
    constexpr int NR = (4 * MAXP + LPA - 1) / LPA;
    const int EQ = E + 3;                        // staged month sums
    const int cnt_l = g.sl < 12 ? R.cnt[g.sl] : 0;
    const unsigned long long segm = (LPA == WAVE) ? ~0ull : (((1ull << LPA) - 1ull) << g.base);
    const unsigned long long below = (1ull << g.lane) - 1ull;
    double xL = 0.0, xg = 0.0, xwp = 0.0;        // this lane's entry of the fetched chunk
    int fm = -1, fj = 0;                         // which chunk the registers hold
    auto fetch = [&](int m, int j0, int n) __attribute__((always_inline)) {
        const int j = j0 + g.sl;
        if (j < n && compact) {   // NbEntC: the load re-derived from the hour's shape value
            const NbEntC* e = reinterpret_cast<const NbEntC*>(R.ent) + m * NB_CAPM + j;
            const double2 v = *reinterpret_cast<const double2*>(e);
            const long long sp = __double_as_longlong(v.y);
            xg = v.x;
            xL = (double)__int_as_float((int)(sp & 0xffffffffll)) * src.load_scale;
            xwp = __longlong_as_double((sp & ~0xffffffffll) | (long long)(unsigned)__float_as_int(1.0f));
        } else if (j < n) {
            const double* e = reinterpret_cast<const double*>(R.ent + m * NB_CAPM + j);
            xL = e[0];
            xg = e[1];
            xwp = e[2];
        }
        fm = m;
        fj = j0;
    };
    double sv[NR];
    auto fetch_sums = [&](int m) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < NR; k++) {
            const int r = g.sl + k * LPA;
            sv[k] = r < 4 * P ? R.sums[(m * MAXP + (r >> 2)) * 4 + (r & 3)] : 0.0;
        }
    };
    fetch_sums(0);
    {
        const int n0 = __shfl(cnt_l, g.base, WAVE);
        fetch(0, 0, n0);
    }
    double total = 0.0, carry = 0.0;
    for (int m = 0; m < 12; m++) {
        const int n_m = __shfl(cnt_l, g.base + m, WAVE);
        const int n_n = __shfl(cnt_l, g.base + (m + 1 < 12 ? m + 1 : 11), WAVE);
        if (n_m > 0 && !(fm == m && fj == 0)) fetch(m, 0, n_m);
        wave_lds_sync();
#pragma unroll
        for (int k = 0; k < NR; k++) S.at(EQ + k) = sv[k];
        wave_lds_sync();
        for (int p = 0; p < P; p++) {
            const double q0 = col0[(EQ + (4 * p) / LPA) * WAVE + (4 * p) % LPA];
            const double q1 = col0[(EQ + (4 * p + 1) / LPA) * WAVE + (4 * p + 1) % LPA];
            const double q2 = col0[(EQ + (4 * p + 2) / LPA) * WAVE + (4 * p + 2) % LPA];
            const double q3 = col0[(EQ + (4 * p + 3) / LPA) * WAVE + (4 * p + 3) % LPA];
            S.at(p) = q0 - (q1 * kws) * s;
            S.at(half + p) = (q2 * kws) * s - q3;
        }
        if (m + 1 < 12) fetch_sums(m + 1);
        int cur = 0;
        double ci = S.at(0), ce = S.at(half);
        PH_T0(tl);
        PH_CNT(10, n_m, g.sl == 0);
        for (int j0 = 0; j0 < n_m; j0 += LPA) {
            const int kn = (n_m - j0 < LPA) ? n_m - j0 : LPA;
            // the chunk is staged grouped by period (hour order within a
            // period), so the running accumulator switches at most P times a
            // chunk while each period still adds its entries in hour order;
            // the slots past the chunk's kn entries hold zero entries of its
            // last period (they add exact zeros), so both segments of the wave
            // run the same trip count
            const int myp = g.sl < kn ? (int)(__double_as_longlong(xwp) >> 32) : MAXP;
            int dst = g.sl, lastp = 0;
            {
                int base = 0;
                for (int q = 0; q < P; q++) {
                    const unsigned long long bm = __ballot(myp == q) & segm;
                    if (myp == q) dst = base + __popcll(bm & below);
                    base += __popcll(bm);
                    if (bm) lastp = q;
                }
            }
            const double pad = __longlong_as_double((long long)lastp << 32);
            wave_lds_sync();
            col0[E * WAVE + dst] = g.sl < kn ? xL : 0.0;
            // the generation term at this evaluation's kW' (cf / 1e6 x kW', the
            // same product every lane formed per entry; the battery case's system
            // output as is), formed once by the staging lane
            col0[(E + 1) * WAVE + dst] = g.sl < kn ? (sysg ? xg : xg * kws) : 0.0;
            col0[(E + 2) * WAVE + dst] = g.sl < kn ? xwp : pad;
            wave_lds_sync();
            if (j0 + LPA < n_m) fetch(m, j0 + LPA, n_m);
            else if (m + 1 < 12 && n_n > 0) fetch(m + 1, 0, n_n);
            const int kw = nb_wave_max<LPA>(kn);
            // per entry, the hourly pass's arithmetic: load, generation
            // cf / 1e6 x kW' (the battery case's system output as is), x the
            // year's factor; an import adds dd, an export adds -dd (x the TS
            // sell weight), the other side an exact 0
            auto run = [&](auto tsw_c) __attribute__((always_inline)) {
                constexpr bool TSW = decltype(tsw_c)::value;
#pragma unroll 4
                for (int k = 0; k < kw; k++) {
                    const double eL = col0[E * WAVE + k];
                    const double eg = col0[(E + 1) * WAVE + k];
                    const double ewp = col0[(E + 2) * WAVE + k];
                    const int64_t wpb = __double_as_longlong(ewp);
                    const int p = (int)(wpb >> 32);
                    if (p != cur) {
                        S.at(cur) = ci;
                        S.at(half + cur) = ce;
                        cur = p;
                        ci = S.at(p);
                        ce = S.at(half + p);
                    }
                    const double dd = eL - eg * s;
                    ci += fmax(dd, 0.0);
                    double e = fmax(-dd, 0.0);
                    if constexpr (TSW) e *= (double)__int_as_float((int)(wpb & 0xffffffff));
                    ce += e;
                }
            };
            if (tsw) run(std::true_type{});
            else run(std::false_type{});
        }
        PH_ADD(11, tl, g.sl == 0);
        S.at(cur) = ci;
        S.at(half + cur) = ce;
        double cr = 0.0;
        for (int p = 0; p < P; p++) {
            const double e = S.at(half + p);
            cr += src.ts ? e : e * t.sell[p][0];
        }
        total += nb_month(t, yl_month_charge(t, m, S, 0), cr, carry);
    }
    wave_lds_sync();
    return total;
}

// Net-billing (mo 2) bill with no system: every hour imports its load, so the
// (month, period) imports are the slot-sum load bins (yl_build_bins).
__device__ __forceinline__ double yl_bill_mo2_nogen(const dgen_tariff& t, const YLds& S) {
    const int P = t.P, half = S.half;
    double total = 0.0;
    for (int m = 0; m < 12; m++) {
        for (int p = 0; p < P; p++) S.at(p) = S.L[m * half + p];
        total += t.fixed + yl_month_charge(t, m, S, 0);
    }
    return total;
}

// The same no-system bill month-parallel (year-independent): lane m < 12 of
// the segment bills month m in its own LDS column, the months added in order.
template <int LPA>
__device__ __forceinline__ double yl_bill_mo2_nogen_par(const dgen_tariff& t, const YLds& S, const Seg<LPA>& g) {
    const int P = t.P, half = S.half;
    const int m = g.sl < 12 ? g.sl : 11;
    for (int p = 0; p < P; p++) S.at(p) = S.L[m * half + p];
    const double b = t.fixed + yl_month_charge(t, m, S, 0);
    double total = 0.0;
    for (int mm = 0; mm < 12; mm++) total += __shfl(b, g.base + mm, WAVE);
    return total;
}

// bins of a tariff from a row's slot sums, one (month, period) cell per lane
template <int LPA>
__device__ __forceinline__ void yl_build_bins(const dgen_tariff& t, const double* __restrict__ lslots,
                                              const double* __restrict__ gslots, double load_scale,
                                              const YLds& S, const Seg<LPA>& g) {
    const int P = t.P;
    for (int cell = g.sl; cell < 12 * P; cell += LPA) {
        int m = cell / P, p = cell % P;
        double la = 0.0, ga = 0.0;
        // the month's 48 slot sums of both rows in batches of BB (2 BB loads
        // in flight, branch-free), then the period's slots added in slot order
        // (the oracle's order; a skipped slot is a select, not a + 0.0)
        constexpr int BB = 8;
        const double* lm = lslots + m * 48;
        const double* gm = gslots + m * 48;
        for (int dt = 0; dt < 2; dt++) {
            const uint8_t* sched = dt ? t.wkend[m] : t.wkday[m];
#pragma unroll 1
            for (int h0 = 0; h0 < 24; h0 += BB) {
                double lv[BB], gv[BB];
#pragma unroll
                for (int k = 0; k < BB; k++) {
                    lv[k] = lm[dt * 24 + h0 + k];
                    gv[k] = gm[dt * 24 + h0 + k];
                }
#pragma unroll
                for (int k = 0; k < BB; k++) {
                    const bool on = sched[h0 + k] == p;
                    la = on ? la + lv[k] : la;
                    ga = on ? ga + gv[k] : ga;
                }
            }
        }
        S.L[m * S.half + p] = la * load_scale;
        S.G[m * S.half + p] = ga;
    }
    wave_lds_sync();
}

// Per-agent loan constants (wave-uniform) + per-lane year factors.
struct YLoan {
    int N, term, market, sl_years, depr_type;
    double r_loan, loan_f, itc_pct, itc_max, ins_rate, debt_frac, fed, sta, rr;
    // lane (year y = lane + 1) factor
    double ins_esc;   // (1 + infl)^(y - 1)
};

__device__ __forceinline__ YLoan yl_make_loan(const dgen_agents& A, const dgen_cfg& cfg, int64_t i,
                                              int N, bool is_res, int y) {
    YLoan L;
    L.N = N;
    L.term = A.loan_term[i];
    L.market = is_res ? 0 : 1;
    double infl = (A.inflation[i] * 100.0) * 0.01;
    double real = (A.real_discount[i] * 100.0) * 0.01;
    double nom = (1.0 + real) * (1.0 + infl) - 1.0;
    L.rr = 1.0 / (1.0 + nom);
    double tax_pct = A.tax_rate[i] * 100.0;
    L.fed = (tax_pct * 0.7) * 0.01;
    L.sta = (tax_pct * 0.3) * 0.01;
    L.r_loan = cfg.loan_rate_pct * 0.01;
    L.loan_f = pow_seq(1.0 + L.r_loan, L.term);
    L.itc_pct = A.itc_frac[i];                 // ff:285: the fraction passed as the percent
    L.itc_max = cfg.itc_fed_max;
    L.ins_rate = cfg.insurance_rate_pct * 0.01;
    L.debt_frac = (100.0 - (A.down_payment[i] * 100.0)) * 0.01;
    L.sl_years = cfg.depr_sl_years;
    L.depr_type = is_res ? 0 : 2;
    L.ins_esc = pow_seq(1.0 + infl, y - 1);
    return L;
}

struct YFlow {
    double npv, payback, pb;   // pb: this lane's cf_payback_with_expenses
};

// Cash flow of one lane's year + the wave reductions (Cashloan subset).
template <int LPA>
__device__ __forceinline__ YFlow yl_cashflow(const YLoan& L, double C, double ev, int y,
                                             const Seg<LPA>& g, bool active, const YLds& S) {
    double debt = L.debt_frac * C;
    double pmt = 0.0;
    if (L.term > 0 && debt != 0.0) {
        if (L.r_loan != 0.0) pmt = debt * L.r_loan / (1.0 - 1.0 / L.loan_f);
        else pmt = debt / (double)L.term;
    }
    double itc = L.itc_pct * 0.01 * C;
    if (itc > L.itc_max) itc = L.itc_max;
    double basis = C - 0.5 * itc;
    double oe = (L.ins_rate * C) * L.ins_esc;
    const bool paying = y <= L.term && pmt != 0.0;
    const double payment = paying ? pmt : 0.0;
    double itc_y = (y == 1) ? itc : 0.0;
    double sta_tax = 0.0, fed_tax = 0.0;
    if (L.market != 0) {
        // interest is deductible for commercial agents only; the balance
        // entering year y follows the same sequential recursion (years past the
        // term or the analysis period leave it unchanged or are unused)
        double bal = debt;
        const int kend = min(min(y, L.term + 1), L.N + 1);
        if (pmt != 0.0)
            for (int k = 1; k < kend; k++) bal = bal - (pmt - bal * L.r_loan);
        const double interest = paying ? bal * L.r_loan : 0.0;
        double dep = depr_frac(L.depr_type, y, L.sl_years) * basis;
        sta_tax = L.sta * (ev - oe - interest - dep);
        fed_tax = L.fed * (ev - oe - interest - dep - sta_tax);
    }
    double taxsav = itc_y - sta_tax - fed_tax;
    double atcf = ev - oe - payment + taxsav;
    double pb = ev - oe + taxsav;
    if (!active) { atcf = 0.0; pb = 0.0; }
    YFlow f;
    // NPV and the payback's cumulative flow in the oracle's order, which is
    // SSC's (libfin::npv: acc = rr acc + atcf_y for y = N .. 1, npv = atcf_0 +
    // acc rr; the cumulative sum year by year from -C), so the search's
    // objective carries no re-association of its own: scipy's parabolic step
    // divides differences of nearly equal objectives and amplifies a few ulps
    // into a different Brent path.  The lanes' flows go
    // through two rows of the lane area (free between bills) and every lane
    // of the segment runs the chains on broadcast reads; lanes past the
    // analysis period hold 0, so chaining over all LPA lanes gives the same bits.
    wave_lds_sync();                          // the bill's last reads of the lane area
    S.lane[0] = atcf;
    S.lane[WAVE] = pb;
    wave_lds_sync();
    const double* col = S.lane - g.lane + g.base;
    // the chains start at the wave's longest analysis period (wave-uniform
    // trip count; a segment's lanes past its own period hold 0).  The other
    // segment may be inactive here (diverged Brent paths): whatever its lane
    // returns, the count stays within [own period, LPA], where every extra
    // step adds an exact zero
    int nmax = L.N < LPA ? L.N : LPA;
    if constexpr (LPA < WAVE) {
        const int o = __shfl_xor(nmax, LPA, WAVE);
        nmax = o > nmax ? (o < LPA ? o : LPA) : nmax;
    }
    nmax = __builtin_amdgcn_readfirstlane(nmax);
    double acc = 0.0, run = -C, cum = -C;
#pragma unroll 4
    for (int k = nmax - 1; k >= 0; k--) acc = L.rr * acc + col[k];
#pragma unroll 4
    for (int k = 0; k < nmax; k++) {
        run = run + col[WAVE + k];
        cum = (g.sl == k) ? run : cum;
    }
    f.npv = -(C - debt) + acc * L.rr;
    const int k = g.first(active && cum > 0.0);          // first paying year - 1
    f.payback = 1e99;
    if (k >= 0) {
        double cum_k = g.bcast(cum, k), pb_k = g.bcast(pb, k);
        f.payback = (pb_k != 0.0) ? (double)(k + 1) - cum_k / pb_k : (double)(k + 1) - 0.5;
    }
    f.pb = pb;
    return f;
}

struct YLast {   // per-lane results of the most recent evaluation
    double total, ev, w, wo;
    YFlow flow;
};

template <int LPA>
struct YCtx {
    const dgen_tariff* tariffs;
    const dgen_tariff* tp;      // current tariff (global record or LDS copy)
    const dgen_switch* sw_rows;
    const dgen_demand* dem_table;
    const dgen_demand* dem;     // current tariff's demand record (charges, or the peaks of kWh/kW tiers)
    int n_dem;
    bool dc_on;                 // demand charges billed (extension mode)
    bool dem_bill;              // the record's charges count (dc_on and the tariff's own record)
    bool pk13;                  // kWh/kW tiers: the demand pass runs ahead of the energy bill
    bool dem_wo_pending;        // wo1 still lacks the new tariff's demand charge
    bool env_ok;                // the demand envelopes of the current tariff fit
    DcEnv env;                  // the agent's envelope storage
    DcStage* stg;               // the segment's LDS stage of the envelope lines (k_size)
    bool stg_ok;                // the current envelope is staged
    char* nb;                   // the agent's net-billing split record (or nullptr)
    bool nb_ok;                 // the split of the current (mo 2) tariff fits
    int nb_tag;                 // 1 + the tariff the record holds the split of (0: none)
    int dc_nq;                  // the batch's demand periods (dgen_tables.max_dc_periods)
    bool nb_pending;            // the current (mo 2) tariff's split is not formed yet
    int env_tag;                // 1 + the tariff the envelopes are of (0: none)
    double tlo, thi;            // generation-scale range of the search
    int sw_cnt;
    int tariff, switched, status;
    double capex, ccm, kwh, yearend, load_scale;
    double r_y, s_y;      // lane factors (1 + infl + esc)^(y-1), (1 - deg)^(y-1)
    double wo1;           // year-1 no-system bill, current tariff
    const double* lslots;
    const double* gslots;
    const double* ts_row;     // the agent's 8760 wholesale row (non-CA), or nullptr
    YSrc src;
    YLds S;
    YLoan loan;
    YLast last;
    Seg<LPA> g;
    int y, N;
    bool active;
    __device__ explicit YCtx(int lane) : g(lane) {}
};

// The current tariff's demand envelopes, built here at the first evaluation
// billed with the tariff (the segment's hour lanes, yl_dc_build_any).  A
// separate prebuild kernel ahead of k_size measured slower (C4 200k: k_size
// 35.7 -> 41.4 ms) and was removed.
template <int LPA>
__device__ __forceinline__ bool yl_dc_ready(YCtx<LPA>& c, const DcEnv& E, DcStage* st, const Seg<LPA>& g) {
    if (!E.lines) return false;
    if (c.env_tag == c.tariff + 1) return true;
    if (c.env_tag == -(c.tariff + 1)) return false;        // k_dc_env found a group over DC_NL lines
    const bool ok = yl_dc_build_any(c.dem, c.src, c.tlo, c.thi, E, st, g);
    c.env_tag = ok ? c.tariff + 1 : 0;
    return ok;
}

// NET: the batch may bill net (it has scratch slots, dgen_size_agents); the
// NEM-only instantiation compiles the net-billing paths out, so the common
// case's register allocation does not carry them (an agent that would still
// reach one flags DGEN_ST_SCRATCH, which assign_scratch rules out).
template <int LPA, bool DC, bool NET, bool PK>
__device__ __forceinline__ void yl_set_tariff(YCtx<LPA>& c, int tix) {
    c.tp = stage_tariff(c.tariffs + tix, c.S, c.g);
    const dgen_tariff& t = *c.tp;
    c.tariff = tix;
    c.status |= t.flags;
    // the 8760 TS sell rate applies under net billing option 2 only (ff:626-641)
    c.src.ts = (t.mo == 2) ? c.ts_row : nullptr;
    double wo_dem = 0.0;
    if constexpr (DC && !PK) {   // launched only with demand charges billed
        c.dem = tariff_demand(c.dem_table, c.n_dem, true, t);
        c.dem_wo_pending = c.dem != nullptr;
    } else if constexpr (PK) {
        const dgen_demand* bill = tariff_demand(c.dem_table, c.n_dem, c.dc_on, t);
        c.pk13 = peak_unit(t);
        c.dem = c.pk13 ? tariff_peaks(c.dem_table, c.n_dem, t) : bill;
        c.dem_bill = bill != nullptr;
        c.dem_wo_pending = c.dem != nullptr;
        if (c.pk13 && (!c.dem || !c.S.pk)) c.status |= DGEN_ST_UNIT;
        if (c.pk13 && c.dem && c.S.pk) {
            // kWh/kW tiers: the month peaks come before the energy bills, so
            // the envelopes are built and the no-system pass runs here (its
            // charge, when billed, joins the no-system bill below)
            c.env_ok = yl_dc_ready(c, c.env, c.stg, c.g);
            c.stg_ok = c.env_ok && c.stg && yl_dc_stage(c.env, c.stg, c.g);
            const double v0 = c.env_ok ? yl_dc_eval(c.dem, c.env, 0.0, 1.0, false, c.S, nullptr, c.dc_nq)
                                       : yl_demand(c.dem, c.src, 0.0, 1.0, false, c.S);
            wo_dem = c.dem_bill ? v0 : 0.0;
            c.dem_wo_pending = false;
        }
    } else {
        if (peak_unit(t)) c.status |= DGEN_ST_UNIT;   // no peaks without the demand machinery
    }
    if (!net_hourly(t)) {
        PH_T0(tn);
        wave_lds_sync();
        yl_build_bins(t, c.lslots, c.gslots, c.load_scale, c.S, c.g);
        c.wo1 = yl_bill_nem_nosys(t, c.S, c.yearend, c.g);
        PH_ADD_KS(12, tn, c.g.sl == 0);        // NEM set_tariff (bins + no-system bill)
    } else if constexpr (NET) {
        // net billing: the no-system bill from the load bins
        wave_lds_sync();
        yl_build_bins(t, c.lslots, c.gslots, c.load_scale, c.S, c.g);
        c.wo1 = yl_bill_mo2_nogen_par(t, c.S, c.g);
        // the split is formed at the first evaluation billed with this tariff
        // (an agent the rate switch moves at its first evaluation never needs
        // its initial tariff's)
        c.nb_pending = true;
    } else {
        c.status |= DGEN_ST_SCRATCH;
        c.wo1 = NAN;
    }
    // other tariffs' no-system demand charge is added by the next objective
    c.wo1 += wo_dem;
}

// calc_system_performance(kw, en_batt=False) with lanes = years; returns -NPV
// (wave-uniform).  Every evaluation leaves its per-lane results in `c.last`:
// after the search they are the outputs of the last evaluation (ff:449-474).
template <int LPA, bool DC, bool NET, bool PK>
__device__ __forceinline__ double yl_objective(YCtx<LPA>& c, double kw) {
    double otc = 0.0;
    if (kw > 0.0) {
        int nt;
        otc = rate_switch(c.sw_rows, c.sw_cnt, kw, &nt);
        if (nt >= 0) {
            c.switched = 1;
            if (nt != c.tariff) yl_set_tariff<LPA, DC, NET, PK>(c, nt);
        }
    }
    const dgen_tariff& t = *c.tp;
    double kws = ((kw * 1000.0) * 0.96) / 1000.0;                  // ff:118-120
    double total = ((c.capex * kw + 0.0) * c.ccm) + 0.0 + otc;     // ff:263,280-282
    double wb;
    double v13 = 0.0;
    if constexpr (PK) {
        if (c.pk13 && c.dem && c.S.pk) {
            // kWh/kW tiers: this evaluation's month peaks (and demand charge)
            // ahead of the energy bill, whose tier caps scale with them
            c.src.gen_scale = kws;
            if (c.env_ok && c.stg_ok) yl_dc_gen(c.stg, kw, c.g);
            const double v = c.env_ok ? yl_dc_eval(c.dem, c.env, kw, c.s_y, true, c.S, c.stg_ok ? c.stg : nullptr, c.dc_nq)
                                      : yl_demand(c.dem, c.src, kw, c.s_y, true, c.S);
            v13 = c.dem_bill ? v : 0.0;
        }
    }
    if (!net_hourly(t)) {
        PH_T0(tn);
        wb = yl_bill_nem(t, c.S, c.s_y * kws, c.yearend);
        PH_ADD_KS(13, tn, c.g.sl == 0);        // NEM evaluation bill
    } else if constexpr (NET) {
        if (c.nb_pending) {
            // the first-evaluation tariff's split comes from k_nb_env (tag);
            // any other is built here
            PH_T0(tb);
            if (c.nb && c.nb_tag != c.tariff + 1) {
                const bool ok = yl_nb_build<false>(t, c.src, c.tlo, c.thi, c.nb, c.S, c.g);
                c.nb_tag = ok ? c.tariff + 1 : 0;
                PH_CNT(7, 1, c.g.sl == 0);
            }
            PH_ADD(1, tb, c.g.sl == 0);
            c.nb_ok = c.nb && c.nb_tag == c.tariff + 1;
            c.nb_pending = false;
        }
        c.src.gen_scale = kws;
        PH_T0(te);
        wb = c.nb_ok ? yl_bill_nb(t, c.src, c.s_y, c.nb, c.S, c.g) : yl_bill_mo2(t, c.src, c.s_y, true, c.S);
        PH_ADD(c.nb_ok ? 2 : 3, te, c.g.sl == 0);
        PH_CNT(8, 1, c.g.sl == 0);
    } else {
        wb = NAN;
    }
    if constexpr (DC) {
        if (PK && c.pk13) {
            wb += v13;
        } else if (c.dem) {
            // one inlined demand pass for both uses: the no-system charge of a
            // newly set tariff (pass 0, once), then this evaluation's (pass 1)
            c.src.gen_scale = kws;
            if (c.dem_wo_pending) {
                PH_T0(tdb);
                c.env_ok = yl_dc_ready(c, c.env, c.stg, c.g);
                c.stg_ok = c.env_ok && c.stg && yl_dc_stage(c.env, c.stg, c.g);
                PH_ADD(1, tdb, c.g.sl == 0);          // demand envelopes: build + stage
                PH_CNT(7, 1, c.g.sl == 0);
            }
            PH_T0(tde);
            if (c.env_ok && c.stg_ok) yl_dc_gen(c.stg, kw, c.g);
            for (int pass = c.dem_wo_pending ? 0 : 1; pass < 2; pass++) {
                const bool wg = pass == 1;
                const double s = wg ? c.s_y : 1.0;
                const double v = c.env_ok ? yl_dc_eval(c.dem, c.env, kw, s, wg, c.S, c.stg_ok ? c.stg : nullptr, c.dc_nq)
                                          : yl_demand(c.dem, c.src, kw, s, wg, c.S);
                if (wg) wb += v;
                else c.wo1 += v;
            }
            PH_ADD(3, tde, c.g.sl == 0);              // demand-charge evaluation
            PH_CNT(8, 1, c.g.sl == 0);
            c.dem_wo_pending = false;
        }
    }
    double w = wb * c.r_y;
    double wo = c.wo1 * c.r_y;
    double ev = wo - w;
    PH_T0(tc);
    YFlow f = yl_cashflow(c.loan, total, ev, c.y, c.g, c.active, c.S);
    PH_ADD_KS(14, tc, c.g.sl == 0);            // cash flow + NPV + payback
    c.last.total = total;
    c.last.ev = ev;
    c.last.w = w;
    c.last.wo = wo;
    c.last.flow = f;
    return -f.npv;
}

// occupancy floor of 3 waves per SIMD (<= 168 VGPRs): the 32-lane variant
// otherwise takes 181 and runs 2 (measured 23.3 -> 18.6 ms at 1M agents)
// DC: demand charges billed (extension mode) -- a separate instantiation so
// the reference mode's register allocation is untouched.  Both DC builds run
// at 2 waves per SIMD (the two-agent one spills; 78 -> 47 ms for C4 200k vs 1
// wave).  Round 1's wrong two-agent results came from a spill placed ahead of
// a divergent join's exec restore; the build guard
// (dgen_amd/spill_guard.py) rejects any build with that pattern and falls
// back to one agent per wave for the flagged kernel.
// PK (with DC): some tariff bills its tiers in kWh/kW (dgen_tables.peak_units):
// the lanes keep the month peaks, which the demand pass computes ahead of the
// energy bill; a separate instantiation so the other builds' registers are
// untouched.
}  // namespace
namespace dgen_srch {
template <int LPA, bool DC, bool NET, bool PK>
__global__ void __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(DC ? 2 : 3)))
k_size_w(dgen_tables T, dgen_agents A, dgen_outputs O, dgen_cfg cfg, int64_t n, int64_t i0, int64_t i1,
         void* dcws, char* nbws, int pre, double* btrace)
#ifdef DGEN_TU_MAIN
;
#else
{
    const int lane = threadIdx.x;
    const int64_t i = i0 + (int64_t)blockIdx.x * (WAVE / LPA) + (LPA == WAVE ? 0 : lane / LPA);
    if (i >= i1) return;
    PH_T0(t_pro);
    const int half = lds_half(T.max_periods);
    YCtx<LPA> c(lane);
    const int sl = c.g.sl;
    c.y = sl + 1;
    c.S = ylds_make(dyn_lds, half, c.g, PK && T.peak_units != 0, yl_mode<DC, NET>());
    c.tariffs = T.tariffs;
    c.dem_table = T.demand;
    c.n_dem = T.n_demand;
    c.dem = nullptr;
    c.dc_on = cfg.skip_demand_charges == 0;
    c.dem_bill = false;
    c.pk13 = false;
    c.dem_wo_pending = false;
    c.env_ok = false;
    c.env.lines = nullptr;
    c.stg = nullptr;
    c.stg_ok = false;
    c.env_tag = 0;
    c.dc_nq = (T.max_dc_periods > 0 && T.max_dc_periods <= DCP) ? T.max_dc_periods : DCP;
    if constexpr (DC) {
        if (dcws) {
            c.env = dc_env_at(dcws, i);
            c.env_tag = (pre & 1) ? *c.env.tag : 0;       // k_dc_env's, this call
        }
        // the segment's envelope stage sits after the year-lane layout
        c.stg = reinterpret_cast<DcStage*>(reinterpret_cast<char*>(dyn_lds) +
                                           ylds_bytes(half, LPA, PK && T.peak_units != 0, yl_mode<DC, NET>())) + lane / LPA;
    }
    {
        const int slot = A.scratch_slot[i];
        c.nb = (nbws && slot >= 0) ? nbws + (size_t)slot * NB_BYTES : nullptr;
        c.nb_ok = false;
        c.nb_tag = (c.nb && (pre & 2)) ? nbr_tag(c.nb) : 0;  // k_nb_env's, this call
        c.nb_pending = false;
    }
    c.sw_rows = T.switches + A.sw_solar_off[i];
    c.sw_cnt = A.sw_solar_cnt[i];
    c.status = 0;
    c.switched = 0;
    const uint8_t fl = A.flags[i];
    const bool is_res = (fl & 1) != 0, is_ca = (fl & 2) != 0;
    c.N = A.econ_life[i];
    c.active = c.y <= c.N;
    c.kwh = A.load_kwh[i];
    c.capex = A.capex[i];
    c.ccm = A.ccm[i];
    c.yearend = cfg.nm_yearend_sell_rate;
    const int lr = A.load_row[i], cr = A.cf_row[i];
    const int t0 = A.tariff0[i];
    const double naep0 = T.cf_naep[cr];
    c.load_scale = c.kwh / T.shape_sum[lr];
    c.lslots = T.shape_slots + (int64_t)lr * NSLOT;
    c.gslots = T.cf_slots + (int64_t)cr * NSLOT;
    const double rate_base = 1.0 + (A.inflation[i] * 100.0) * 0.01 + (A.escalator[i] * 100.0) * 0.01;
    const double sys_base = 1.0 - (A.pv_deg[i] * 100.0) * 0.01;
    c.r_y = pow_seq(rate_base, c.y - 1);
    c.s_y = pow_seq(sys_base, c.y - 1);
    c.loan = yl_make_loan(A, cfg, i, c.N, is_res, c.y);
    c.src.shape = T.shapes + (int64_t)lr * NH;
    c.src.cf = T.cfs + (int64_t)cr * NH;
    c.src.sysgen = nullptr;
    c.src.sys_stride = 0;
    c.src.load_scale = c.load_scale;
    c.src.gen_scale = 0.0;
    const int wr = A.wholesale_row[i];
    c.ts_row = (!is_ca && wr >= 0 && T.wholesale) ? T.wholesale + (int64_t)wr * NH : nullptr;
    c.src.ts = nullptr;                       // set per tariff (yl_set_tariff)
    c.src.ts_mult = A.price_mult[i];

    bool bad = false;
    if (c.N < 1 || c.N > MAXY || c.N > LPA) { c.status |= DGEN_ST_YEARS; bad = true; }
    if (t0 < 0 || t0 >= T.n_tariffs) { c.status |= DGEN_ST_TARIFF; bad = true; }
    // kWh/kW tier units scale the caps by the month's peak import: the
    // batch's demand machinery supplies it (DC kernels, dgen_tables.peak_units,
    // a record behind `dc`); without it the agent is reported unsized, per
    // agent (DGEN_ST_UNIT), instead of being billed with the wrong caps
    else if ((T.tariffs[t0].flags & DGEN_ST_UNIT) ||
             (peak_unit(T.tariffs[t0]) &&
              !(PK && T.peak_units && tariff_peaks(T.demand, T.n_demand, T.tariffs[t0])))) {
        c.status |= DGEN_ST_UNIT;
        bad = true;
    }
    const double max_load = c.kwh / naep0;                         // ff:440-444
    const double low = max_load * 0.8, high = max_load * 1.25;
    const double span = high - low;
    const double tl = (span > 1.0 ? span : 1.0) * 1e-3;
    const double fl_tl = floor(tl);
    const double xatol = fl_tl < 2.0 ? 2.0 : fl_tl;
    if (!isfinite(low) || !isfinite(high)) { c.status |= DGEN_ST_BOUNDS; bad = true; }
    if (c.kwh == 0.0) c.status |= DGEN_ST_ZERO_LOAD;
    if (bad) {
        if (sl == 0) {
            O.status[i] = c.status;
            O.nfev[i] = 0;
            O.system_kw[i] = NAN; O.x_last[i] = NAN; O.npv[i] = NAN;
            O.payback_raw[i] = NAN; O.payback_period[i] = NAN;
            O.first_with[i] = NAN; O.first_without[i] = NAN; O.price_per_kwh[i] = NAN;
            O.tariff_final[i] = t0; O.switched[i] = 0;
        }
        const int64_t row = i * (MAXY + 1);
        for (int k = sl; k <= MAXY; k += LPA) {
            O.cash_flow[row + k] = NAN; O.cfev_pv[row + k] = NAN;
            O.bill_w_pv[row + k] = NAN; O.bill_wo_pv[row + k] = NAN;
        }
        return;
    }
    {   // generation-scale range the search can evaluate (envelopes, net-billing split)
        const int ln = (c.N >= 1 && c.N <= LPA) ? c.N - 1 : 0;
        const double sN = c.g.bcast(c.s_y, ln);
        const double s_lo = sN < 1.0 ? sN : 1.0, s_hi = sN > 1.0 ? sN : 1.0;
        c.tlo = (((low * 1000.0) * 0.96) / 1000.0) * s_lo;
        c.thi = (((high * 1000.0) * 0.96) / 1000.0) * s_hi;
    }
    PH_ADD_KS(15, t_pro, sl == 0);             // prologue: agent loads, loan, bracket
    PH_T0(t_all);
    yl_set_tariff<LPA, DC, NET, PK>(c, t0);
    int nfev = 0;
    double x_last = 0.0;
    double kw_star = brent_bounded(
        [&](double x) __attribute__((always_inline)) {
            return yl_objective<LPA, DC, NET, PK>(c, x);
        },
        low, high, xatol, &nfev, &x_last, (btrace && sl == 0) ? btrace + i * BT_MAX : nullptr);
    const YLast& l = c.last;
    const YFlow& f = l.flow;
    const double w1 = c.g.bcast(l.w, 0);
    const int64_t row = i * (MAXY + 1);
    if (sl == 0) {
        O.cash_flow[row] = -l.total;
        O.cfev_pv[row] = 0.0;
        O.bill_w_pv[row] = 0.0;
        O.bill_wo_pv[row] = 0.0;
    }
    if (c.active) {
        O.cash_flow[row + c.y] = f.pb;
        O.cfev_pv[row + c.y] = l.ev;
        O.bill_w_pv[row + c.y] = l.w;
        O.bill_wo_pv[row + c.y] = l.wo;
    }
    if (sl == 0) {
        O.npv[i] = f.npv;
        O.payback_raw[i] = f.payback;
        double pb = isfinite(f.payback) ? f.payback : 30.1;
        O.payback_period[i] = rint(pb * 10.0) / 10.0;
        O.first_with[i] = w1;
        O.first_without[i] = c.wo1;
        O.price_per_kwh[i] = c.wo1 / c.kwh;
        O.system_kw[i] = kw_star;
        O.x_last[i] = x_last;
        O.nfev[i] = nfev;
        O.tariff_final[i] = c.tariff;
        O.switched[i] = c.switched;
        O.status[i] = c.status;
    }
    PH_ADD(0, t_all, sl == 0);
    PH_CNT(9, nfev, sl == 0);
}
#endif
}  // namespace dgen_srch
namespace {
using dgen_srch::k_size_w;

// The tariff an agent bills its first Brent evaluation with: scipy's first
// point a + golden_mean (b - a) (brent_bounded) through the solar rate switch
// (yl_objective) -- the initial tariff, or the row the switch lands on, which
// the rest of the narrow bracket almost always keeps.
__device__ __forceinline__ int first_eval_tariff(const dgen_tables& T, const dgen_agents& A, int64_t i,
                                                 double low, double high) {
    const double x = low + 0.3819660112501051 * (high - low);
    int t = A.tariff0[i];
    if (x > 0.0) {
        int nt;
        (void)rate_switch(T.switches + A.sw_solar_off[i], A.sw_solar_cnt[i], x, &nt);
        if (nt >= 0) t = nt;
    }
    return t;
}

// ---------------------------------------------------------------------------
// Demand envelopes of every agent's first-evaluation tariff (first_eval_tariff),
// built ahead of k_size by day lanes (k_dc_env).  The hour-lane build inside
// k_size (yl_dc_build_coop) reads each profile value with its own 4-byte load
// and walks the year twice; at k_size's 256 VGPRs and 2 waves per SIMD those
// walks wait on their loads (C4 200k: build + stage 55 % of k_size's cycles).
// Here one wave takes one agent and two months at a time: lane l of half h
// holds day l of month 2j + h, the day's 24 hours of load shape and cf come
// in as 6 + 6 16-B loads (consecutive lanes read consecutive 96-B days of the
// row), both passes run on those registers, and the reductions over a month's
// days are 32-lane butterflies.  Same rule as yl_dc_build: per (month, demand
// period) A and B are the first maximisers (ties to the earlier hour) of the
// import at tlo and at thi, the lines kept are A, B and every other hour above
// their hull at the crossing less the 1e-10 slack, more than DC_NL lines is an
// overflow (tag < 0: k_size then bills that agent with the hourly pass without
// rebuilding).  An evaluation takes the max over the kept lines, so results do
// not depend on which build ran (the kept set is the same; its order is hour
// order here).  k_size uses the envelopes when its tariff is the tag's.
// ---------------------------------------------------------------------------
constexpr int DCE_WPB = 4;          // agents (one wave each) per block

// (k_dc_env takes cf_per_kw_fast after a per-day range check and leaves an
// agent with a larger value to k_size's build)

// first maximiser over the lane's 32-lane half: larger value, ties to the
// earlier hour
__device__ __forceinline__ void dce_first_max(double& v, int& h) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
        const double ov = __shfl_xor(v, o, WAVE);
        const int oh = __shfl_xor(h, o, WAVE);
        const bool t = (ov > v) | ((ov == v) & (oh < h));    // selects, no branch
        v = t ? ov : v;
        h = t ? oh : h;
    }
}

}  // namespace
namespace dgen_srch {
template <int NQ>
__global__ void __launch_bounds__(WAVE * DCE_WPB) __attribute__((amdgpu_waves_per_eu(NQ <= 4 ? 3 : 2)))
k_dc_env(dgen_tables T, dgen_agents A, dgen_cfg cfg, int64_t i0, int64_t i1, void* dcws)
#ifdef DGEN_TU_MAIN
;
#else
{
    const int lane = threadIdx.x & (WAVE - 1);
    // the wave's agent: wave-uniform (readfirstlane), so its scalars and
    // addresses live in SGPRs
    const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    const int64_t i = i0 + (int64_t)blockIdx.x * DCE_WPB + wid;
    if (i >= i1) return;
    const DcEnv E = dc_env_at(dcws, i);
    const int lr = A.load_row[i], cr = A.cf_row[i];
    const double kwh = A.load_kwh[i];
    const double max_load = kwh / T.cf_naep[cr];                    // ff:440-444, as k_size
    const double low = max_load * 0.8, high = max_load * 1.25;
    const int N = A.econ_life[i];
    const int t0 = (isfinite(low) && isfinite(high)) ? first_eval_tariff(T, A, i, low, high) : -1;
    const dgen_demand* D = nullptr;
    if (t0 >= 0 && t0 < T.n_tariffs && N >= 1 && N <= MAXY) {
        // k_size's record for the tariff (yl_set_tariff): the kWh/kW tier
        // peaks' where the batch bills those (PK kernels), else the charges'
        const dgen_tariff& t = T.tariffs[t0];
        D = (T.peak_units && peak_unit(t)) ? tariff_peaks(T.demand, T.n_demand, t)
                                           : tariff_demand(T.demand, T.n_demand,
                                                           T.peak_units ? cfg.skip_demand_charges == 0 : true, t);
    }
    if (!D) {
        if (lane == 0) *E.tag = 0;
        return;
    }
    const double sys_base = 1.0 - (A.pv_deg[i] * 100.0) * 0.01;
    const double sN = pow_seq(sys_base, N - 1);                    // k_size's s_y of year N
    const double s_lo = sN < 1.0 ? sN : 1.0, s_hi = sN > 1.0 ? sN : 1.0;
    const double tlo = (((low * 1000.0) * 0.96) / 1000.0) * s_lo;
    const double thi = (((high * 1000.0) * 0.96) / 1000.0) * s_hi;
    const double ls = kwh / T.shape_sum[lr];
    const float* const shp = T.shapes + (int64_t)lr * NH;
    const int32_t* const cfp = T.cfs + (int64_t)cr * NH;
    const int nq = (T.max_dc_periods > 0 && T.max_dc_periods <= DCP) ? T.max_dc_periods : DCP;
    const int dl = lane & 31;
    bool ok = true;
#pragma unroll 1
    for (int j = 0; j < 6; j++) {
        const int m = 2 * j + (lane >> 5);
        const int d0 = c_month_start_day[m], d1 = c_month_start_day[m + 1];
        const bool act = d0 + dl < d1;
        const int d = act ? d0 + dl : d1 - 1;                      // idle lanes read a real day
        const uint8_t* sc = ((d % 7) >= 5) ? D->wkend[m] : D->wkday[m];
        float sh[24];
        int32_t cv[24];
        uint32_t pw[6];
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const float4 a = reinterpret_cast<const float4*>(shp + d * 24)[k];
            const int4 b = reinterpret_cast<const int4*>(cfp + d * 24)[k];
            sh[4 * k] = a.x; sh[4 * k + 1] = a.y; sh[4 * k + 2] = a.z; sh[4 * k + 3] = a.w;
            cv[4 * k] = b.x; cv[4 * k + 1] = b.y; cv[4 * k + 2] = b.z; cv[4 * k + 3] = b.w;
            pw[k] = reinterpret_cast<const uint32_t*>(sc)[k];
        }
        bool big = false;
#pragma unroll
        for (int hh = 0; hh < 24; hh++) big = big | (cv[hh] > 20000000) | (cv[hh] < -20000000);
        if (__ballot(big) != 0ull) {           // cf_per_kw's slow path: k_size builds this agent
            if (lane == 0) *E.tag = 0;
            return;
        }
        // periods present in the month (both day types: every month has both)
        uint32_t mask = 0;
#pragma unroll
        for (int hh = 0; hh < 24; hh++) mask |= 1u << ((pw[hh >> 2] >> (8 * (hh & 3))) & 0xffu);
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) mask |= (uint32_t)__shfl_xor((int)mask, o, WAVE);
        // pass 1: per period the lane's first maximisers at tlo / thi, max load
        double av[NQ], bv[NQ], ml[NQ];
        int ah[NQ], bh[NQ];
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            av[q] = -INFINITY; bv[q] = -INFINITY; ml[q] = 0.0;
            ah[q] = 0x7fffffff; bh[q] = 0x7fffffff;
        }
#pragma unroll
        for (int hh = 0; hh < 24; hh++) {
            const int p = (int)((pw[hh >> 2] >> (8 * (hh & 3))) & 0xffu);
            const double L = (double)sh[hh] * ls;
            const double gp = cf_per_kw_fast(cv[hh]);
            const double vlo = L - gp * tlo, vhi = L - gp * thi;
            const int h = d * 24 + hh;
#pragma unroll
            for (int q = 0; q < NQ; q++) {          // selects, no branches
                const bool sel = act & (p == q);
                const bool ua = sel & (vlo > av[q]), ub = sel & (vhi > bv[q]);
                ml[q] = (sel & (L > ml[q])) ? L : ml[q];
                av[q] = ua ? vlo : av[q];
                ah[q] = ua ? h : ah[q];
                bv[q] = ub ? vhi : bv[q];
                bh[q] = ub ? h : bh[q];
            }
        }
        // the month's maximisers, crossings and bounds per period
        double ts[NQ], Ms[NQ];
        int tot[NQ];
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            dce_first_max(av[q], ah[q]);
            dce_first_max(bv[q], bh[q]);
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) {
                const double x = __shfl_xor(ml[q], o, WAVE);
                ml[q] = x > ml[q] ? x : ml[q];
            }
            const bool here = q < nq && ((mask >> q) & 1u) && ah[q] != 0x7fffffff && bh[q] != 0x7fffffff;
            double AL = 0.0, Ag = 0.0, BL = 0.0, Bg = 0.0;
            if (here) {      // the maximisers' (L, g), formed as in pass 1 (the same bits)
                AL = (double)shp[ah[q]] * ls; Ag = cf_per_kw_fast(cfp[ah[q]]);
                BL = (double)shp[bh[q]] * ls; Bg = cf_per_kw_fast(cfp[bh[q]]);
            }
            double t_ = tlo;
            if (Ag > Bg) {
                t_ = (AL - BL) / (Ag - Bg);
                t_ = t_ < tlo ? tlo : (t_ > thi ? thi : t_);
            }
            const double va = AL - Ag * t_, vb = BL - Bg * t_;
            double M_ = va > vb ? va : vb;
            M_ -= 1e-10 * (fabs(AL) + fabs(BL) + 1.0);               // the slack
            ts[q] = t_;
            Ms[q] = here ? M_ : INFINITY;                            // absent: keeps nothing
            tot[q] = 2;
            if (here && dl == q) {
                E.lines[(m * DCP + q) * DC_NL] = make_double2(AL, Ag);
                E.lines[(m * DCP + q) * DC_NL + 1] = make_double2(BL, Bg);
            }
        }
        // pass 2: the other hours above the bound, written in hour order
        uint32_t keep = 0;
        int cnt[NQ];
#pragma unroll
        for (int q = 0; q < NQ; q++) cnt[q] = 0;
#pragma unroll
        for (int hh = 0; hh < 24; hh++) {
            const int p = (int)((pw[hh >> 2] >> (8 * (hh & 3))) & 0xffu);
            const double L = (double)opaque_f(sh[hh]) * ls;   // recomputed, not kept from pass 1
            const double gp = cf_per_kw_fast(opaque_i(cv[hh]));
            const int h = d * 24 + hh;
#pragma unroll
            for (int q = 0; q < NQ; q++) {
                const bool k = act & (p == q) & (h != ah[q]) & (h != bh[q]) & (L - gp * ts[q] > Ms[q]);
                keep |= k ? 1u << hh : 0u;
                cnt[q] += k ? 1 : 0;
            }
        }
        int pos[NQ];
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            int incl = cnt[q];
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) {
                const int t = __shfl_up(incl, o, WAVE);
                if (dl >= o) incl += t;
            }
            pos[q] = 2 + incl - cnt[q];
            tot[q] = 2 + __shfl(incl, (lane & 32) + 31, WAVE);
        }
        // the kept hours (a few per month and period), one at a time from the
        // lane's bit mask; their values re-read from the (cache-hot) rows
        while (keep) {
            const int hh = __builtin_ctz(keep);
            keep &= keep - 1u;
            const int h = d * 24 + hh;
            const int p = (int)sc[hh];
            const double L = (double)shp[h] * ls;
            const double gp = cf_per_kw_fast(cfp[h]);
#pragma unroll
            for (int q = 0; q < NQ; q++) {
                if (p == q) {
                    if (pos[q] < DC_NL) E.lines[(m * DCP + q) * DC_NL + pos[q]] = make_double2(L, gp);
                    pos[q]++;
                }
            }
        }
        // the month's counts and max loads (lane q of the half writes period q)
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const bool here = q < nq && ((mask >> q) & 1u) && Ms[q] != INFINITY;
            if (here && tot[q] > DC_NL) ok = false;
            if (dl == q) {
                E.cnt[m * DCP + q] = here ? (tot[q] < DC_NL ? tot[q] : DC_NL) : 0;
                E.maxl[m * DCP + q] = here ? ml[q] : 0.0;
            }
        }
        if (dl >= NQ && dl < DCP) {            // periods past the batch's: absent
            E.cnt[m * DCP + dl] = 0;
            E.maxl[m * DCP + dl] = 0.0;
        }
    }
    const bool bad = __ballot(!ok) != 0ull;
    if (lane == 0) *E.tag = bad ? -(t0 + 1) : t0 + 1;
}
#endif
}  // namespace dgen_srch
namespace {
using dgen_srch::k_dc_env;

// The PV-only search's net-billing split of every agent's first-evaluation
// tariff (first_eval_tariff), built ahead of k_size on the same stream (yl_nb_build<false> over the same
// range [tlo, thi]; k_size builds only for a tariff the rate switch moves to).
// The build ran at k_size's occupancy with its registers; here it runs alone.
// tag = 1 + the tariff (0: not built -- no slot, not billed net, or invalid).
}  // namespace
namespace dgen_srch {
template <int LPA>
__global__ void __launch_bounds__(WAVE)
k_nb_env(dgen_tables T, dgen_agents A, int64_t i0, int64_t i1, char* nbws)
#ifdef DGEN_TU_MAIN
;
#else
{
    const int lane = threadIdx.x;
    const int64_t i = i0 + (int64_t)blockIdx.x * (WAVE / LPA) + (LPA == WAVE ? 0 : lane / LPA);
    if (i >= i1) return;
    const int slot = A.scratch_slot[i];
    if (slot < 0) return;
    const Seg<LPA> g(lane);
    char* const nbp = nbws + (size_t)slot * NB_BYTES;
    const int lr = A.load_row[i], cr = A.cf_row[i];
    const double kwh = A.load_kwh[i];
    const double max_load = kwh / T.cf_naep[cr];                    // ff:440-444, as k_size
    const double low = max_load * 0.8, high = max_load * 1.25;
    const bool fin = isfinite(low) && isfinite(high);
    const int t0 = fin ? first_eval_tariff(T, A, i, low, high) : -1;
    int tag = 0;
    if (t0 >= 0 && t0 < T.n_tariffs && net_hourly(T.tariffs[t0])) {
        const dgen_tariff& t = T.tariffs[t0];
        const int N = A.econ_life[i];
        if (N >= 1 && N <= MAXY) {
            const double sys_base = 1.0 - (A.pv_deg[i] * 100.0) * 0.01;
            const double sN = pow_seq(sys_base, N - 1);            // k_size's s_y of year N
            const double s_lo = sN < 1.0 ? sN : 1.0, s_hi = sN > 1.0 ? sN : 1.0;
            const double tlo = (((low * 1000.0) * 0.96) / 1000.0) * s_lo;
            const double thi = (((high * 1000.0) * 0.96) / 1000.0) * s_hi;
            const bool is_ca = (A.flags[i] & 2) != 0;
            const int wr = A.wholesale_row[i];
            YSrc src;
            src.shape = T.shapes + (int64_t)lr * NH;
            src.cf = T.cfs + (int64_t)cr * NH;
            src.sysgen = nullptr;
            src.sys_stride = 0;
            src.load_scale = kwh / T.shape_sum[lr];
            src.gen_scale = 0.0;
            src.ts = (t.mo == 2 && !is_ca && wr >= 0 && T.wholesale) ? T.wholesale + (int64_t)wr * NH : nullptr;
            src.ts_mult = A.price_mult[i];
            YLds S;                                   // the build's 4 LDS slots per lane
            S.trf = nullptr;
            S.L = S.G = S.pk = nullptr;
            S.half = 0;
            S.lane = dyn_lds + lane;
            NbStage* const stg = reinterpret_cast<NbStage*>(dyn_lds + 4 * WAVE) + lane / LPA;
            if (yl_nb_build_stg<LPA>(t, src, tlo, thi, nbp, S, g, stg)) tag = t0 + 1;
        }
    }
    if (g.sl == 0) nbr_tag(nbp) = tag;
}
#endif
}  // namespace dgen_srch
namespace {
using dgen_srch::k_nb_env;

// Battery-case Utilityrate5 + Cashloan (ff:178-288), lanes = years.
template <int LPA, bool DC, bool NET, bool PK>
__global__ void __launch_bounds__(WAVE)
k_batt_finance_w(dgen_tables T, dgen_agents A, dgen_outputs O, dgen_cfg cfg, int64_t n, void* ws,
                 int64_t n_scratch, int64_t i0, int64_t i1, char* nbws, int nb_scan, char* dcr, int dc_nq) {
    const int lane = threadIdx.x;
    const int64_t i = i0 + (int64_t)blockIdx.x * (WAVE / LPA) + (LPA == WAVE ? 0 : lane / LPA);
    if (i >= i1) return;
    const int st = O.status[i];
    if (st & (DGEN_ST_BOUNDS | DGEN_ST_TARIFF | DGEN_ST_YEARS | DGEN_ST_SCRATCH | DGEN_ST_UNIT)) return;
    PH_T0(t_all);
    const Seg<LPA> g(lane);
    const int y = g.sl + 1;
    const int half = lds_half(T.max_periods);
    YLds S = ylds_make(dyn_lds, half, g, PK && T.peak_units != 0, yl_mode<DC, NET>());
    WsLayout W = ws_layout(ws, n);
    const bool is_res = (A.flags[i] & 1) != 0;
    const bool is_ca = (A.flags[i] & 2) != 0;
    const int N = A.econ_life[i];
    const bool active = y <= N;
    const dgen_tariff& t = *stage_tariff(T.tariffs + O.tariff_final[i], S, g);
    const double kw = O.system_kw[i];
    const double bank = O.batt_kwh[i];
    const double otc = W.otc_b[i];
    const bool same_tariff = W.aux[i] == 0.0;    // no storage switch: k_size's wo1 applies
    const double rate_base = 1.0 + (A.inflation[i] * 100.0) * 0.01 + (A.escalator[i] * 100.0) * 0.01;
    const double sys_base = 1.0 - (A.pv_deg[i] * 100.0) * 0.01;
    const double r_y = pow_seq(rate_base, y - 1), s_y = pow_seq(sys_base, y - 1);
    const YLoan L = yl_make_loan(A, cfg, i, N, is_res, y);
    double system_costs = (kw > 0.0) ? A.capex_combined[i] * kw : A.capex[i] * kw;   // ff:203-216
    double batt_costs = A.batt_capex_kwh[i] * bank * 0.7;                           // ff:219
    double total = ((system_costs + batt_costs) * A.ccm[i]) + 0.0 + otc;
    const double vor = A.vor[i];
    const bool mo2 = net_hourly(t);
    // demand record: its charges (extension mode), or the month peaks the
    // kWh/kW tiers scale with (pk13: that pass runs ahead of the energy bills)
    const dgen_demand* bill_dem = DC ? tariff_demand(T, cfg, t) : nullptr;
    const bool pk13 = PK && peak_unit(t) && S.pk != nullptr && tariff_peaks(T.demand, T.n_demand, t);
    const dgen_demand* dem = pk13 ? tariff_peaks(T.demand, T.n_demand, t) : bill_dem;
    // the segment's LDS stage of the staged demand pass sits after the year-lane layout
    DemStage* const stage = reinterpret_cast<DemStage*>(reinterpret_cast<char*>(dyn_lds) +
                                                        ylds_bytes(half, LPA, S.pk != nullptr, yl_mode<DC, NET>())) + (lane / LPA);
    YSrc src;
    {
        const int lr = A.load_row[i];
        src.shape = T.shapes + (int64_t)lr * NH;
        src.cf = nullptr;
        src.load_scale = A.load_kwh[i] / T.shape_sum[lr];
        src.gen_scale = 0.0;
        src.sys_stride = n_scratch;
        const int slot = A.scratch_slot[i];
        src.sysgen = (slot >= 0) ? W.scratch + (int64_t)slot * 24 : nullptr;   // day tiles (sys_index)
        const int wr = A.wholesale_row[i];
        src.ts = (t.mo == 2 && !is_ca && wr >= 0 && T.wholesale) ? T.wholesale + (int64_t)wr * NH : nullptr;
        src.ts_mult = A.price_mult[i];
    }
    // the battery-case demand record this step's k_hourly_batt built (flag 1),
    // else the staged pass over the system-output plane
    DcrRec drec{nullptr, nullptr, nullptr, nullptr, nullptr};
    bool dr = false;
    if (DC && dcr && A.scratch_slot[i] >= 0) {
        drec = dcr_rec(dcr, A.scratch_slot[i]);
        dr = *drec.flag == 1;
    }
    double wo1 = NAN, wb = NAN;
    // kWh/kW tiers: the no-system month peaks ahead of the no-system bill (k_size's
    // first_without already holds it for the same tariff), the battery case's
    // ahead of its bill
    double v0 = 0.0, v1 = 0.0;
    if (pk13 && !same_tariff) v0 = yl_demand_staged(dem, src, 1.0, false, S, stage, g, dr, drec, dc_nq);
    if (!mo2) {
        const double2* lg = W.LGb + (int64_t)i * NBIN;
        for (int cell = g.sl; cell < 12 * t.P; cell += LPA) {
            int m = cell / t.P, p = cell % t.P;
            const double2 b = lg[cell];
            S.L[m * half + p] = b.x;
            S.G[m * half + p] = b.y;
        }
        wave_lds_sync();
        wo1 = same_tariff ? O.first_without[i] : yl_bill_nem_nosys(t, S, cfg.nm_yearend_sell_rate, g);
        if (pk13) v1 = yl_demand_staged(dem, src, s_y, true, S, stage, g, dr, drec, dc_nq);
        wb = yl_bill_nem(t, S, s_y, cfg.nm_yearend_sell_rate);
    } else if constexpr (NET) {
        if (same_tariff) {
            wo1 = O.first_without[i];
        } else {   // k_size's no-system form: the slot-sum load bins
            const int lr = A.load_row[i], cr = A.cf_row[i];
            yl_build_bins(t, T.shape_slots + (int64_t)lr * NSLOT, T.cf_slots + (int64_t)cr * NSLOT,
                          src.load_scale, S, g);
            wo1 = yl_bill_mo2_nogen_par(t, S, g);
        }
        if (pk13) v1 = yl_demand_staged(dem, src, s_y, true, S, stage, g, dr, drec, dc_nq);
        // the split of the battery-case hours over the lanes' degradation
        // factors [s_lo, s_hi] (the agent's net-billing record is free: its
        // search finished in k_size)
        const int slot = A.scratch_slot[i];
        bool nb_ok = false;
        if (nbws && slot >= 0 && src.sysgen) {
            const int ln = (N >= 1 && N <= LPA) ? N - 1 : 0;
            const double sN = g.bcast(s_y, ln);
            const double s_lo = sN < 1.0 ? sN : 1.0, s_hi = sN > 1.0 ? sN : 1.0;
            src.gen_scale = 1.0;
            char* nbp = nbws + (size_t)slot * NB_BYTES;
            PH_T0(tb);
            // this step's k_hourly_batt built it in its scan: compact entries
            // (flag 1) or, for a TS sell rate, full 24-B entries (flag 4)
            const int nb_fl = nbr_flag(nbp);
            const bool scan_rec = nb_scan && (nb_fl == 1 || nb_fl == 4);
            if (scan_rec) {
                const NbRec R = nb_rec(nbp);
                nb_ok = g.first(g.sl < 12 && R.cnt[g.sl] > NB_CAPM) < 0;
            } else {
                nb_ok = yl_nb_build<true>(t, src, s_lo, s_hi, nbp, S, g);
            }
            PH_ADD(5, tb, g.sl == 0);
            PH_T0(te);
            if (nb_ok) wb = yl_bill_nb(t, src, s_y, nbp, S, g, scan_rec && nb_fl == 1);
            PH_ADD(6, te, g.sl == 0);
        }
        if (!nb_ok) wb = yl_bill_net(t, src, s_y, true, S);
    }
    if (pk13) {
        if (bill_dem) {
            wb += v1;
            if (!same_tariff) wo1 += v0;
        }
    } else if (DC && dem) {   // k_size's first_without already carries the no-system demand charge
        PH_T0(tds);
        for (int pass = same_tariff ? 1 : 0; pass < 2; pass++) {
            const bool wg = pass == 1;
            const double v = yl_demand_staged(dem, src, wg ? s_y : 1.0, wg, S, stage, g, dr, drec, dc_nq);
            if (wg) wb += v;
            else wo1 += v;
        }
        PH_ADD(5, tds, g.sl == 0);                // battery-case staged demand pass
    }
    double w = wb * r_y;
    double wo = wo1 * r_y;
    double ev = (wo - w) + vor;                                    // ff:275
    YFlow f = yl_cashflow(L, total, ev, y, g, active, S);
    const int64_t row = i * (MAXY + 1);
    if (g.sl == 0) {
        O.cfev_batt[row] = 0.0;
        O.bill_w_batt[row] = 0.0;
        O.bill_wo_batt[row] = 0.0;
        O.npv_pv_batt[i] = f.npv;
    }
    if (active) {
        O.cfev_batt[row + y] = ev;
        O.bill_w_batt[row + y] = w;
        O.bill_wo_batt[row + y] = wo;
    }
    PH_ADD(4, t_all, g.sl == 0);
}

// ---------------------------------------------------------------------------
// Brent self-test kernel (closed-form objective; tests the search alone)
// ---------------------------------------------------------------------------
__global__ void k_brent_selftest(const double* lo, const double* hi, const double* xatol,
                                 const double* c2, const double* x0, const double* c1, int64_t n,
                                 double* xs, int maxn, double* xopt, int32_t* nfev) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int k = 0;
    double a2 = c2[i], b0 = x0[i], a1 = c1[i];
    double* rec = xs + i * maxn;
    int nf = 0;
    double xl = 0.0;
    double xo = brent_bounded(
        [&](double x) __attribute__((always_inline)) {
            if (k < maxn) rec[k] = x;
            k++;
            double d = x - b0;
            return a2 * d * d + a1 * x;
        },
        lo[i], hi[i], xatol[i], &nf, &xl);
    xopt[i] = xo;
    nfev[i] = nf;
}

// ---------------------------------------------------------------------------
// k_segment_sums: one 256-thread block per (segment, plane)
// ---------------------------------------------------------------------------
template <typename V>
__global__ void __launch_bounds__(256)
k_segment_sums(const V* __restrict__ v1, const double* __restrict__ w1, const V* __restrict__ v2,
               const double* __restrict__ w2, int k, int64_t n, const int64_t* __restrict__ seg_off,
               int64_t n_seg, double* __restrict__ out) {
    __shared__ double red[256];
    const int64_t s = blockIdx.x;
    const int j = blockIdx.y;
    if (s >= n_seg || j >= k) return;
    const int64_t lo = seg_off[s], hi = seg_off[s + 1];
    const V* p1 = v1 + (int64_t)j * n;
    const V* p2 = v2 ? v2 + (int64_t)j * n : nullptr;
    double acc = 0.0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
        double t = (double)p1[i] * (w1 ? w1[i] : 1.0);
        if (p2) t += (double)p2[i] * w2[i];
        acc += t;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[s * k + j] = red[0];
}


// Rows of each segment summed in row order: out[s][j] = ((in[r0][j] + in[r0+1][j])
// + ...) for the rows r of [seg_off[s], seg_off[s+1]).  The model-year loop's
// per-state rows are sums of per-chunk partials (fixed 8192-agent chunks of
// each state's members, dgen_amd/partition.py) taken in chunk order, so a
// state whose chunks sit on several ranks sums to the same bits as on one.
__global__ void k_rows_seq_sum(const double* __restrict__ in, int64_t k, const int64_t* __restrict__ seg_off,
                               int64_t n_seg, double* __restrict__ out) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t s = blockIdx.y;
    if (j >= k || s >= n_seg) return;
    double acc = 0.0;
    for (int64_t r = seg_off[s]; r < seg_off[s + 1]; r++) acc += in[r * k + j];
    out[s * k + j] = acc;
}

// ---------------------------------------------------------------------------
// Diffusion step, thread per agent
// ---------------------------------------------------------------------------
__device__ __forceinline__ double np_maximum(double a, double b) {   // propagates NaN
    if (a != a || b != b) return NAN;
    return a > b ? a : b;
}

// financial_functions.calc_max_market_share (ff:1264-1310): clip payback to the
// curve's range (NaN -> min, pandas Series.where), round to 0.1 (half-even),
// factor = round(100 x), left-merge on (sector, factor).
__global__ void k_max_market_share(dgen_mms_table tb, const double* __restrict__ payback,
                                   const int32_t* __restrict__ row, int64_t n,
                                   double* __restrict__ bounded, int64_t* __restrict__ factor,
                                   double* __restrict__ mms) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double pb = payback[i];
    if (!(pb >= tb.min_pb)) pb = tb.min_pb;
    if (!(pb <= tb.max_pb)) pb = tb.max_pb;
    double r1 = rint(pb * 10.0) / 10.0;
    double fac = rint(r1 * 100.0);
    bounded[i] = r1;
    int64_t fi = (int64_t)fac;
    factor[i] = fi;
    int r = row[i];
    int64_t k = fi - tb.factor_min;
    double v = NAN;
    if (r >= 0 && r < tb.n_rows && k >= 0 && k < tb.n_factors) v = tb.mms[(int64_t)r * tb.n_factors + k];
    mms[i] = v;
}

// calc_equiv_time -> calc_diffusion_market_share -> bass_diffusion -> the
// market-share floor / cap and cumulative updates of calc_diffusion_solar.
__global__ void k_diffusion(dgen_diffusion_in in, dgen_diffusion_out out, int64_t n, int first) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double mms = in.max_market_share[i];
    const double msly = in.market_share_last_year[i];
    const double p = in.bass_p[i], q = in.bass_q[i];
    const double mfix = (mms == 0.0) ? 1e-9 : mms;
    const double ratio = (msly > mfix) ? 0.0 : msly / mfix;
    const double teq = log((1.0 - ratio) / (1.0 + ratio * (q / p))) / (-1.0 * (p + q));
    const double teq2 = first ? teq + in.teq_yr1[i] : teq + 2.0;
    const double f = pow(M_E, -1.0 * (p + q) * teq2);               // np.e ** (...)
    const double naf = (1.0 - f) / (1.0 + (q / p) * f);
    const double bms = mms * naf;
    const double dms = (msly > bms) ? msly : bms;
    const double ms = np_maximum(dms, msly);
    double nms = ms - msly;
    if (ms > mms) nms = 0.0;
    const double na = nms * in.developable_agent_weight[i];
    const double skw = in.system_kw[i];
    const double nmv = (na * skw) * in.system_capex_per_kw[i];
    const double nskw = na * skw;
    out.mms_fix_zeros[i] = mfix;
    out.ratio[i] = ratio;
    out.bass_params_teq[i] = teq;
    out.teq2[i] = teq2;
    out.f[i] = f;
    out.new_adopt_fraction[i] = naf;
    out.bass_market_share[i] = bms;
    out.diffusion_market_share[i] = dms;
    out.market_share[i] = ms;
    out.new_market_share[i] = nms;
    out.new_adopters[i] = na;
    out.new_market_value[i] = nmv;
    out.new_system_kw[i] = nskw;
    out.number_of_adopters[i] = in.adopters_cum_last_year[i] + na;
    out.market_value[i] = in.market_value_last_year[i] + nmv;
    out.system_kw_cum[i] = in.system_kw_cum_last_year[i] + nskw;
}

// ---------------------------------------------------------------------------
// Battery attachment: attachment_rate_functions.py:58-138
// largest-remainder integer battery adopters per (state, sector) group, and
// the per-state hourly export weights / sums (:141-206).
// ---------------------------------------------------------------------------
constexpr int ATT_BLOCK = 256;

struct NewVal {
    const double* p;
    __device__ double operator()(int i) const { return p[i]; }
};

// Block-wide int64 sum (every thread gets the total).
__device__ __forceinline__ int64_t block_sum_i64(int64_t v, int64_t* red) {
    const int t = threadIdx.x;
    red[t] = v;
    __syncthreads();
    for (int w = ATT_BLOCK / 2; w > 0; w >>= 1) {
        if (t < w) red[t] += red[t + w];
        __syncthreads();
    }
    const int64_t r = red[0];
    __syncthreads();
    return r;
}

// One radix-select pass: histogram of digit (key >> shift) & 0xff over the
// group's candidates (key & mask) == prefix, then the digit holding the k-th
// key in the requested direction.  Updates prefix / mask / k (k-th among the
// candidates left with that digit).  Keys come from key_of(i).
template <class K>
__device__ void radix_pass(const K& key_of, int64_t lo, int64_t hi, int shift, bool descending,
                           uint64_t& prefix, uint64_t& mask, int64_t& k, uint32_t* hist,
                           int64_t* sel) {
    const int t = threadIdx.x;
    hist[t] = 0;
    __syncthreads();
    for (int64_t i = lo + t; i < hi; i += ATT_BLOCK) {
        const uint64_t key = key_of(i);
        if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 0xffu], 1u);
    }
    __syncthreads();
    if (t == 0) {
        int64_t cum = 0;
        int d = descending ? 255 : 0;
        for (int s = 0; s < 256; s++, d += descending ? -1 : 1) {
            const int64_t c = hist[d];
            if (cum + c >= k) break;
            cum += c;
        }
        sel[0] = d;
        sel[1] = cum;
    }
    __syncthreads();
    const uint64_t d = (uint64_t)sel[0];
    k -= sel[1];
    prefix |= d << shift;
    mask |= (uint64_t)0xff << shift;
    __syncthreads();
}

// One block per group (agents [seg_off[g], seg_off[g+1]) in the reference's
// row order).  rate: per group.  aid_rank: rank of str(agent_id) (the
// reference's tie-break sorts agent ids as strings, :125-128).
__global__ void __launch_bounds__(ATT_BLOCK)
k_batt_attach(dgen_attach_in in, dgen_attach_out out, const int64_t* __restrict__ seg_off,
              const double* __restrict__ rate, int64_t n_seg) {
    __shared__ uint32_t hist[256];
    __shared__ int64_t red[ATT_BLOCK];
    __shared__ int64_t sel[2];
    __shared__ double tot;
    const int64_t g = blockIdx.x;
    if (g >= n_seg) return;
    const int64_t lo = seg_off[g], hi = seg_off[g + 1];
    const int t = threadIdx.x;
    double r = rate[g];
    r = fmax(0.0, fmin(1.0, r));                                   // :109
    if (t == 0) tot = np_sum(NewVal{in.new_adopters + lo}, (int)(hi - lo));   // n.sum()
    __syncthreads();
    const double S = tot;
    const bool active = (hi > lo) && !(S <= 0.0 || r <= 0.0);      // :112
    int64_t rem = 0;
    if (active) {
        const int64_t target = (int64_t)rint(r * S);               // :116 round half even
        int64_t bsum = 0;
        for (int64_t i = lo + t; i < hi; i += ATT_BLOCK) bsum += (int64_t)floor(r * in.new_adopters[i]);
        rem = target - block_sum_i64(bsum, red);                   // :121
    }
    // winners: frac desc, agent id (string) asc; threshold (T1, T2) by radix select
    uint64_t p1 = 0, m1 = 0, p2 = 0, m2 = 0;
    int64_t k1 = 0;
    const bool pick = active && rem > 0;
    const bool all = pick && rem >= hi - lo;
    if (pick && !all) {
        auto fkey = [&](int64_t i) -> uint64_t {
            const double f = r * in.new_adopters[i];
            const double fr = f - (double)(int64_t)floor(f);
            return (uint64_t)__double_as_longlong(fr);             // fr >= 0: bits are monotone
        };
        k1 = rem;
        for (int sh = 56; sh >= 0; sh -= 8) radix_pass(fkey, lo, hi, sh, true, p1, m1, k1, hist, sel);
        // k1 = winners still needed among frac == T1: smallest string ranks
        auto rkey = [&](int64_t i) -> uint64_t {
            return fkey(i) == p1 ? (uint64_t)in.aid_rank[i] : ~(uint64_t)0;
        };
        int64_t k2 = k1;
        for (int sh = 56; sh >= 0; sh -= 8) radix_pass(rkey, lo, hi, sh, false, p2, m2, k2, hist, sel);
    }
    for (int64_t i = lo + t; i < hi; i += ATT_BLOCK) {
        int64_t a = 0;
        if (active) {
            const double f = r * in.new_adopters[i];
            a = (int64_t)floor(f);
            if (all) {
                a += 1;
            } else if (pick) {
                const uint64_t key = (uint64_t)__double_as_longlong(f - (double)a);
                if (key > p1 || (key == p1 && (uint64_t)in.aid_rank[i] <= p2)) a += 1;
            }
        }
        const double nkw = (double)a * in.batt_kw[i];               // :133-136
        const double nkwh = (double)a * in.batt_kwh[i];
        out.added[i] = a;
        out.new_batt_kw[i] = nkw;
        out.new_batt_kwh[i] = nkwh;
        out.batt_kw_cum[i] = in.batt_kw_cum_last_year[i] + nkw;
        out.batt_kwh_cum[i] = in.batt_kwh_cum_last_year[i] + nkwh;
    }
}

// Per-agent multipliers of the per-state export (:181-190):
// w_pvo = pvo_cum, w_batt = batt_cum, w_non = max(n_cust - n_adopt, 0).
__global__ void k_export_weights(const double* __restrict__ customers, const double* __restrict__ adopters,
                                 const double* __restrict__ bkw_cum_ly, const double* __restrict__ bkw,
                                 const int64_t* __restrict__ added, int64_t n, double* __restrict__ w_pvo,
                                 double* __restrict__ w_batt, double* __restrict__ w_non) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double eps = 1e-9;
    const double n_cust = customers[i], n_adopt = adopters[i];
    const double b = bkw[i];
    const double den = fmax(b != 0.0 ? b : eps, eps);              // max(float(x) or eps, eps)
    const double prev = rint(fmax(bkw_cum_ly[i] / den, 0.0));      // int(round(max(., 0)))
    double bc = prev + (double)added[i];
    bc = bc > 0.0 ? bc : 0.0;
    double pc = rint(n_adopt) - bc;
    pc = pc > 0.0 ? pc : 0.0;
    w_pvo[i] = pc;
    w_batt[i] = bc;
    const double nn = n_cust - n_adopt;
    w_non[i] = 0.0 > nn ? 0.0 : nn;                                // Python max(nn, 0.0): NaN stays
}

// Per-state hourly net sums from the three hourly planes:
//   out[s * nh + h] = (sum_i pvo*w_pvo + wbt*w_batt + base*w_non) / 1000  (MW)
// f32 planes are dgen_size_agents' outputs in place, in its hour-quad tiles
// ((h, i) at ((h / 4) * n + i) * 4 + h % 4: one 16-B load per agent and 4
// hours); f64 planes are plain [h][n].  Members of state s are
// idx[seg_off[s] .. seg_off[s+1]) (idx null: the plane columns themselves,
// states contiguous).  Block per (state, tile of SH_TILE hours): the three
// weights and the column index of an agent are read once per tile (32 B per
// 32 hours against 384 B of planes).  The plane reads are coalesced only when
// a state's columns are a contiguous ascending range (the year loop's
// state-major device order); a scattered idx fetches a 128-B line per 16-B
// quad.  Fixed reduction order.
// COMB: `base` is k_hourly_batt<XP>'s combined plane (f64 tiles; pvo / wbt /
// weights unused): each agent-hour adds the value the three-plane form adds.
constexpr int SH_TILE = 32;
template <typename V, bool TILED, bool COMB = false>
__global__ void __launch_bounds__(256)
k_state_hourly(const V* __restrict__ base, const V* __restrict__ pvo,
               const V* __restrict__ wbt, const double* __restrict__ w_pvo,
               const double* __restrict__ w_batt, const double* __restrict__ w_non,
               const int64_t* __restrict__ idx, int64_t n, int nh,
               const int64_t* __restrict__ seg_off, int64_t n_seg, double* __restrict__ out) {
    __shared__ double red[4][SH_TILE];
    const int64_t s = blockIdx.x;
    const int h0 = blockIdx.y * SH_TILE;
    if (s >= n_seg || h0 >= nh) return;
    const int nt = nh - h0 < SH_TILE ? nh - h0 : SH_TILE;
    const int64_t lo = seg_off[s], hi = seg_off[s + 1];
    double acc[SH_TILE];
#pragma unroll
    for (int t = 0; t < SH_TILE; t++) acc[t] = 0.0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
        const int64_t c = idx ? idx[i] : i;
        if constexpr (COMB) {
#pragma unroll
            for (int q = 0; q < SH_TILE / 4; q++) {
                if (4 * q < nt) {
                    const int64_t r = (((int64_t)(h0 >> 2) + q) * n + c) * 4;
                    const double2 x0 = *reinterpret_cast<const double2*>(base + r);
                    const double2 x1 = *reinterpret_cast<const double2*>(base + r + 2);
                    acc[4 * q] += x0.x;
                    acc[4 * q + 1] += x0.y;
                    acc[4 * q + 2] += x1.x;
                    acc[4 * q + 3] += x1.y;
                }
            }
            continue;
        }
        const double a = w_pvo[c], b = w_batt[c], d = w_non[c];
        if constexpr (TILED) {
            // nh % 4 == 0 (host), h0 % 4 == 0: whole quads
#pragma unroll
            for (int q = 0; q < SH_TILE / 4; q++) {
                if (4 * q < nt) {
                    const int64_t r = (((int64_t)(h0 >> 2) + q) * n + c) * 4;
                    double vp[4], vw[4], vb[4];
                    if constexpr (sizeof(V) == 4) {
                        const f32x4 xp = *reinterpret_cast<const f32x4*>(pvo + r);
                        const f32x4 xw = *reinterpret_cast<const f32x4*>(wbt + r);
                        const f32x4 xb = *reinterpret_cast<const f32x4*>(base + r);
#pragma unroll
                        for (int u = 0; u < 4; u++) { vp[u] = xp[u]; vw[u] = xw[u]; vb[u] = xb[u]; }
                    } else {
#pragma unroll
                        for (int u = 0; u < 4; u += 2) {
                            const double2 xp = *reinterpret_cast<const double2*>(pvo + r + u);
                            const double2 xw = *reinterpret_cast<const double2*>(wbt + r + u);
                            const double2 xb = *reinterpret_cast<const double2*>(base + r + u);
                            vp[u] = xp.x; vp[u + 1] = xp.y; vw[u] = xw.x; vw[u + 1] = xw.y;
                            vb[u] = xb.x; vb[u + 1] = xb.y;
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        acc[4 * q + u] += (vp[u] * a + vw[u] * b) + vb[u] * d;
                }
            }
        } else {
            const int64_t o = (int64_t)h0 * n + c;
#pragma unroll
            for (int t = 0; t < SH_TILE; t++) {
                if (t < nt) {
                    const int64_t r = o + (int64_t)t * n;
                    acc[t] += ((double)pvo[r] * a + (double)wbt[r] * b) + (double)base[r] * d;
                }
            }
        }
    }
    // butterfly within each wave (static acc indices: no scratch), then the
    // four wave partials in wave order
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int t = 0; t < SH_TILE; t++) {
        double v = acc[t];
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
        if (lane == 0) red[wv][t] = v;
    }
    __syncthreads();
    if (threadIdx.x < nt)
        out[s * nh + h0 + threadIdx.x] =
            (((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x]) / 1000.0;
}

// Per-state hourly export from the with-battery plane alone (the model-year
// loop's form: dgen_size_agents with only the with-battery plane, WO): the
// load and PV-only net load of agent-hour (i, h) are recomputed from the
// profile rows exactly as k_hourly_batt forms them -- ld = shape x ls, pl = cf
// x cl6, the float32 roundings of ld and max(ld - pl, 0) -- so every term, and
// the sums (k_state_hourly's tiled order), are the three-plane form's, bit for
// bit, from 4 B of plane per agent-hour instead of 12 (or a re-run scan).
// Per agent once per call: the two scalars every hour tile of the agent
// needs (ls, cl6), so the tiles read one 16-B record instead of the
// load_row -> shape_sum chain, status, x_last and three divisions each.
__global__ void k_state_rows_prep(dgen_tables T, dgen_agents A, dgen_outputs O, int64_t n,
                                  double2* __restrict__ scal) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const int lr = A.load_row[c];
    const double ls = A.load_kwh[c] / T.shape_sum[lr];
    const bool unsized = (O.status[c] & DGEN_ST_UNIT) != 0;
    const double x_last = unsized ? 0.0 : O.x_last[c];
    const double cl6 = (((x_last * 1000.0) * 0.96) / 1000.0) / 1e6;
    scal[c] = make_double2(ls, cl6);
}

__global__ void __launch_bounds__(256)
k_state_hourly_rows(dgen_tables T, dgen_agents A, const double2* __restrict__ scal, const float* __restrict__ wbt,
                    const double* __restrict__ w_pvo, const double* __restrict__ w_batt,
                    const double* __restrict__ w_non, const int64_t* __restrict__ idx, int64_t n,
                    const int64_t* __restrict__ seg_off, int64_t n_seg, double* __restrict__ out) {
    __shared__ double red[4][SH_TILE];
    const int64_t s = blockIdx.x;
    const int h0 = blockIdx.y * SH_TILE;
    if (s >= n_seg || h0 >= NH) return;
    const int nt = NH - h0 < SH_TILE ? NH - h0 : SH_TILE;
    const int64_t lo = seg_off[s], hi = seg_off[s + 1];
    double acc[SH_TILE];
#pragma unroll
    for (int t = 0; t < SH_TILE; t++) acc[t] = 0.0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
        const int64_t c = idx ? idx[i] : i;
        const double a = w_pvo[c], b = w_batt[c], d = w_non[c];
        const int lr = A.load_row[c], cr = A.cf_row[c];
        const double2 sc = scal[c];
        const double ls = sc.x, cl6 = sc.y;                          // k_state_rows_prep
        const float* shp = T.shapes + (int64_t)lr * NH + h0;
        const int32_t* cfp = T.cfs + (int64_t)cr * NH + h0;
#pragma unroll
        for (int q = 0; q < SH_TILE / 4; q++) {
            if (4 * q < nt) {
                const int64_t r = (((int64_t)(h0 >> 2) + q) * n + c) * 4;
                const f32x4 xw = *reinterpret_cast<const f32x4*>(wbt + r);
                const float4 sv = reinterpret_cast<const float4*>(shp)[q];
                const int4 cv = reinterpret_cast<const int4*>(cfp)[q];
                const float sh4[4] = {sv.x, sv.y, sv.z, sv.w};
                const int32_t cf4[4] = {cv.x, cv.y, cv.z, cv.w};
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const double ld = (double)sh4[u] * ls;
                    const double pl = (double)cf4[u] * cl6;
                    const double vb = (double)(float)ld;
                    const double vp = (double)(float)fmax(ld - pl, 0.0);
                    const double vw = (double)xw[u];
                    acc[4 * q + u] += (vp * a + vw * b) + vb * d;
                }
            }
        }
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int t = 0; t < SH_TILE; t++) {
        double v = acc[t];
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
        if (lane == 0) red[wv][t] = v;
    }
    __syncthreads();
    if (threadIdx.x < nt)
        out[s * NH + h0 + threadIdx.x] =
            (((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x]) / 1000.0;
}

// ---------------------------------------------------------------------------
// Per-year agent attributes: the elec.apply_* left merges as
// gathers from host-compiled per-year tables (include/dgen_hip.h
// dgen_year_inputs); thread per agent.  apply_load_growth (elec.py:398-411):
// residential agents scale their per-customer load, the others their
// customer count; every agent its load in bin.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double yt_get(const double* tab, int64_t n_rows, int ncol, int32_t k, int c) {
    return (k >= 0 && k < n_rows) ? tab[(int64_t)k * ncol + c] : NAN;
}
__device__ __forceinline__ int32_t yt_int(double v) {   // NaN (merge miss) -> -1
    return (v == v) ? (int32_t)v : -1;
}

__global__ void k_year_inputs(dgen_year_keys K, dgen_year_tables T, dgen_year_out O, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t ks = K.k_sector[i], kc = K.k_sector_county[i], kt = K.k_state_sector[i];
    auto S = [&](int c) { return yt_get(T.by_sector, T.n_sector, DGEN_YS_COLS, ks, c); };
    auto C = [&](int c) { return yt_get(T.by_sector_county, T.n_sector_county, DGEN_YC_COLS, kc, c); };
    const double mult = C(DGEN_YC_LOAD_MULT);
    const bool res = K.is_res[i] != 0;
    const double l0 = K.load_kwh_initial[i], c0 = K.customers_initial[i];
    O.load_kwh[i] = res ? l0 * mult : l0;
    O.customers_in_bin[i] = res ? c0 : c0 * mult;
    O.load_kwh_in_bin[i] = K.load_in_bin_initial[i] * mult;
    O.price_mult[i] = C(DGEN_YC_PRICE_MULT);
    O.escalator[i] = C(DGEN_YC_ESCALATOR);
    O.inflation[i] = T.inflation_rate;
    O.capex[i] = S(DGEN_YS_CAPEX);
    O.capex_combined[i] = S(DGEN_YS_CAPEX_COMBINED);
    O.batt_capex_kwh[i] = S(DGEN_YS_BATT_CAPEX_KWH);
    O.pv_deg[i] = S(DGEN_YS_PV_DEG);
    O.itc_frac[i] = S(DGEN_YS_ITC);
    O.econ_life[i] = yt_int(S(DGEN_YS_ECON_LIFE));
    O.loan_term[i] = yt_int(S(DGEN_YS_LOAN_TERM));
    O.down_payment[i] = S(DGEN_YS_DOWN_PAYMENT);
    O.real_discount[i] = S(DGEN_YS_REAL_DISCOUNT);
    O.tax_rate[i] = S(DGEN_YS_TAX_RATE);
    O.vor[i] = yt_get(T.by_state_sector, T.n_state_sector, 1, kt, 0);
    if (O.wholesale_row) {
        const int32_t kk = K.k_county[i];
        O.wholesale_row[i] = (T.wholesale_row && kk >= 0 && kk < T.n_county) ? T.wholesale_row[kk] : -1;
    }
}

// ---------------------------------------------------------------------------
// First-year market seeding (elec.estimate_initial_market_shares,
// elec.py:701-765).  Block per (state, sector, tech) group: lane 0 runs
// pandas' group_sum over the group's rows in frame order (Kahan-compensated,
// NaN skipped and not counted, a NaN compensation reset to 0 -- pandas
// _libs/groupby.pyx group_sum), then the block writes every member's columns.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_initial_shares(dgen_init_in in, dgen_init_out out, const int64_t* __restrict__ idx,
                 const int64_t* __restrict__ seg_off, const double* __restrict__ caps, int64_t n_seg) {
    __shared__ double s_sum;
    __shared__ int64_t s_cnt;
    const int64_t g = blockIdx.x;
    if (g >= n_seg) return;
    const int64_t lo = seg_off[g], hi = seg_off[g + 1];
    if (threadIdx.x == 0) {
        double sum = 0.0, comp = 0.0;
        int64_t cnt = 0;
        for (int64_t r = lo; r < hi; r++) {
            const double v = in.developable_agent_weight[idx[r]];
            if (v != v) continue;
            cnt++;
            const double y = v - comp;
            const double t = sum + y;
            comp = (t - sum) - y;
            if (comp != comp) comp = 0.0;
            sum = t;
        }
        s_sum = sum;
        s_cnt = cnt;
        out.developable_customers_in_state[g] = sum;
        out.agent_count[g] = cnt;
    }
    __syncthreads();
    const double dev = s_sum;
    const double cntd = (double)s_cnt;
    const double* cp = caps + g * 5;
    const double sys_mw = cp[0], batt_mw = cp[1], batt_mwh = cp[2], pv_n = cp[3], batt_n = cp[4];
    auto z = [](double v) { return (v == v) ? v : 0.0; };    // fillna(0)
    for (int64_t r = lo + threadIdx.x; r < hi; r += blockDim.x) {
        const int64_t i = idx[r];
        const double w = in.developable_agent_weight[i];
        const double portion = (dev > 0.0) ? w / dev : 1.0 / cntd;
        const double adopt = portion * pv_n;
        const double skc = (portion * sys_mw) * 1000.;
        const double bkw = (portion * batt_mw) * 1000.0;
        const double bkwh = (portion * batt_mwh) * 1000.0;
        const double ms = (w == 0.0) ? 0.0 : adopt / w;
        const double mv = in.system_capex_per_kw[i] * skc;
        out.adopters_cum_last_year[i] = z(adopt);
        out.system_kw_cum_last_year[i] = z(skc);
        out.batt_kw_cum_last_year[i] = z(bkw);
        out.batt_kwh_cum_last_year[i] = z(bkwh);
        out.market_share_last_year[i] = z(ms);
        out.market_value_last_year[i] = z(mv);
        out.initial_number_of_adopters[i] = z(adopt);
        out.initial_pv_kw[i] = z(skc);
        out.initial_batt_kw[i] = z(bkw);
        out.initial_batt_kwh[i] = z(bkwh);
        out.initial_market_share[i] = z(ms);
        out.initial_market_value[i] = 0.0;
        (void)batt_n;
    }
}

// ---------------------------------------------------------------------------
// Finance-series export: finance_series_export._norm25 over the
// six 26-long yearly arrays of every agent, finance_series_export.py:9-20 --
// first 25 entries, zero past the agent's list length (N + 1), non-finite -> 0.
// Thread per (agent, series, entry); out [6][n][25].
// ---------------------------------------------------------------------------
constexpr int NORM25 = 25;
struct Series6 {
    const double* p[6];
};
__global__ void k_finance_series(Series6 src, const int32_t* __restrict__ len, int64_t n,
                                 int32_t stride, double* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 6 * n * NORM25) return;
    const int c = (int)(t / (n * NORM25));
    const int64_t r = t - (int64_t)c * n * NORM25;
    const int64_t i = r / NORM25;
    const int k = (int)(r - i * NORM25);
    double v = 0.0;
    if (k < len[i]) v = src.p[c][i * stride + k];
    out[t] = isfinite(v) ? v : 0.0;
}

#ifndef DGEN_TU_SEARCH
// ===========================================================================
// Certified Brent paths (round 6).  k_size bills from re-associated sums (the
// rows' slot sums, the net-billing split), so its objective differs from the
// oracle's -- SSC's hour order -- by a few ulps, and scipy's parabolic step can
// amplify such a difference into another Brent path.
// Each search traces its objective values (brent_bounded's trace);
// k_brent_certify replays the search from them with a bound on |device -
// oracle| carried through every state variable, and lists the agents where a
// decision is not certain under that bound; k_size_exact re-runs those
// agents' searches in the oracle's own arithmetic (oracle/orc.c
// perf_no_batt / orc_ur5 / orc_cashloan, op for op, hours in time order), so
// every agent's Brent path, bills and NPV are the reference driver's.
// ===========================================================================
constexpr double BT_EPS = 2.220446049250313e-16;
// Error model of one evaluation (k_brent_certify), u = eps / 2 the unit
// roundoff of round-to-nearest:
// * a recursive sum of n terms errs by at most gamma_(n-1) ~ (n - 1) u x the
//   sum of their magnitudes (Higham, Accuracy and Stability, 4.2): a (month,
//   period) bin holds <= 744 hours, the slot / split forms add < 100 terms of
//   their own and each hourly term <= 4 roundings, so device and oracle bins
//   differ by <= ~850 u x (load + generation);
// * a bill moves by at most 2 x the largest price per kWh of bin change (a
//   tier share's re-weighting at most doubles the marginal price; NEM credits
//   are billed once, at a buy, sell or true-up price); so |bill_d - bill_o| <=
//   1710 u x price x (load + generation) <= BT_GAMMA x 2 eps x ... with
//   BT_GAMMA = 512 (= 2048 u; round 6's first form counted eps per rounding,
//   BT_GAMMA 1024, twice the slack);
// * NPV adds the years' bill differences discounted (D) with weight <= 1 (the
//   commercial tax factors are below 1), plus the cash flow's own roundings.
// Every single operation's rounding in the replay (bt_rnd) keeps eps.
constexpr double BT_GAMMA = 512.0;

struct BtModel {
    double c0, c1, ce;   // |f_device - f_oracle| <= c0 + c1 x + ce |f| at the same x
    double lip;          // |f(x) - f(x')| <= lip |x - x'| between rate switches
};

// bound of an operation's result: exact inputs give bit-identical results on
// both sides; inexact ones add one rounding of the result
__device__ __forceinline__ double bt_rnd(double d, double v) { return d > 0.0 ? d + BT_EPS * fabs(v) : 0.0; }

// is the comparison of u and v (bounds du, dv) decided the same way on both sides?
__device__ __forceinline__ bool bt_sure(double u, double du, double v, double dv) {
    const double s = du + dv;
    return s == 0.0 || fabs(u - v) > s;
}
// equality of two Brent points: the same evaluation's x is equal on both sides
__device__ __forceinline__ bool bt_sure_eq(double u, double du, int pu, double v, double dv, int pv) {
    return pu == pv || bt_sure(u, du, v, dv);
}

// brent_bounded replayed from its traced objective values with bounds: true
// when every decision (comparisons, branch tests, the rate switch's
// thresholds, the final x's to 1e-10) is the oracle's under the model M.
// The values follow brent_bounded's operations exactly (same x's).
// bt_replay's undecided comparisons by kind (DGEN_PHASE_PROF builds: phase
// slots 1 switch thresholds / x order / final x's, 2 fu vs fx, 3 the other
// point updates, 7 the termination tests, 8 the parabolic step's tests)
#if DGEN_PHASE_PROF
#define BT_FAIL(k) do { atomicAdd(&g_phase[k], 1ull); return false; } while (0)
#else
#define BT_FAIL(k) return false
#endif
__device__ bool bt_replay(const double* __restrict__ f, int nfev, double x1, double x2, double xatol,
                          const BtModel& M, const dgen_switch* sw, int sw_cnt) {
    const double sqrt_eps = 1.4832396974191326e-08;
    const double golden_mean = 0.3819660112501051;
    double a = x1, b = x2, da = 0.0, db = 0.0;
    double fulc = a + golden_mean * (b - a);
    double nfc = fulc, xf = fulc;
    double dfulc = 0.0, dnfc = 0.0, dxf = 0.0;
    int pfulc = 0, pnfc = 0, pxf = 0;             // evaluation each point came from
    double rat = 0.0, e = 0.0, drat = 0.0, de = 0.0;
    double x = xf, dx = 0.0, dx_last = 0.0;
    double fx = 0.0, ffulc = 0.0, fnfc = 0.0, dfx = 0.0, dffulc = 0.0, dfnfc = 0.0;
    int num = 0;
    for (;;) {
        if (num >= nfev || num >= BT_MAX) BT_FAIL(1);
        // the evaluation at x: the sticky solar switch's row test must agree
        if (!bt_sure(x, dx, 0.0, 0.0)) BT_FAIL(8);
        for (int r = 0; r < sw_cnt; r++)
            if (!bt_sure(x, dx, sw[r].min_kw, 0.0) || !bt_sure(x, dx, sw[r].max_kw, 0.0)) BT_FAIL(1);
        const double fu = f[num];
        const double dfu = M.c0 + M.c1 * fabs(x) + M.ce * fabs(fu) + M.lip * dx;
        const int px = num;
        dx_last = dx;
        num += 1;
        if (num == 1) {
            fx = fu; ffulc = fu; fnfc = fu;
            dfx = dfu; dffulc = dfu; dfnfc = dfu;
        } else {
            if (!bt_sure(fu, dfu, fx, dfx)) BT_FAIL(2);
            if (!bt_sure(x, dx, xf, dxf)) BT_FAIL(1);
            if (fu <= fx) {
                if (x >= xf) { a = xf; da = dxf; } else { b = xf; db = dxf; }
                fulc = nfc; dfulc = dnfc; pfulc = pnfc; ffulc = fnfc; dffulc = dfnfc;
                nfc = xf; dnfc = dxf; pnfc = pxf; fnfc = fx; dfnfc = dfx;
                xf = x; dxf = dx; pxf = px; fx = fu; dfx = dfu;
            } else {
                if (x < xf) { a = x; da = dx; } else { b = x; db = dx; }
                // (fu <= fnfc) || (nfc == xf): decided when both tests are, or
                // when a decided test settles the ||
                const bool ca = bt_sure(fu, dfu, fnfc, dfnfc), ra = fu <= fnfc;
                const bool cb = bt_sure_eq(nfc, dnfc, pnfc, xf, dxf, pxf), rb = nfc == xf;
                if (!((ca && cb) || (ca && ra) || (cb && rb))) BT_FAIL(3);
                if (ra || rb) {
                    fulc = nfc; dfulc = dnfc; pfulc = pnfc; ffulc = fnfc; dffulc = dfnfc;
                    nfc = x; dnfc = dx; pnfc = px; fnfc = fu; dfnfc = dfu;
                } else {
                    const bool cc = bt_sure(fu, dfu, ffulc, dffulc), rc = fu <= ffulc;
                    const bool cd = bt_sure_eq(fulc, dfulc, pfulc, xf, dxf, pxf), rd = fulc == xf;
                    const bool ce = bt_sure_eq(fulc, dfulc, pfulc, nfc, dnfc, pnfc), re = fulc == nfc;
                    const bool any_true = (cc && rc) || (cd && rd) || (ce && re);
                    if (!any_true && !(cc && cd && ce)) BT_FAIL(3);
                    if (rc || rd || re) { fulc = x; dfulc = dx; pfulc = px; ffulc = fu; dffulc = dfu; }
                }
            }
        }
        const double xm = 0.5 * (a + b);
        const double dxm = bt_rnd(0.5 * (da + db), xm);
        const double tol1 = sqrt_eps * fabs(xf) + xatol / 3.0;
        const double dtol1 = bt_rnd(sqrt_eps * dxf, tol1);
        const double tol2 = 2.0 * tol1, dtol2 = 2.0 * dtol1;
        if (num >= 500) break;
        {
            const double lhs = fabs(xf - xm), rhs = tol2 - 0.5 * (b - a);
            const double dl = bt_rnd(dxf + dxm, lhs), dr = bt_rnd(dtol2 + 0.5 * (da + db), rhs);
            if (!bt_sure(lhs, dl, rhs, dr)) BT_FAIL(7);
            if (!(lhs > rhs)) break;
        }
        bool golden = true, rat_tol = false;
        if (!bt_sure(fabs(e), de, tol1, dtol1)) BT_FAIL(7);
        if (fabs(e) > tol1) {
            golden = false;
            const bool s1 = pxf == pnfc, s2 = pxf == pfulc;     // exact zero differences
            const double u1 = xf - nfc, du1 = s1 ? 0.0 : bt_rnd(dxf + dnfc, u1);
            const double u2 = xf - fulc, du2 = s2 ? 0.0 : bt_rnd(dxf + dfulc, u2);
            const double v1 = fx - ffulc, dv1 = s2 ? 0.0 : bt_rnd(dfx + dffulc, v1);
            const double v2 = fx - fnfc, dv2 = s1 ? 0.0 : bt_rnd(dfx + dfnfc, v2);
            double r = u1 * v1;
            const double dr = bt_rnd(fabs(u1) * dv1 + fabs(v1) * du1 + du1 * dv1, r);
            double q = u2 * v2;
            double dq = bt_rnd(fabs(u2) * dv2 + fabs(v2) * du2 + du2 * dv2, q);
            const double t1 = u2 * q, t2 = u1 * r;
            const double dt1 = bt_rnd(fabs(u2) * dq + fabs(q) * du2 + du2 * dq, t1);
            const double dt2 = bt_rnd(fabs(u1) * dr + fabs(r) * du1 + du1 * dr, t2);
            double p = t1 - t2;
            double dp = bt_rnd(dt1 + dt2, p);
            q = 2.0 * (q - r);
            dq = bt_rnd(2.0 * (dq + dr), q);
            if (pnfc == pfulc) { dp = 0.0; dq = 0.0; }       // the same point twice: r == q, p == 0
            const double r2 = e, dr2 = de;
            e = rat; de = drat;
            // (fabs(p) < fabs(0.5 q r)) && (p > q (a - xf)) && (p < q (b - xf)),
            // after p = -p when q > 0 and q = |q|
            const double aq = fabs(q);
            const double c1l = fabs(p), c1r = fabs(0.5 * aq * r2);
            const double dc1r = bt_rnd(0.5 * (aq * dr2 + fabs(r2) * dq + dq * dr2), c1r);
            if (!bt_sure(c1l, dp, c1r, dc1r)) BT_FAIL(8);
            bool para = false;
            if (c1l < c1r) {
                if (!bt_sure(q, dq, 0.0, 0.0)) BT_FAIL(8);
                p = q > 0.0 ? -p : p;
                const double ta = aq * (a - xf), dta = bt_rnd(aq * (da + dxf) + fabs(a - xf) * dq + dq * (da + dxf), ta);
                if (!bt_sure(p, dp, ta, dta)) BT_FAIL(8);
                if (p > ta) {
                    const double tb = aq * (b - xf), dtb = bt_rnd(aq * (db + dxf) + fabs(b - xf) * dq + dq * (db + dxf), tb);
                    if (!bt_sure(p, dp, tb, dtb)) BT_FAIL(8);
                    para = p < tb;
                }
            } else if (q > 0.0) {
                p = -p;
            }
            q = aq;
            if (para) {
                rat = (p + 0.0) / q;
                // |p'/q' - p/q| <= (dp + |p/q| dq) / (|q| - dq), |q| > dq above
                drat = bt_rnd((dp + fabs(rat) * dq) / (q - dq), rat);
                x = xf + rat;
                dx = bt_rnd(dxf + drat, x);
                // ((x - a) < tol2) || ((b - x) < tol2)
                const double xa = x - a, dxa = bt_rnd(dx + da, xa);
                const double bx = b - x, dbx = bt_rnd(db + dx, bx);
                const bool c1 = bt_sure(xa, dxa, tol2, dtol2), r1 = xa < tol2;
                const bool c2 = bt_sure(bx, dbx, tol2, dtol2), r2b = bx < tol2;
                if (!((c1 && c2) || (c1 && r1) || (c2 && r2b))) BT_FAIL(8);
                if (r1 || r2b) {
                    const double dm = xm - xf, ddm = bt_rnd(dxm + dxf, dm);
                    if (!bt_sure(dm, ddm, 0.0, 0.0)) BT_FAIL(8);
                    const double si = np_sign(dm) + ((dm == 0.0) ? 1.0 : 0.0);
                    rat = tol1 * si;
                    drat = dtol1;
                    rat_tol = true;                   // |rat| == tol1 on both sides
                }
            } else {
                golden = true;
            }
        }
        if (golden) {
            if (!bt_sure(xf, dxf, xm, dxm)) BT_FAIL(8);
            if (xf >= xm) { e = a - xf; de = bt_rnd(da + dxf, e); }
            else { e = b - xf; de = bt_rnd(db + dxf, e); }
            rat = golden_mean * e;
            drat = bt_rnd(golden_mean * de, rat);
        }
        if (!bt_sure(rat, drat, 0.0, 0.0)) BT_FAIL(8);
        const double si = np_sign(rat) + ((rat == 0.0) ? 1.0 : 0.0);
        const double ar = fabs(rat);
        if (!rat_tol && !bt_sure(ar, drat, tol1, dtol1)) BT_FAIL(8);
        const bool big = ar > tol1;
        x = xf + si * (big ? ar : tol1);
        dx = bt_rnd(dxf + (big ? drat : dtol1), x);
    }
    if (num != nfev) BT_FAIL(1);
    // the reported x's (system_kw = xf, x_last) within 1e-7 of the oracle's
    // under the bound (the decisions above fix the path; the observed
    // differences of certified agents are ~1e-13)
    if (dxf > 1e-7 * fmax(1.0, fabs(xf)) || dx_last > 1e-7 * fmax(1.0, fabs(x))) BT_FAIL(1);
    return true;
}

// Price bounds of the tariffs an agent's search can bill with (its initial
// tariff and every solar switch row): energy ($/kWh: buy, sell, the true-up
// rate, the TS sell rate), demand ($/kW a month) and the kWh/kW tier caps'
// sensitivity to the month peak.  From dgen_tables.bt_tariff (3 per tariff,
// Engine.set_tariffs) when present, else from the records.
__device__ void bt_prices(const dgen_tables& T, const dgen_cfg& cfg, int tix, double& pm, double& pmdc, double& pku,
                          bool& mo2) {
    const dgen_tariff& t = T.tariffs[tix];
    mo2 = mo2 || t.mo == 2;
    if (T.bt_tariff) {
        pm = fmax(pm, T.bt_tariff[3 * tix]);
        pmdc = fmax(pmdc, cfg.skip_demand_charges == 0 ? T.bt_tariff[3 * tix + 1] : 0.0);
        pku = fmax(pku, T.bt_tariff[3 * tix + 2]);
        return;
    }
    double e = 0.0, cap = 0.0;
    for (int p = 0; p < t.P && p < MAXP; p++)
        for (int k = 0; k < t.T && k < MAXT; k++) e = fmax(e, fmax(fabs(t.buy[p][k]), fabs(t.sell[p][k])));
    for (int k = 0; k < t.T && k < MAXT; k++) cap += fabs(t.cap[k]);
    pm = fmax(pm, e);
    if (t.unit == 1 || t.unit == 3) pku = fmax(pku, 2.0 * e * cap * (t.unit == 3 ? 31.0 : 1.0));
    if (cfg.skip_demand_charges == 0 && t.dc > 0) pmdc = INFINITY;   // no bound without the table
}

// One thread per agent: replay its traced search, list it when not certain.
// list[0] counts the chunk's listed agents, list[1 ..] their rows.
__global__ void __launch_bounds__(256)
k_brent_certify(dgen_tables T, dgen_agents A, dgen_outputs O, dgen_cfg cfg, int64_t i0, int64_t i1,
                const double* __restrict__ trace, int32_t* list, int mode) {
    const int64_t i = i0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool flag = false;
    if (i < i1) {
        const int nfev = O.nfev[i];
        const int st = O.status[i];
        if (nfev > 0 && !(st & (DGEN_ST_BOUNDS | DGEN_ST_TARIFF | DGEN_ST_UNIT | DGEN_ST_YEARS))) {
            flag = true;
            if (mode == 1 && nfev <= BT_MAX) {
                const int N = A.econ_life[i];
                const double kwh = A.load_kwh[i];
                const int lr = A.load_row[i], cr = A.cf_row[i];
                const double naep0 = T.cf_naep[cr];
                const double max_load = kwh / naep0;               // k_size's bracket
                const double low = max_load * 0.8, high = max_load * 1.25;
                const double span = high - low;
                const double tl = (span > 1.0 ? span : 1.0) * 1e-3;
                const double fl_tl = floor(tl);
                const double xatol = fl_tl < 2.0 ? 2.0 : fl_tl;
                // prices of every tariff the search can bill with
                double pm = fabs(cfg.nm_yearend_sell_rate), pmdc = 0.0, pku = 0.0, otc = 0.0;
                bool mo2 = false;
                const int t0 = A.tariff0[i];
                bt_prices(T, cfg, t0, pm, pmdc, pku, mo2);
                const dgen_switch* sw = T.switches + A.sw_solar_off[i];
                const int sw_cnt = A.sw_solar_cnt[i];
                bool ok = true;
                for (int r = 0; r < sw_cnt; r++) {
                    const int tt = sw[r].tariff;
                    if (tt < 0 || tt >= T.n_tariffs) { ok = false; break; }
                    bt_prices(T, cfg, tt, pm, pmdc, pku, mo2);
                    otc = fmax(otc, fabs(sw[r].one_time_charge));
                }
                const bool is_ca = (A.flags[i] & 2) != 0;
                const int wr = A.wholesale_row[i];
                if (mo2 && !is_ca && wr >= 0 && T.wholesale) {
                    if (!T.bt_ts_max) ok = false;
                    else pm = fmax(pm, T.bt_ts_max[wr] * fabs(A.price_mult[i]) * (1.0 + 1e-6));
                }
                // discounted escalation over the analysis period, D = sum_y rr^y
                // (1 + infl + esc)^(y - 1), and the largest degradation factor
                const double infl = A.inflation[i], real = A.real_discount[i];
                const double rr = 1.0 / ((1.0 + real) * (1.0 + infl));
                const double rb = fabs(1.0 + infl + A.escalator[i]);
                const double sb = fabs(1.0 - A.pv_deg[i]);
                double D = 0.0, dr = 1.0, er = 1.0, smax = 1.0, sy = 1.0;
                for (int y = 1; y <= N && y <= MAXY; y++) {
                    dr *= rr;
                    D += dr * er;
                    er *= rb;
                    smax = fmax(smax, sy);
                    sy *= sb;
                }
                D *= 1.01;
                // peak load (kW) and per-kW generation of the agent's rows
                const double S = T.shape_sum[lr];
                const double lmax = T.bt_shape_max ? T.bt_shape_max[lr] * fabs(kwh / S) : INFINITY;
                const double gmax = T.bt_cf_max ? T.bt_cf_max[cr] * 1e-6 : INFINITY;
                const double capc = fabs(A.capex[i] * A.ccm[i]);
                const double dem = pmdc + pku;                    // $/kW a month of peak
                const double g = BT_GAMMA * BT_EPS;
                BtModel M;
                // bills (BT_GAMMA's model): 2 x price x (load + generation) a
                // year for the with-system bill and the no-system one; demand:
                // 12 months x price x (peak load + generation at the peak hour)
                // (4 x: a coarser bound, the extension mode only)
                M.c0 = g * (2.0 * D * pm * 2.0 * fabs(kwh) + (dem > 0.0 ? 4.0 * D * dem * 24.0 * lmax : 0.0) + otc);
                M.c1 = g * (2.0 * D * smax * 0.96 * pm * fabs(naep0) + (dem > 0.0 ? 4.0 * D * smax * 0.96 * dem * 12.0 * gmax : 0.0) +
                            4.0 * capc);
                M.ce = g;
                // Lipschitz: NPV moves by <= (3 + 0.02 D) x the cost change (the
                // debt's payments at up to twice their principal, tax shields,
                // insurance) and by <= 2 x price x generation of the bills
                // (+10 %); demand: 12 months x price x generation per kW
                M.lip = (3.0 + 0.02 * D) * capc + 2.2 * D * smax * 0.96 * pm * fabs(naep0) +
                        (dem > 0.0 ? 4.0 * D * smax * 0.96 * dem * 12.0 * gmax : 0.0);
                if (ok && isfinite(M.c0) && isfinite(M.c1) && isfinite(M.lip) && isfinite(xatol))
                    flag = !bt_replay(trace + i * BT_MAX, nfev, low, high, xatol, M, sw, sw_cnt);
            }
        }
    }
    // compact the wave's listed agents (one counter add per wave)
    const unsigned long long m = __ballot(flag);
    const int lane = threadIdx.x & (WAVE - 1);
    int base = 0;
    if (m) {
        const int lead = __ffsll((long long)m) - 1;
        if (lane == lead) base = atomicAdd(list, __popcll(m));
        base = __shfl(base, lead, WAVE);
        if (flag) list[1 + base + __popcll(m & ((1ull << lane) - 1ull))] = (int32_t)i;
    }
}

// ---------------------------------------------------------------------------
// k_size_exact: the listed agents' searches in the oracle's arithmetic.  One
// block per agent at a time (the blocks stride over the list).  Per tariff the
// block lists each month's hours by period (time order kept within a period:
// the hours of one bin are a subsequence of the month's, so a bin summed over
// its list in list order is oracle bin_year's own sum).  Per evaluation a wave
// takes one (month, period) bin at a time with lane = analysis year: the
// wave stages the bin's hours 64 at a time in LDS (load, this evaluation's
// generation, TS rate; every hour's generation formed once, by one lane) and
// each lane walks them in order with its year's degradation factor, so all
// years of the bin share one pass over its hours (broadcast LDS reads).  A
// thread per year then bills its months in order (year_bill, year_demand) and
// thread 0 runs the cash flow (orc_cashloan).  The search state and the
// objective are block-uniform (scalar branches).
// (v4, one lane per (year, month, period) cell gathering its hours from global
// memory through the hour list, was latency-bound: national 200k, 7 163 agents
// listed, 80 ms.)
// ---------------------------------------------------------------------------
// a block-uniform double (every thread holds the same value, read from LDS):
// readfirstlane makes it a scalar, so the search's branches on it are scalar
// branches, not exec-masked ones
__device__ __forceinline__ double ex_uniform(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(b & 0xffffffffull));
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}


// fr: the year thread's scratch for the periods' shares u_p / U, formed once
// per month (the oracle forms the same quotient per tier: equal bits)
__device__ __forceinline__ double ex_month_charge(const dgen_tariff& t, int m, const double* u, double peak,
                                                  double* fr) {
    double U = 0.0;
    for (int p = 0; p < t.P; p++) U += u[p];
    // (the oracle returns 0 for U <= 0 first; here the charge is formed
    // anyway and discarded -- no branch on the lanes' data)
    const bool pos = U > 0.0;
    if (t.T == 1) {
        double charge = 0.0;
        for (int p = 0; p < t.P; p++) charge += u[p] * t.buy[p][0];
        return pos ? charge : 0.0;
    }
    const double days = (double)c_days_in_month[m];
    // oracle: unit 2 days, 1 peak, 3 peak x days, else 1 -- as one product of
    // selects (x * 1.0 == x), so the year threads' divergent region holds no
    // branch on the unit
    const double f_pk = (t.unit == 1 || t.unit == 3) ? peak : 1.0;
    const double f_days = (t.unit == 2 || t.unit == 3) ? days : 1.0;
    const double scale = f_pk * f_days;
    for (int p = 0; p < t.P; p++) fr[p] = u[p] / U;
    double charge = 0.0, prev = 0.0;
    for (int k = 0; k < t.T; k++) {
        const double hi = (k == t.T - 1) ? INFINITY : t.cap[k] * scale;
        const double top = U < hi ? U : hi;
        const double amt0 = top - prev;
        const double amt = amt0 < 0.0 ? 0.0 : amt0;
        prev = hi > prev ? hi : prev;
        for (int p = 0; p < t.P; p++) charge += fr[p] * amt * t.buy[p][k];
    }
    return pos ? charge : 0.0;
}

__device__ __forceinline__ double ex_dc_tier(double peak, const double* cap, const double* price, int nt) {
    double charge = 0.0, prev = 0.0;
    for (int k = 0; k < nt; k++) {
        const double hi = (k == nt - 1) ? INFINITY : cap[k];
        const double top = peak < hi ? peak : hi;
        const double amt0 = top - prev;
        const double amt = amt0 < 0.0 ? 0.0 : amt0;
        prev = hi > prev ? hi : prev;
        charge += amt * price[k];
    }
    return charge;
}

// Scratch of k_size_exact.  Per block slot, in global memory: the current
// tariff's hour list -- per month, period 0's hours, then period 1's, ...,
// each in time order -- with every listed hour's load, generation per kW and
// TS sell rate in list order (so an evaluation streams them contiguously),
// and the bins of every analysis year.  In LDS: the list offsets, each wave's
// stage of 64 hours, the per-year bill state and the cash-flow rows.
constexpr int EX_THREADS = 256;
constexpr int EX_BLOCKS = 1024;
constexpr int EX_HOFF = MAXP + 1;                  // list offsets per month
static_assert(MAXY + 1 <= 64, "k_size_exact: one lane per analysis year and the no-system year");
__host__ __device__ inline size_t ex_ws_base() {
    return ((size_t)3 * NH * sizeof(double) + (size_t)NH * sizeof(uint16_t) + 255) / 256 * 256;
}
__host__ __device__ inline size_t ex_ws_bytes(int P, bool dcb) {
    const size_t bins = (size_t)(MAXY + 1) * 12 * (size_t)P * (3 + (dcb ? (size_t)DCP : 0)) * sizeof(double);
    return ex_ws_base() + (bins + 255) / 256 * 256;
}
struct ExLds {
    double* Lp;        // [8760] load of the listed hours, list order (global)
    double* Cp;        // [8760] generation per kW (cf / 1e6) of the listed hours (global)
    double* Tp;        // [8760] TS sell rate of the listed hours (global)
    uint16_t* hl;      // [8760] the hour list (global)
    int32_t* hoff;     // [12][EX_HOFF] list offsets (absolute; LDS)
    double* bins;      // [MAXY][12][2 P]: mo 0/1 net | mo 4 load, gen | mo 2/3 import, export ($ with TS) (global)
    double* cmax;      // [MAXY][12][P] each bin's largest import (the month peak: their max, from 0) (global)
    double* dcm;       // [MAXY][12][P][DCP] each bin's largest import per demand period (billed demand only; global)
    double* stg;       // [waves][4][256] the wave's staged hours: load, generation, TS rate, demand period (LDS)
    double* yr;        // [MAXY + 1][3 MAXP] per-year-thread credit / billed kWh / period shares (LDS)
    double* res;       // [6][MAXY + 1] aev, bill_w, bill_wo, cf_payback, cf_energy_value, atcf; + 8 scalars (LDS)
    int bny;           // the bins' year stride (LDS: the batch's N + 1; global: MAXY + 1)
    int ptab;          // the table's periods (the bins' layout)
    bool dcb;          // dcm present
};

__host__ __device__ inline size_t ex_lds_bytes() {
    return sizeof(double) * ((size_t)(EX_THREADS / 64) * 4 * 256 + (size_t)(MAXY + 1) * 3 * MAXP + 6 * (size_t)(MAXY + 1) + 8) +
           sizeof(int32_t) * (size_t)12 * EX_HOFF;   // = ex_stg + ex_yr + ex_res + ex_hoff
}

// The LDS parts at fixed offsets of dyn_lds (the compiler then knows they
// are LDS and emits ds_* accesses; through the generic pointers of a struct
// they became flat loads with memory-path latency)
constexpr size_t EX_STG_QW = (size_t)(EX_THREADS / 64) * 4 * 256;
constexpr size_t EX_YR_QW = (size_t)(MAXY + 1) * 3 * MAXP;
constexpr size_t EX_RES_QW = 6 * (size_t)(MAXY + 1) + 8;
__device__ __forceinline__ double* ex_stg(int wv) { return dyn_lds + (size_t)wv * 4 * 256; }
__device__ __forceinline__ double* ex_yr() { return dyn_lds + EX_STG_QW; }
__device__ __forceinline__ double* ex_res() { return dyn_lds + EX_STG_QW + EX_YR_QW; }
__device__ __forceinline__ int32_t* ex_hoff() {
    return reinterpret_cast<int32_t*>(dyn_lds + EX_STG_QW + EX_YR_QW + EX_RES_QW);
}
// the bins, their peaks and demand-period peaks: LB, in LDS after the list
// offsets (ds_* accesses: the year bills' reads are latency-bound), else the
// block's global scratch
struct ExB {
    double* bins;
    double* cmax;
    double* dcm;
};
template <bool LB>
__device__ __forceinline__ ExB ex_b(const double* gbins, int bny, int P, bool dcb) {
    ExB b;
    if constexpr (LB) b.bins = reinterpret_cast<double*>(ex_hoff() + 12 * EX_HOFF);
    else b.bins = const_cast<double*>(gbins);
    b.cmax = b.bins + (size_t)bny * 12 * 2 * P;
    b.dcm = dcb ? b.cmax + (size_t)bny * 12 * P : nullptr;
    return b;
}

struct ExAgent {
    const dgen_demand* demand;
    int n_demand;
    bool dc_on;
    bool has_ts;
    int N;
    double rate_base, sys_base, yearend;
};

// The hour list of tariff t and the listed hours' values: wave w takes
// months w, w + waves, ...; lanes = the month's hours 64 at a time (a ballot
// per period: lane order = time order); the month's two day-type schedules
// come in once (lanes 0-47) and each lane takes its hour's period by a
// shuffle.  Every hour's load (elec.py:571-577 scale_array_sum), generation
// per kW (cf / 1e6, ff:350) and TS sell rate (ff:182,246,372 x multiplier,
// float32-rounded) are read in time order and written at the hour's list
// position.
constexpr int EX_HQ = 4;            // chunks of profile values in flight (ex_hour_lists)
__device__ void ex_hour_lists(const dgen_tariff& t, const ExLds& L, const float* __restrict__ sh, double S,
                              double kwh, const int32_t* __restrict__ cfr, const double* __restrict__ wrow,
                              double pmul) {
    const int P = t.P;
    const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE, nw = blockDim.x / WAVE;
    const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (WAVE - lane));
    for (int m = wv; m < 12; m += nw) {
        const int h0 = c_month_start_day[m] * 24, h1 = c_month_start_day[m + 1] * 24;
        const int sched = lane < 24 ? (int)t.wkday[m][lane] : (lane < 48 ? (int)t.wkend[m][lane - 24] : 0);
        auto period = [&](int i) __attribute__((always_inline)) -> int {
            const int src = (((i % 168) >= 120) ? 24 : 0) + i % 24;
            const int pr = __shfl(sched, src, WAVE);
            return i < h1 ? pr : -1;
        };
        // the month's first EX_HQ chunks of values in flight across the
        // counting pass, then EX_HQ chunks ahead of the one being placed (a
        // ring of registers; at one chunk ahead each chunk waited out its
        // loads' latency)
        float shq[EX_HQ];
        int32_t cfq[EX_HQ];
        double whq[EX_HQ];
        auto fetch = [&](int d, int c) __attribute__((always_inline)) {
            const int i2 = c + lane;
            const bool in2 = i2 < h1;
            shq[d] = in2 ? sh[i2] : 0.0f;
            cfq[d] = in2 ? cfr[i2] : 0;
            whq[d] = (in2 && wrow) ? wrow[i2] : 0.0;
        };
#pragma unroll
        for (int d = 0; d < EX_HQ; d++) fetch(d, h0 + d * WAVE);
        int cnt = 0;                                   // lane p < P: hours of period p
        for (int c = h0; c < h1; c += WAVE) {
            const int per = period(c + lane);
            for (int p = 0; p < P; p++) {
                const unsigned long long b = __ballot(per == p);
                if (lane == p) cnt += __popcll(b);
            }
        }
        // exclusive prefix over the period lanes
        int incl = lane < P ? cnt : 0;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const int v = __shfl_up(incl, o, WAVE);
            if (lane >= o) incl += v;
        }
        int cur = h0 + incl - (lane < P ? cnt : 0);    // lane p: first position of period p
        if (lane <= P) ex_hoff()[m * EX_HOFF + lane] = lane < P ? cur : h1;
        for (int c0 = h0; c0 < h1; c0 += EX_HQ * WAVE)
#pragma unroll
        for (int d = 0; d < EX_HQ; d++) {
            const int c = c0 + d * WAVE;
            if (c >= h1) break;
            const int i = c + lane;
            const float shv = shq[d];
            const int32_t cfv = cfq[d];
            const double whv = whq[d];
            fetch(d, c + EX_HQ * WAVE);
            const int per = period(i);
            int pos = 0;
            for (int p = 0; p < P; p++) {
                const unsigned long long b = __ballot(per == p);
                const int base = __shfl(cur, p, WAVE);
                if (per == p) pos = base + __popcll(b & below);
                if (lane == p) cur += __popcll(b);
            }
            if (per >= 0) {
                L.hl[pos] = (uint16_t)i;
                L.Lp[pos] = ((double)shv / S) * kwh;
                L.Cp[pos] = cf_per_kw(cfv);
                L.Tp[pos] = wrow ? (double)(float)(whv * pmul) : 0.0;
            }
        }
    }
}

// global scratch written by some lanes, read by others: every store done,
// a barrier, the CU's L1 lines dropped (agent-scope acquire)
__device__ __forceinline__ void ex_handoff() {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// bin_year's bins of years [0, ny) (GEN false: the no-system year 0, at
// kW 0).  Lane = year.  Wave w takes a contiguous run of the 12 P (month,
// period) bins -- a contiguous run of the list -- and streams it 64 hours at
// a time through its LDS stage (the next 64 in flight while these are
// walked; each hour's generation at kW formed once, by the lane that stages
// it); every lane adds the hours of a bin in list order, the oracle's order,
// and writes the bin where the next one starts.  One instantiation per
// billing form, so an hour costs only its form's operations: EX_NEM (options
// 0 / 1: the net kWh), EX_BA (4: load and generation), EX_NB (2 / 3: import,
// export, x the TS rate when TS); PK: the bins' largest imports (kWh/kW tier
// units 1 / 3, demand charges), DEM: per demand period too.  Every sum is the
// oracle bin_year's (a skipped sum is one the bill never reads).
constexpr int EX_NEM = 0, EX_BA = 1, EX_NB = 2;
constexpr int EX_R = 4, EX_CH = EX_R * 64;         // hours per lane / per chunk
template <int FORM, bool GEN, bool PK, bool DEM, bool TS, bool LB, bool HW>
__device__ void ex_run(const ExAgent& a, const dgen_tariff& t, const dgen_demand* dem, int ny, double kw,
                       const ExLds& L, int nsl) {
    // HW: two runs of bins per wave, one per half-wave (lane = year within
    // the half: N + 1 <= 32), so 50 of 64 lanes work instead of 25
    constexpr int HL = HW ? 32 : WAVE;                 // lanes per run
    constexpr int CH = EX_R * HL;                      // hours per chunk per run
    const int P = t.P;
    const ExB B = ex_b<LB>(L.bins, L.bny, L.ptab, L.dcb);
    const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE, nw = blockDim.x / WAVE;
    const int h = lane / HL, yl = lane % HL;
    // the lane's year's degradation factor; lane nsl (when >= 0): the
    // no-system year, factor 0 -- its generation term is +-0, so every sum
    // is the kW-0 pass's (load - 0 == load)
    const double s = yl == nsl ? 0.0 : pow_seq(a.sys_base, yl);
    double* const sL = ex_stg(wv) + h * CH;
    double* const sG = ex_stg(wv) + EX_CH + h * CH;
    double* const sT = ex_stg(wv) + 2 * EX_CH + h * CH;
    int* const sQ = reinterpret_cast<int*>(ex_stg(wv) + 3 * EX_CH) + h * CH;
    const int nb = 12 * P;
    // list position where bin b starts (b == nb: the end of the list)
    auto bstart = [&](int b) __attribute__((always_inline)) -> int {
        const int m = b / P;
        const int v = b >= nb ? NH : ex_hoff()[m * EX_HOFF + (b - m * P)];
        if constexpr (HW) return v;
        else return __builtin_amdgcn_readfirstlane(v);
    };
    const int wA = (wv * nb) / nw, wB = ((wv + 1) * nb) / nw;
    if (wA >= wB) return;
    // the wave's bins, split between the halves at the bin nearest the
    // middle hour of the run
    int bA = wA, bB = wB;
    if constexpr (HW) {
        const int mid = (bstart(wA) + bstart(wB)) / 2;
        int bM = wA + 1;
        while (bM < wB && bstart(bM) < mid) bM++;
        bA = h == 0 ? wA : bM;
        bB = h == 0 ? bM : wB;
    }
    const int kA = bstart(bA), kB = bstart(bB);
    int b = bA, kn = bstart(bA + 1), m = bA / P;
    double b0 = 0.0, b1 = 0.0, mx = 0.0;
    double dq[DEM ? DCP : 1];
#pragma unroll
    for (int q = 0; q < (DEM ? DCP : 1); q++) dq[q] = 0.0;
    auto flush = [&]() __attribute__((always_inline)) {
        if (yl < ny || yl == nsl) {
            const int p = b - m * P;
            double* bn = B.bins + ((size_t)yl * 12 + m) * 2 * P;
            bn[p] = b0;
            bn[P + p] = b1;
            B.cmax[((size_t)yl * 12 + m) * P + p] = mx;
            if constexpr (DEM) {
#pragma unroll
                for (int q = 0; q < DCP; q++) B.dcm[(((size_t)yl * 12 + m) * P + p) * DCP + q] = dq[q];
            }
        }
        b0 = 0.0; b1 = 0.0; mx = 0.0;
#pragma unroll
        for (int q = 0; q < (DEM ? DCP : 1); q++) dq[q] = 0.0;
        b += 1;
        kn = bstart(b + 1);
        m = b / P;
    };
    // one hour, the oracle's operations (imports and exports as selects)
    auto step = [&](int j) __attribute__((always_inline)) {
        const double ld = sL[j];
        // (option 4 sums the generation itself: the no-system lane's is +0)
        const double g = GEN ? ((FORM == EX_BA && yl == nsl) ? 0.0 : sG[j] * s) : 0.0;
        const double dd = ld - g;
        if constexpr (PK) mx = dd > mx ? dd : mx;
        if constexpr (FORM == EX_NEM) {
            b0 += dd;
        } else if constexpr (FORM == EX_BA) {
            b0 += ld;
            b1 += g;
        } else {
            const bool imp = dd > 0.0;
            const double ex = -dd;
            const double xv = TS ? ex * sT[j] : ex;
            b0 += imp ? dd : 0.0;
            b1 += imp ? 0.0 : xv;
        }
        if constexpr (DEM) {      // year_demand's TOU peaks: maxima, any order
            const int q = sQ[j];
#pragma unroll
            for (int k = 0; k < DCP; k++) {
                const double up = dd > dq[k] ? dd : dq[k];
                dq[k] = (k == q) ? up : dq[k];
            }
        }
    };
    // the hour's demand period: from the hour and its month
    auto dper = [&](int k) __attribute__((always_inline)) -> int {
        const int i = L.hl[k];
        int mm = 0;
        while (mm < 11 && i >= c_month_start_day[mm + 1] * 24) mm++;
        const int hh = i % 24;
        return ((i % 168) >= 120) ? dem->wkend[mm][hh] : dem->wkday[mm][hh];
    };
    // chunks of CH hours per run (EX_R per lane); the next chunk's values in
    // registers while this one is walked (a chunk's walk outlasts the loads'
    // latency from L2 / MALL)
    double lv[EX_R], cv[EX_R], tv[EX_R];
    int qv[EX_R];
    auto fetch = [&](int c0) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < EX_R; r++) {
            const int kk = c0 + r * HL + yl;
            const bool v = kk < kB;
            lv[r] = v ? L.Lp[kk] : 0.0;
            if constexpr (GEN) cv[r] = v ? L.Cp[kk] : 0.0;
            if constexpr (TS) tv[r] = v ? L.Tp[kk] : 0.0;
            if constexpr (DEM) qv[r] = v ? dper(kk) : 0;
        }
    };
    // the chunk count of the wave: the longer run's (each half's own count
    // in HW; a half past its run walks nothing)
    int nch = (kB - kA + CH - 1) / CH;
    if constexpr (HW) {
        const int n0 = __builtin_amdgcn_readlane(nch, 0), n1 = __builtin_amdgcn_readlane(nch, HL);
        nch = n0 > n1 ? n0 : n1;
    }
    fetch(kA);
    for (int ci = 0; ci < nch; ci++) {
        const int c = kA + ci * CH;
        const int n = (kB - c) < CH ? ((kB - c) > 0 ? kB - c : 0) : CH;   // this run's hours in the chunk
        wave_lds_sync();                               // the previous chunk's reads
#pragma unroll
        for (int r = 0; r < EX_R; r++) {
            const int o = r * HL + yl;
            sL[o] = lv[r];
            // ff:117-120 generation of the hour at kW, oracle perf_no_batt's order
            if constexpr (GEN) sG[o] = ref_gen(cv[r], kw);
            if constexpr (TS) sT[o] = tv[r];
            if constexpr (DEM) sQ[o] = qv[r];
        }
        wave_lds_sync();
        if (ci + 1 < nch) fetch(c + CH);               // the next chunk in flight
        if constexpr (!HW) {
            int j = 0;
            while (j < n) {
                while (c + j == kn) flush();           // the bins that end here (empty ones too)
                const int je = (kn - c) < n ? (kn - c) : n;
                for (; j + 4 <= je; j += 4) {
#pragma unroll
                    for (int u = 0; u < 4; u++) step(j + u);
                }
                for (; j < je; j++) step(j);
            }
        } else {
            // the halves walk their own hours in step; a segment runs to the
            // nearer of the two halves' next events (a bin's end, the run's
            // end in this chunk), where the half it belongs to flushes
            const int n0 = __builtin_amdgcn_readlane(n, 0), n1 = __builtin_amdgcn_readlane(n, HL);
            const int nmax = n0 > n1 ? n0 : n1;
            int j = 0;
            while (j < nmax) {
                while (j < n && c + j == kn) flush();  // this half's bins that end here
                const int ev = j < n ? ((kn - c) < n ? (kn - c) : n) : nmax;
                const int e0 = __builtin_amdgcn_readlane(ev, 0), e1 = __builtin_amdgcn_readlane(ev, HL);
                const int je = e0 < e1 ? e0 : e1;
                if (j < n) {                           // (a half past its run's hours sits out)
                    int jj = j;
                    for (; jj + 4 <= je; jj += 4) {
#pragma unroll
                        for (int u = 0; u < 4; u++) step(jj + u);
                    }
                    for (; jj < je; jj++) step(jj);
                }
                j = je;
            }
        }
    }
    // the run's last bin and any empty bins after it
    while (b < bB) flush();
}

template <bool LB, bool HW>
__device__ void ex_cells_h(const ExAgent& a, const dgen_tariff& t, const dgen_demand* dem, int ny, double kw,
                         const ExLds& L, int nsl) {
    const bool pk = dem != nullptr || t.unit == 1 || t.unit == 3;
    const bool ts = a.has_ts && t.mo == 2;
    if (t.mo == 0 || t.mo == 1) {
        if (dem) ex_run<EX_NEM, true, true, true, false, LB, HW>(a, t, dem, ny, kw, L, nsl);
        else if (pk) ex_run<EX_NEM, true, true, false, false, LB, HW>(a, t, dem, ny, kw, L, nsl);
        else ex_run<EX_NEM, true, false, false, false, LB, HW>(a, t, dem, ny, kw, L, nsl);
    } else if (t.mo == 4) {
        if (dem) ex_run<EX_BA, true, true, true, false, LB, HW>(a, t, dem, ny, kw, L, nsl);
        else if (pk) ex_run<EX_BA, true, true, false, false, LB, HW>(a, t, dem, ny, kw, L, nsl);
        else ex_run<EX_BA, true, false, false, false, LB, HW>(a, t, dem, ny, kw, L, nsl);
    } else if (ts) {
        if (dem) ex_run<EX_NB, true, true, true, true, LB, HW>(a, t, dem, ny, kw, L, nsl);
        else if (pk) ex_run<EX_NB, true, true, false, true, LB, HW>(a, t, dem, ny, kw, L, nsl);
        else ex_run<EX_NB, true, false, false, true, LB, HW>(a, t, dem, ny, kw, L, nsl);
    } else {
        if (dem) ex_run<EX_NB, true, true, true, false, LB, HW>(a, t, dem, ny, kw, L, nsl);
        else if (pk) ex_run<EX_NB, true, true, false, false, LB, HW>(a, t, dem, ny, kw, L, nsl);
        else ex_run<EX_NB, true, false, false, false, LB, HW>(a, t, dem, ny, kw, L, nsl);
    }
}

template <bool LB>
__device__ void ex_cells(const ExAgent& a, const dgen_tariff& t, const dgen_demand* dem, int ny, double kw,
                         const ExLds& L, int nsl) {
    // two runs per wave when the analysis years and the no-system lane fit
    // a half-wave
    if (ny + 1 <= 32) ex_cells_h<LB, true>(a, t, dem, ny, kw, L, nsl);
    else ex_cells_h<LB, false>(a, t, dem, ny, kw, L, nsl);
}

// The same bill with the periods' credits, billed kWh and shares in
// registers (P <= PREG, the common case): loops run to the compile-time bound
// under the guard p < P, so every sum keeps ex_year_bill's order (and the
// oracle's); the bins' loads of a month issue together.
__device__ __forceinline__ double ex_month_charge_reg(const dgen_tariff& t, int m, const double (&u)[PREG],
                                                      double peak) {
    const int P = t.P;
    double U = 0.0;
#pragma unroll
    for (int p = 0; p < PREG; p++)
        if (p < P) U += u[p];
    const bool pos = U > 0.0;
    if (t.T == 1) {
        double charge = 0.0;
#pragma unroll
        for (int p = 0; p < PREG; p++)
            if (p < P) charge += u[p] * t.buy[p][0];
        return pos ? charge : 0.0;
    }
    const double days = (double)c_days_in_month[m];
    const double f_pk = (t.unit == 1 || t.unit == 3) ? peak : 1.0;
    const double f_days = (t.unit == 2 || t.unit == 3) ? days : 1.0;
    const double scale = f_pk * f_days;
    double fr[PREG];
#pragma unroll
    for (int p = 0; p < PREG; p++) fr[p] = p < P ? u[p] / U : 0.0;
    double charge = 0.0, prev = 0.0;
    for (int k = 0; k < t.T; k++) {
        const double hi = (k == t.T - 1) ? INFINITY : t.cap[k] * scale;
        const double top = U < hi ? U : hi;
        const double amt0 = top - prev;
        const double amt = amt0 < 0.0 ? 0.0 : amt0;
        prev = hi > prev ? hi : prev;
#pragma unroll
        for (int p = 0; p < PREG; p++)
            if (p < P) charge += fr[p] * amt * t.buy[p][k];
    }
    return pos ? charge : 0.0;
}

template <bool LB>
__device__ __forceinline__ double ex_year_bill_reg(const ExAgent& a, const dgen_tariff& t, const dgen_demand* dem,
                                                   int yl, const ExLds& L) {
    const int P = t.P;
    const ExB B = ex_b<LB>(L.bins, L.bny, L.ptab, L.dcb);
    double credit[PREG], u[PREG];
#pragma unroll
    for (int p = 0; p < PREG; p++) { credit[p] = 0.0; u[p] = 0.0; }
    const bool ts = a.has_ts && t.mo == 2;
    double total = 0.0, carry = 0.0, dtot = 0.0;
    for (int m = 0; m < 12; m++) {
        const double* bn = B.bins + ((size_t)yl * 12 + m) * 2 * P;
        const double* cm = B.cmax + ((size_t)yl * 12 + m) * P;
        double b0[PREG], b1[PREG], c0[PREG];
#pragma unroll
        for (int p = 0; p < PREG; p++) {
            b0[p] = p < P ? bn[p] : 0.0;
            b1[p] = p < P ? bn[P + p] : 0.0;
            c0[p] = p < P ? cm[p] : 0.0;
        }
        double pk = 0.0;
#pragma unroll
        for (int p = 0; p < PREG; p++)
            if (p < P) pk = c0[p] > pk ? c0[p] : pk;
        double bill = t.fixed;
        if (t.mo == 0) {
#pragma unroll
            for (int p = 0; p < PREG; p++) {
                if (p < P) {
                    const double n = b0[p];
                    const double cp = credit[p];
                    const double use = n < cp ? n : cp;
                    const bool ps = n >= 0.0;
                    u[p] = ps ? n - use : 0.0;
                    credit[p] = ps ? cp - use : cp + -n;
                }
            }
            bill += ex_month_charge_reg(t, m, u, pk);
            if (m == 11) {
                double cc = 0.0;
#pragma unroll
                for (int p = 0; p < PREG; p++)
                    if (p < P) cc += credit[p];
                bill -= cc * a.yearend;
            }
        } else if (t.mo == 1) {
            double cr = 0.0;
#pragma unroll
            for (int p = 0; p < PREG; p++) {
                if (p < P) {
                    const double n = b0[p];
                    u[p] = n > 0.0 ? n : 0.0;
                    cr += (n < 0.0 ? -n : 0.0) * t.sell[p][0];
                }
            }
            const double e = ex_month_charge_reg(t, m, u, pk) - cr - carry;
            carry = e < 0.0 ? -e : 0.0;
            bill += e < 0.0 ? 0.0 : e;
        } else if (t.mo == 4) {
            double cr = 0.0;
#pragma unroll
            for (int p = 0; p < PREG; p++) {
                if (p < P) {
                    u[p] = b0[p];
                    cr += b1[p] * t.sell[p][0];
                }
            }
            bill += ex_month_charge_reg(t, m, u, pk) - cr;
        } else {
            double cr = 0.0;
#pragma unroll
            for (int p = 0; p < PREG; p++)
                if (p < P) u[p] = b0[p];
            const double charge = ex_month_charge_reg(t, m, u, pk);
            if (ts) {
#pragma unroll
                for (int p = 0; p < PREG; p++)
                    if (p < P) cr += b1[p];
            } else {
#pragma unroll
                for (int p = 0; p < PREG; p++)
                    if (p < P) cr += b1[p] * t.sell[p][0];
            }
            if (t.mo == 3) {
                const double e = charge - cr - carry;
                carry = e < 0.0 ? -e : 0.0;
                bill += e < 0.0 ? 0.0 : e;
            } else {
                bill += charge;
                bill -= cr;
            }
        }
        total += bill;
        if (dem) {
            double c = ex_dc_tier(pk, dem->flat_cap[m], dem->flat_price[m], dem->flat_nt[m]);
            for (int q = 0; q < DCP; q++) {
                double v = 0.0;
                for (int p = 0; p < P; p++) {
                    const double w = B.dcm[(((size_t)yl * 12 + m) * P + p) * DCP + q];
                    v = w > v ? w : v;
                }
                c += ex_dc_tier(v, dem->tou_cap[q], dem->tou_price[q], dem->tou_nt[q]);
            }
            dtot += c;
        }
    }
    return dem ? total + dtot : total;
}

// oracle year_bill (+ year_demand) of year y0 + yl from its cells
template <bool LB>
__device__ __forceinline__ double ex_year_bill(const ExAgent& a, const dgen_tariff& t, const dgen_demand* dem, int yl,
                               const ExLds& L) {
    if (t.P <= PREG) return ex_year_bill_reg<LB>(a, t, dem, yl, L);
    const int P = t.P;
    const ExB B = ex_b<LB>(L.bins, L.bny, L.ptab, L.dcb);
    double* credit = ex_yr() + (size_t)yl * 3 * MAXP;     // credit, u, shares
    double* u = credit + MAXP;
    for (int p = 0; p < MAXP; p++) credit[p] = 0.0;
    const bool ts = a.has_ts && t.mo == 2;
    double total = 0.0, carry = 0.0, dtot = 0.0;
    for (int m = 0; m < 12; m++) {
        const double* bn = B.bins + ((size_t)yl * 12 + m) * 2 * P;
        const double* cm = B.cmax + ((size_t)yl * 12 + m) * P;
        double pk = 0.0;
        for (int p = 0; p < P; p++) pk = cm[p] > pk ? cm[p] : pk;
        double bill = t.fixed;
        if (t.mo == 0) {
            for (int p = 0; p < P; p++) {     // oracle's branches as selects (same operations)
                const double n = bn[p];
                const double cp = credit[p];
                const double use = n < cp ? n : cp;
                const bool pos = n >= 0.0;
                u[p] = pos ? n - use : 0.0;
                credit[p] = pos ? cp - use : cp + -n;
            }
            bill += ex_month_charge(t, m, u, pk, u + MAXP);
            if (m == 11) {
                double cc = 0.0;
                for (int p = 0; p < P; p++) cc += credit[p];
                bill -= cc * a.yearend;
            }
        } else if (t.mo == 1) {
            double cr = 0.0;
            for (int p = 0; p < P; p++) {
                const double n = bn[p];
                u[p] = n > 0.0 ? n : 0.0;
                cr += (n < 0.0 ? -n : 0.0) * t.sell[p][0];
            }
            const double e = ex_month_charge(t, m, u, pk, u + MAXP) - cr - carry;
            carry = e < 0.0 ? -e : 0.0;
            bill += e < 0.0 ? 0.0 : e;
        } else if (t.mo == 4) {
            double cr = 0.0;
            for (int p = 0; p < P; p++) {
                u[p] = bn[p];
                cr += bn[P + p] * t.sell[p][0];
            }
            bill += ex_month_charge(t, m, u, pk, u + MAXP) - cr;
        } else {
            double cr = 0.0;
            for (int p = 0; p < P; p++) u[p] = bn[p];
            const double charge = ex_month_charge(t, m, u, pk, u + MAXP);
            if (ts) {
                for (int p = 0; p < P; p++) cr += bn[P + p];
            } else {
                for (int p = 0; p < P; p++) cr += bn[P + p] * t.sell[p][0];
            }
            if (t.mo == 3) {
                const double e = charge - cr - carry;
                carry = e < 0.0 ? -e : 0.0;
                bill += e < 0.0 ? 0.0 : e;
            } else {
                bill += charge;
                bill -= cr;
            }
        }
        total += bill;
        if (dem) {
            // flat peak: the month's largest import (from 0) = pk; TOU peaks:
            // the bins' per-period maxima combined
            double c = ex_dc_tier(pk, dem->flat_cap[m], dem->flat_price[m], dem->flat_nt[m]);
            for (int q = 0; q < DCP; q++) {
                double v = 0.0;
                for (int p = 0; p < P; p++) {
                    const double w = B.dcm[(((size_t)yl * 12 + m) * P + p) * DCP + q];
                    v = w > v ? w : v;
                }
                c += ex_dc_tier(v, dem->tou_cap[q], dem->tou_price[q], dem->tou_nt[q]);
            }
            dtot += c;
        }
    }
    return dem ? total + dtot : total;
}

// oracle orc_cashloan over aev[0 .. N] (thread 0); returns npv, payback
__device__ void ex_cashloan(const dgen_agents& A, const dgen_cfg& cfg, int64_t i, int N, double C, const double* aev,
                            double* cf_payback, double* cf_ev, double* atcf, double* npv_out, double* pb_out) {
    const bool is_res = (A.flags[i] & 1) != 0;
    const int market = is_res ? 0 : 1;
    const int depr_type = is_res ? 0 : 2;
    const double infl = (A.inflation[i] * 100.0) * 0.01;
    const double real = (A.real_discount[i] * 100.0) * 0.01;
    const double nom = (1.0 + real) * (1.0 + infl) - 1.0;
    const double fed = ((A.tax_rate[i] * 100.0) * 0.7) * 0.01, sta = ((A.tax_rate[i] * 100.0) * 0.3) * 0.01;
    const double debt = (100.0 - (A.down_payment[i] * 100.0)) * 0.01 * C;
    const double r = cfg.loan_rate_pct * 0.01;
    const int term = A.loan_term[i];
    double pmt = 0.0;
    if (term > 0 && debt != 0.0) {
        if (r != 0.0) {
            const double f = pow_seq(1.0 + r, term);
            pmt = debt * r / (1.0 - 1.0 / f);
        } else {
            pmt = debt / (double)term;
        }
    }
    double itc = A.itc_frac[i] * 0.01 * C;
    if (itc > cfg.itc_fed_max) itc = cfg.itc_fed_max;
    const double basis = C - 0.5 * itc;
    const double ins = cfg.insurance_rate_pct * 0.01 * C;
    double balance = debt;
    atcf[0] = -(C - debt);
    cf_payback[0] = -C;
    cf_ev[0] = 0.0;
    for (int y = 1; y <= N; y++) {
        const double ev = aev[y];
        const double oe = ins * pow_seq(1.0 + infl, y - 1);
        double interest = 0.0, payment = 0.0;
        if (y <= term && pmt != 0.0) {
            interest = balance * r;
            payment = pmt;
            balance = balance - (pmt - interest);
        }
        const double itc_y = (y == 1) ? itc : 0.0;
        double sta_tax = 0.0, fed_tax = 0.0;
        if (market != 0) {
            const double dep = depr_frac(depr_type, y, cfg.depr_sl_years) * basis;
            sta_tax = sta * (ev - oe - interest - dep);
            fed_tax = fed * (ev - oe - interest - dep - sta_tax);
        }
        const double taxsav = itc_y - sta_tax - fed_tax;
        atcf[y] = ev - oe - payment + taxsav;
        cf_payback[y] = ev - oe + taxsav;
        cf_ev[y] = ev;
    }
    const double rr = 1.0 / (1.0 + nom);
    double acc = 0.0;
    for (int y = N; y > 0; y--) acc = rr * acc + atcf[y];
    *npv_out = atcf[0] + acc * rr;
    double cum = cf_payback[0];
    double pb = 1e99;
    for (int y = 1; y <= N; y++) {
        cum += cf_payback[y];
        if (cum > 0.0) {
            pb = (cf_payback[y] != 0.0) ? (double)y - cum / cf_payback[y] : (double)y - 0.5;
            break;
        }
    }
    *pb_out = pb;
}

// orc_cashloan with the years on the block's threads: thread y (1 .. N)
// forms year y's flows with the sequential form's operations (the loan
// balance entering year y by the same recursion from year 1), thread 0 then
// runs the NPV (Horner from year N) and payback chains over them.  Returns
// npv, payback through sc[1], sc[2] (LDS; read after a barrier).
__device__ void ex_cashloan_par(const dgen_agents& A, const dgen_cfg& cfg, int64_t i, int N, double C,
                                const double* aev, double* cf_payback, double* cf_ev, double* atcf, double* sc) {
    const bool is_res = (A.flags[i] & 1) != 0;
    const int market = is_res ? 0 : 1;
    const int depr_type = is_res ? 0 : 2;
    const double infl = (A.inflation[i] * 100.0) * 0.01;
    const double real = (A.real_discount[i] * 100.0) * 0.01;
    const double nom = (1.0 + real) * (1.0 + infl) - 1.0;
    const double fed = ((A.tax_rate[i] * 100.0) * 0.7) * 0.01, sta = ((A.tax_rate[i] * 100.0) * 0.3) * 0.01;
    const double debt = (100.0 - (A.down_payment[i] * 100.0)) * 0.01 * C;
    const double r = cfg.loan_rate_pct * 0.01;
    const int term = A.loan_term[i];
    double pmt = 0.0;
    if (term > 0 && debt != 0.0) {
        if (r != 0.0) {
            const double f = pow_seq(1.0 + r, term);
            pmt = debt * r / (1.0 - 1.0 / f);
        } else {
            pmt = debt / (double)term;
        }
    }
    double itc = A.itc_frac[i] * 0.01 * C;
    if (itc > cfg.itc_fed_max) itc = cfg.itc_fed_max;
    const double basis = C - 0.5 * itc;
    const double ins = cfg.insurance_rate_pct * 0.01 * C;
    const int y = (int)threadIdx.x;
    if (y == 0) {
        atcf[0] = -(C - debt);
        cf_payback[0] = -C;
        cf_ev[0] = 0.0;
    } else if (y <= N) {
        double balance = debt;
        const bool pays = pmt != 0.0;
        for (int k = 1; k < y; k++)
            if (k <= term && pays) balance = balance - (pmt - balance * r);
        const double ev = aev[y];
        const double oe = ins * pow_seq(1.0 + infl, y - 1);
        double interest = 0.0, payment = 0.0;
        if (y <= term && pays) {
            interest = balance * r;
            payment = pmt;
        }
        const double itc_y = (y == 1) ? itc : 0.0;
        double sta_tax = 0.0, fed_tax = 0.0;
        if (market != 0) {
            const double dep = depr_frac(depr_type, y, cfg.depr_sl_years) * basis;
            sta_tax = sta * (ev - oe - interest - dep);
            fed_tax = fed * (ev - oe - interest - dep - sta_tax);
        }
        const double taxsav = itc_y - sta_tax - fed_tax;
        atcf[y] = ev - oe - payment + taxsav;
        cf_payback[y] = ev - oe + taxsav;
        cf_ev[y] = ev;
    }
    __syncthreads();
    if (y == 0) {
        const double rr = 1.0 / (1.0 + nom);
        double acc = 0.0;
        for (int k = N; k > 0; k--) acc = rr * acc + atcf[k];
        sc[1] = atcf[0] + acc * rr;
        double cum = cf_payback[0];
        double pb = 1e99;
        for (int k = 1; k <= N; k++) {
            cum += cf_payback[k];
            if (cum > 0.0) {
                pb = (cf_payback[k] != 0.0) ? (double)k - cum / cf_payback[k] : (double)k - 0.5;
                break;
            }
        }
        sc[2] = pb;
    }
}

__global__ void __launch_bounds__(EX_THREADS) __attribute__((amdgpu_waves_per_eu(2)))
k_size_exact(dgen_tables T, dgen_agents A, dgen_outputs O, dgen_cfg cfg, const int32_t* __restrict__ list,
             char* exws, int64_t wsb, int lds_ny, int32_t* next) {
    const int cnt = list[0];
    // next (a zeroed counter): the blocks take the listed agents one at a
    // time from it, so a block that drew short searches takes more of them
    // (the grid is the device's resident blocks); nullptr: block b takes
    // agents b, b + grid, ...
    __shared__ int s_next;
    ExLds L;
    {
        char* g = exws + (size_t)blockIdx.x * (size_t)wsb;
        const int P = T.max_periods > 0 && T.max_periods <= MAXP ? T.max_periods : MAXP;
        const bool dcb = cfg.skip_demand_charges == 0 && T.n_demand > 0;
        L.Lp = reinterpret_cast<double*>(g);
        L.Cp = L.Lp + NH;
        L.Tp = L.Cp + NH;
        L.hl = reinterpret_cast<uint16_t*>(L.Tp + NH);
        L.bins = reinterpret_cast<double*>(g + ex_ws_base());
        L.cmax = L.bins + (size_t)(MAXY + 1) * 12 * 2 * P;
        L.dcm = dcb ? L.cmax + (size_t)(MAXY + 1) * 12 * P : nullptr;
        L.bny = MAXY + 1;
        L.ptab = P;
        L.dcb = dcb;
        double* d = dyn_lds;
        L.stg = ex_stg(0);
        L.yr = ex_yr();
        L.res = ex_res();
        L.hoff = ex_hoff();
        if (lds_ny > 0) L.bny = lds_ny;   // the bins of lds_ny (>= every listed agent's N + 1) years in LDS (ex_b<true>)
    }
    double* const aev = ex_res();
    double* const bw = aev + (MAXY + 1);
    double* const bwo = aev + 2 * (MAXY + 1);
    double* const cfpb = aev + 3 * (MAXY + 1);
    double* const cfev = aev + 4 * (MAXY + 1);
    double* const atcf = aev + 5 * (MAXY + 1);
    double* const sc = aev + 6 * (MAXY + 1);          // [0] wo1, [1] npv, [2] payback
    ExAgent a;
    a.demand = T.demand;
    a.n_demand = T.n_demand;
    a.dc_on = cfg.skip_demand_charges == 0;
    a.yearend = cfg.nm_yearend_sell_rate;
    for (int w0 = blockIdx.x;; w0 += gridDim.x) {
        int w = w0;
        if (next) {
            if (threadIdx.x == 0) s_next = atomicAdd(next, 1);
            __syncthreads();
            w = __builtin_amdgcn_readfirstlane(s_next);
        }
        if (w >= cnt) break;
        const int64_t i = __builtin_amdgcn_readfirstlane(list[1 + w]);
        const int lr = A.load_row[i], cr = A.cf_row[i];
        const double kwh = A.load_kwh[i];
        const uint8_t fl = A.flags[i];
        const bool is_ca = (fl & 2) != 0;
        const int wr = A.wholesale_row[i];
        a.N = A.econ_life[i];
        a.has_ts = !is_ca && wr >= 0 && T.wholesale != nullptr;
        a.rate_base = 1.0 + (A.inflation[i] * 100.0) * 0.01 + (A.escalator[i] * 100.0) * 0.01;
        a.sys_base = 1.0 - (A.pv_deg[i] * 100.0) * 0.01;
        const double S = T.shape_sum[lr];
        const float* sh = T.shapes + (int64_t)lr * NH;
        const double* wrow = a.has_ts ? T.wholesale + (int64_t)wr * NH : nullptr;
        const double pmul = A.price_mult[i];
        const int32_t* cfr = T.cfs + (int64_t)cr * NH;
        const double naep0 = T.cf_naep[cr];
        const double max_load = kwh / naep0;
        const double low = max_load * 0.8, high = max_load * 1.25;
        const double span = high - low;
        const double tl = (span > 1.0 ? span : 1.0) * 1e-3;
        const double fl_tl = floor(tl);
        const double xatol = fl_tl < 2.0 ? 2.0 : fl_tl;
        const dgen_switch* sw = T.switches + A.sw_solar_off[i];
        const int sw_cnt = A.sw_solar_cnt[i];
        int tariff = __builtin_amdgcn_readfirstlane(A.tariff0[i]), switched = 0;
        int status = O.status[i] | T.tariffs[tariff].flags;
        int wo_tag = -1;
        double wo1 = 0.0, total = 0.0, npv = 0.0, pb = 0.0;
        auto perf = [&](double kw) __attribute__((always_inline)) -> double {
            double otc = 0.0;
            if (kw > 0.0) {
                int nt;
                otc = rate_switch(sw, sw_cnt, kw, &nt);
                if (nt >= 0) {
                    tariff = __builtin_amdgcn_readfirstlane(nt);
                    switched = 1;
                    status |= T.tariffs[tariff].flags;
                }
            }
            const dgen_tariff& t = T.tariffs[tariff];
            const dgen_demand* dem = (a.dc_on && t.dc > 0 && t.dc <= a.n_demand) ? a.demand + (t.dc - 1) : nullptr;
            PH_T0(tw);
            const bool need_wo = wo_tag != tariff;
            if (need_wo) {
                // the tariff's hour list (its no-system bill, orc_ur5's wo1,
                // comes with this evaluation's bins below)
                __syncthreads();                          // the previous list's and bins' readers
                ex_hour_lists(t, L, sh, S, kwh, cfr, wrow, pmul);
                ex_handoff();
            }
            // (phase slots 4, 5, 6, 10, 11: the exact re-run's cells, year
            // bills, cash flow, tariff set-up and evaluations; DGEN_PHASE_PROF)
            PH_ADD(10, tw, threadIdx.x == 0);
            PH_CNT(11, 1, threadIdx.x == 0);
            // the analysis years' bins (lane = year, N < MAXY + 1 <= 64) and,
            // with a new tariff, the no-system year's on lane N, then a
            // thread per year bills them
            PH_T0(tc);
            if (lds_ny > 0) ex_cells<true>(a, t, dem, a.N, kw, L, need_wo ? a.N : -1);
            else ex_cells<false>(a, t, dem, a.N, kw, L, need_wo ? a.N : -1);
            ex_handoff();
            PH_ADD(4, tc, threadIdx.x == 0);
            PH_T0(ty);
            const int y = (int)threadIdx.x;
            if (y < a.N || (need_wo && y == a.N)) {
                const double wb = lds_ny > 0 ? ex_year_bill<true>(a, t, dem, y, L) : ex_year_bill<false>(a, t, dem, y, L);
                if (y < a.N) bw[y + 1] = wb;
                else sc[0] = wb;
            }
            __syncthreads();
            if (need_wo) {
                wo1 = ex_uniform(sc[0]);
                wo_tag = tariff;
            }
            if (y < a.N) {
                const double r = pow_seq(a.rate_base, y);
                const double wv = bw[y + 1] * r;
                const double wo = wo1 * r;
                bw[y + 1] = wv;
                bwo[y + 1] = wo;
                aev[y + 1] = wo - wv;
            }
            __syncthreads();
            PH_ADD(5, ty, threadIdx.x == 0);
            PH_T0(tf);
            total = ((A.capex[i] * kw + 0.0) * A.ccm[i]) + 0.0 + otc;
            if (threadIdx.x == 0) {
                aev[0] = 0.0;
                bw[0] = 0.0;
                bwo[0] = 0.0;
            }
            ex_cashloan_par(A, cfg, i, a.N, total, aev, cfpb, cfev, atcf, sc);
            __syncthreads();
            PH_ADD(6, tf, threadIdx.x == 0);
            npv = ex_uniform(sc[1]);
            pb = ex_uniform(sc[2]);
            return -npv;
        };
        int nfev = 0;
        double x_last = 0.0;
        const double kw_star = brent_bounded(perf, low, high, xatol, &nfev, &x_last);
        __syncthreads();
        // the driver's last-evaluation capture (ff:449-474), as k_size writes it
        const int64_t row = i * (MAXY + 1);
        for (int k = threadIdx.x; k <= a.N; k += blockDim.x) {
            O.cash_flow[row + k] = k == 0 ? -total : cfpb[k];
            O.cfev_pv[row + k] = k == 0 ? 0.0 : cfev[k];
            O.bill_w_pv[row + k] = bw[k];
            O.bill_wo_pv[row + k] = bwo[k];
        }
        if (threadIdx.x == 0) {
            O.npv[i] = npv;
            O.payback_raw[i] = pb;
            const double pbr = isfinite(pb) ? pb : 30.1;
            O.payback_period[i] = rint(pbr * 10.0) / 10.0;
            O.first_with[i] = bw[1];
            O.first_without[i] = wo1;
            O.price_per_kwh[i] = wo1 / kwh;
            O.system_kw[i] = kw_star;
            O.x_last[i] = x_last;
            O.nfev[i] = nfev;
            O.tariff_final[i] = tariff;
            O.switched[i] = switched;
            O.status[i] = status;
        }
        __syncthreads();
    }
}
#endif  // !DGEN_TU_SEARCH

}  // namespace

// The year-lane search kernels (k_size_w, k_dc_env, k_nb_env) have external
// linkage so that dgen_amd/build.py can compile them in a translation unit of
// their own (DGEN_TU_SEARCH) with the code generator's scheduling options for
// them, while this file's other kernels and the host API build as
// DGEN_TU_MAIN, where the three are declarations only.  Without either macro
// the file is one translation unit, as before (the ablation builds).
#ifdef DGEN_TU_SEARCH
namespace dgen_srch {
#define DGEN_INST_SIZE(L, D, N, P)                                                                       \
    template __global__ void k_size_w<L, D, N, P>(dgen_tables, dgen_agents, dgen_outputs, dgen_cfg,   \
                                                  int64_t, int64_t, int64_t, void*, char*, int, double*);
#if !DGEN_NO2_SIZE
DGEN_INST_SIZE(32, false, false, false)
DGEN_INST_SIZE(32, false, true, false)
#endif
#if !DGEN_NO2_SIZE_DC
DGEN_INST_SIZE(32, true, true, false)
DGEN_INST_SIZE(32, true, false, false)
#endif
#if !DGEN_NO2_SIZE_PK
DGEN_INST_SIZE(32, true, true, true)
#endif
DGEN_INST_SIZE(64, false, false, false)
DGEN_INST_SIZE(64, false, true, false)
DGEN_INST_SIZE(64, true, true, false)
DGEN_INST_SIZE(64, true, false, false)
DGEN_INST_SIZE(64, true, true, true)
#undef DGEN_INST_SIZE
template __global__ void k_dc_env<2>(dgen_tables, dgen_agents, dgen_cfg, int64_t, int64_t, void*);
template __global__ void k_dc_env<4>(dgen_tables, dgen_agents, dgen_cfg, int64_t, int64_t, void*);
template __global__ void k_dc_env<DGEN_DCP>(dgen_tables, dgen_agents, dgen_cfg, int64_t, int64_t, void*);
template __global__ void k_nb_env<32>(dgen_tables, dgen_agents, int64_t, int64_t, char*);
}  // namespace dgen_srch
#else

// ===========================================================================
// C-ABI
// ===========================================================================
// Each dgen_size_agents call records, per chunk, five events: around k_size
// on the caller's stream (0, 1) and around k_hourly_batt / k_batt_finance on
// the ctx's second stream (2, 3, 4).  Kernel time = sum over chunks.
struct dgen_ctx {
    int device;
    dgen_cfg cfg;
    static constexpr int RING = 16;
    static constexpr int MAXCH = 16;
    hipEvent_t ev[RING][MAXCH][5];
    int nch[RING];     // chunks recorded in the slot
    hipEvent_t fork, join;
    hipStream_t s2;    // hourly + finance stream of the chunk pipeline
    static constexpr int MAXSPLIT = 4;
    hipStream_t sx[MAXSPLIT - 1];       // the hourly scan's other parts' streams
    hipEvent_t hb_join[MAXSPLIT - 1];
    hipStream_t st[MAXSPLIT];           // each part's TS scan (k_hourly_batt<TS>), beside its NB scan
    hipEvent_t ts_join[MAXSPLIT];
    int hb_split;      // parts of a chunk's hourly scan, each on its own stream (1..4; DGEN_HB_SPLIT)
    int hb_nem;        // 1: batches without scratch slots run the bins-only scan (DGEN_HB_NEM=0: off)
    int ts_scan;       // 1: the TS sell-rate agents' split built in their own scan (DGEN_TS_SCAN=0: off, A/B)
    int dc_pre;        // 1: the first-evaluation tariff's demand envelopes prebuilt by k_dc_env (DGEN_DC_PREBUILD=0: off)
    int nb_pre;        // 1: its net-billing split prebuilt by k_nb_env (DGEN_NB_PREBUILD=0: off, k_size builds it)
    int64_t nem_hi;    // rows [0, nem_hi) of a batch hold no scratch-slot agent (dgen_set_nem_rows)
    int64_t ts_lo, ts_hi;   // the batch rows holding every TS-capable agent (dgen_set_ts_rows)
    int chunks;        // pipeline depth (dgen_set_pipeline)
    int hb_months;     // months per k_hourly_batt launch (dgen_set_hourly_segment)
    int battery;       // PV+battery forward run (dgen_set_battery)
    int nb_scan;       // battery-case split in the hourly scan: its per-month entry capacity, 0 = off (dgen_set_nb_scan)
    int32_t last_paths[DGEN_PATHS_N] = {0};   // the record forms the last dgen_size_agents call took (dgen_last_paths)
    int head;          // next ring slot to record
    int pending;       // recorded, not yet folded
    double sum_ms[3];
    int64_t count;
    void* dc_buf = nullptr;   // demand-charge envelopes, DCW_BYTES per agent (grown on demand)
    size_t dc_cap = 0;
    void* rows_buf = nullptr; // dgen_state_hourly_rows' per-agent scalars, 16 B per agent (grown on demand)
    size_t rows_cap = 0;
    void* dcr_buf = nullptr;  // battery-case demand records, DCR_BYTES per scratch slot (grown on demand)
    size_t dcr_cap = 0;
    int dcr_enable = DCR_CAP; // kept hours per record, 0 = off (dgen_set_dc_records)
    // certified Brent paths (dgen_set_exact): the search traces, the listed
    // agents per chunk, the exact re-run's per-block hour scratch
    int exact = 1;
    char* ex_ws = nullptr;         // [EX_BLOCKS][ex_ws_bytes(P, demand)]
    size_t ex_ws_cap = 0;
    int lds_max = 65536;           // the device's LDS per work-group (hipDeviceAttributeMaxSharedMemoryPerBlock)
    double* bt_buf = nullptr;      // [n][BT_MAX] objective values
    size_t bt_cap = 0;
    int32_t* ex_list = nullptr;    // chunk j: [i0 + j] count, then its rows
    size_t ex_list_cap = 0;
    int32_t* ex_next = nullptr;    // [MAXCH] the re-run's work counters (k_size_exact's next)
    int ex_dyn = 1;                // 0: static agent order over EX_BLOCKS blocks (DGEN_EX_DYN=0, A/B)
    int n_cu = 256;                // the device's compute units
    int ex_last_nch = 0;
    int64_t ex_last_off[MAXCH] = {0};
};

static int fold_one(dgen_ctx* c, int slot) {
    const int k = c->nch[slot];
    HIP_TRY(hipEventSynchronize(c->ev[slot][k - 1][4]));
    for (int j = 0; j < k; j++) {
        hipEvent_t* e = c->ev[slot][j];
        float a = 0.f, b = 0.f, f = 0.f;
        HIP_TRY(hipEventElapsedTime(&a, e[0], e[1]));
        HIP_TRY(hipEventElapsedTime(&b, e[2], e[3]));
        HIP_TRY(hipEventElapsedTime(&f, e[3], e[4]));
        c->sum_ms[0] += a;
        c->sum_ms[1] += b;
        c->sum_ms[2] += f;
    }
    c->count++;
    return 0;
}

extern "C" {

#if DGEN_PHASE_PROF
__attribute__((visibility("default"))) int dgen_phase_read(uint64_t* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(uint64_t) * 16) != hipSuccess) return -1;
    if (reset) {
        static const uint64_t z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

int32_t dgen_abi_version(void) { return DGEN_ABI_VERSION; }

int32_t dgen_last_error(char* buf, size_t n) {
    if (!buf || n == 0) return DGEN_E_ARG;
    snprintf(buf, n, "%s", g_err);
    return DGEN_OK;
}

int32_t dgen_open(int32_t device, const dgen_cfg* cfg, dgen_ctx** out) {
    if (!cfg || !out) { set_err("dgen_open: null argument"); return DGEN_E_ARG; }
    if (cfg->skip_demand_charges != 0 && cfg->skip_demand_charges != 1) {
        set_err("dgen_open: skip_demand_charges must be 1 (the reference, ff:35) or 0 (extension)");
        return DGEN_E_ARG;
    }
    if (!(cfg->batt_v_nom > 0.0) || !(cfg->batt_q_full > 0.0) || !(cfg->batt_eta_in > 0.0) ||
        !(cfg->batt_eta_out > 0.0) || cfg->depr_sl_years < 1) {
        set_err("dgen_open: invalid battery/loan configuration");
        return DGEN_E_ARG;
    }
    if (cfg->batt_month_floor != 0 && cfg->batt_month_floor != 1) {
        set_err("dgen_open: batt_month_floor must be 0 or 1");
        return DGEN_E_ARG;
    }
    if (cfg->batt_loss_model != 0 && cfg->batt_loss_model != 1) {
        set_err("dgen_open: batt_loss_model must be 0 (constant efficiencies) or 1 (Li-ion loss model)");
        return DGEN_E_ARG;
    }
    if (cfg->batt_loss_model == 1 &&
        (!(cfg->batt_r_cell >= 0.0) || !(cfg->batt_conv_eff > 0.0 && cfg->batt_conv_eff <= 1.0) ||
         !(cfg->batt_v_cell_empty > 0.0) || !(cfg->batt_v_cell_full > 0.0))) {
        set_err("dgen_open: loss model needs batt_r_cell >= 0, 0 < batt_conv_eff <= 1 and positive cell voltages");
        return DGEN_E_ARG;
    }
    if (cfg->batt_update_hours != 24 && cfg->batt_update_hours != 1) {
        set_err("dgen_open: batt_update_hours must be 24 (a plan per day) or 1 (re-planned every hour)");
        return DGEN_E_ARG;
    }
    HIP_TRY(hipSetDevice(device));
    dgen_ctx* c = new (std::nothrow) dgen_ctx();
    if (!c) { set_err("dgen_open: out of host memory"); return DGEN_E_ARG; }
    c->device = device;
    c->cfg = *cfg;
    {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, device) == hipSuccess && v > 0)
            c->lds_max = v;
        else
            (void)hipGetLastError();
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && v > 0)
            c->n_cu = v;
        else
            (void)hipGetLastError();
        const char* e = getenv("DGEN_EX_DYN");
        if (e && e[0] == '0') c->ex_dyn = 0;
    }
    c->head = 0; c->pending = 0; c->count = 0;
    c->chunks = DGEN_DEFAULT_CHUNKS;
    c->hb_months = DGEN_DEFAULT_HOURLY_MONTHS;
    c->battery = 1;
    c->nb_scan = DGEN_NB_CAPM;
    c->sum_ms[0] = c->sum_ms[1] = c->sum_ms[2] = 0.0;
    {
        const char* v = getenv("DGEN_HB_SPLIT");
        c->hb_split = (v && v[0] >= '1' && v[0] <= '4') ? v[0] - '0' : DGEN_DEFAULT_HOURLY_SPLIT;
        const char* w = getenv("DGEN_HB_NEM");
        c->hb_nem = (w && w[0] == '0') ? 0 : 1;
        const char* x = getenv("DGEN_TS_SCAN");
        c->ts_scan = (x && x[0] == '0') ? 0 : 1;
        const char* y = getenv("DGEN_DC_PREBUILD");
        c->dc_pre = (y && y[0] == '0') ? 0 : 1;
        const char* z = getenv("DGEN_NB_PREBUILD");
        c->nb_pre = (z && z[0] == '0') ? 0 : 1;
    }
    c->ts_lo = 0;
    c->ts_hi = INT64_MAX;
    c->nem_hi = 0;
    hipError_t e = hipStreamCreateWithFlags(&c->s2, hipStreamNonBlocking);
    for (int k = 0; k < dgen_ctx::MAXSPLIT - 1 && e == hipSuccess; k++) {
        e = hipStreamCreateWithFlags(&c->sx[k], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->hb_join[k], hipEventDisableTiming);
    }
    for (int k = 0; k < dgen_ctx::MAXSPLIT && e == hipSuccess; k++) {
        e = hipStreamCreateWithFlags(&c->st[k], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ts_join[k], hipEventDisableTiming);
    }
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->join, hipEventDisableTiming);
    for (int r = 0; r < dgen_ctx::RING && e == hipSuccess; r++) {
        c->nch[r] = 0;
        for (int j = 0; j < dgen_ctx::MAXCH && e == hipSuccess; j++)
            for (int k = 0; k < 5 && e == hipSuccess; k++) e = hipEventCreate(&c->ev[r][j][k]);
    }
    if (e != hipSuccess) {
        set_err("dgen_open: stream/event creation failed: %s", hipGetErrorString(e));
        delete c;   // leaks the handles created so far; the process is failing anyway
        return DGEN_E_HIP;
    }
    *out = c;
    return DGEN_OK;
}

int32_t dgen_close(dgen_ctx* c) {
    if (!c) return DGEN_OK;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->s2);
    for (int k = 0; k < dgen_ctx::MAXSPLIT - 1; k++) (void)hipStreamSynchronize(c->sx[k]);
    for (int k = 0; k < dgen_ctx::MAXSPLIT; k++) (void)hipStreamSynchronize(c->st[k]);
    for (int r = 0; r < dgen_ctx::RING; r++)
        for (int j = 0; j < dgen_ctx::MAXCH; j++)
            for (int k = 0; k < 5; k++) (void)hipEventDestroy(c->ev[r][j][k]);
    (void)hipEventDestroy(c->fork);
    (void)hipEventDestroy(c->join);
    (void)hipStreamDestroy(c->s2);
    for (int k = 0; k < dgen_ctx::MAXSPLIT - 1; k++) {
        (void)hipStreamDestroy(c->sx[k]);
        (void)hipEventDestroy(c->hb_join[k]);
    }
    for (int k = 0; k < dgen_ctx::MAXSPLIT; k++) {
        (void)hipStreamDestroy(c->st[k]);
        (void)hipEventDestroy(c->ts_join[k]);
    }
    if (c->dc_buf) (void)hipFree(c->dc_buf);
    if (c->dcr_buf) (void)hipFree(c->dcr_buf);
    if (c->rows_buf) (void)hipFree(c->rows_buf);
    if (c->bt_buf) (void)hipFree(c->bt_buf);
    if (c->ex_ws) (void)hipFree(c->ex_ws);
    if (c->ex_list) (void)hipFree(c->ex_list);
    if (c->ex_next) (void)hipFree(c->ex_next);
    delete c;
    return DGEN_OK;
}

int32_t dgen_prep_shapes(dgen_ctx* c, const float* shapes, int64_t n_rows, double* row_sum,
                         double* row_slots, void* stream) {
    if (!c || !shapes || !row_sum || !row_slots || n_rows <= 0) {
        set_err("dgen_prep_shapes: bad argument");
        return DGEN_E_ARG;
    }
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_row_pairwise_shape, dim3((unsigned)((n_rows + 127) / 128)), dim3(128), 0, s,
                       shapes, n_rows, row_sum);
    int64_t tot = n_rows * NSLOT;
    hipLaunchKernelGGL(k_row_slots_shape, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s,
                       shapes, n_rows, row_slots);
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

int32_t dgen_prep_cfs(dgen_ctx* c, const int32_t* cfs, int64_t n_rows, double* row_naep,
                      double* row_slots, void* stream) {
    if (!c || !cfs || !row_naep || !row_slots || n_rows <= 0) {
        set_err("dgen_prep_cfs: bad argument");
        return DGEN_E_ARG;
    }
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_row_pairwise_cf, dim3((unsigned)((n_rows + 127) / 128)), dim3(128), 0, s,
                       cfs, n_rows, row_naep);
    int64_t tot = n_rows * NSLOT;
    hipLaunchKernelGGL(k_row_slots_cf, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s,
                       cfs, n_rows, row_slots);
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

size_t dgen_workspace_bytes(int64_t n, int64_t n_scratch) {
    if (n < 0 || n_scratch < 0) return 0;
    return sizeof(double) * ((size_t)4 * NBIN * (size_t)n + (size_t)n + (size_t)NH * (size_t)n_scratch) +
           NB_BYTES * (size_t)n_scratch;
}

int32_t dgen_size_agents(dgen_ctx* c, const dgen_tables* T, const dgen_agents* A,
                         const dgen_outputs* O, int64_t n, void* ws, size_t ws_bytes,
                         int64_t n_scratch, void* stream) {
    if (!c || !T || !A || !O) { set_err("dgen_size_agents: null argument"); return DGEN_E_ARG; }
    if (n <= 0) return DGEN_OK;
    if (!T->shapes || !T->shape_sum || !T->shape_slots || !T->cfs || !T->cf_naep || !T->cf_slots ||
        !T->tariffs || T->n_tariffs <= 0 || T->n_demand < 0 || (T->n_demand > 0 && !T->demand)) {
        set_err("dgen_size_agents: incomplete tables");
        return DGEN_E_ARG;
    }
    const void* req_a[] = {A->load_row, A->cf_row, A->wholesale_row, A->tariff0, A->sw_solar_off,
                           A->sw_solar_cnt, A->sw_storage_off, A->sw_storage_cnt, A->scratch_slot,
                           A->flags, A->econ_life, A->loan_term, A->load_kwh, A->price_mult,
                           A->inflation, A->pv_deg, A->escalator, A->down_payment, A->tax_rate,
                           A->real_discount, A->itc_frac, A->capex, A->capex_combined,
                           A->batt_capex_kwh, A->ccm, A->vor};
    for (const void* p : req_a)
        if (!p) { set_err("dgen_size_agents: missing agent column"); return DGEN_E_ARG; }
    const void* req_o[] = {O->system_kw, O->x_last, O->annual_kwh, O->naep, O->capacity_factor,
                           O->price_per_kwh, O->npv, O->payback_raw, O->payback_period,
                           O->first_with, O->first_without, O->batt_kw, O->batt_kwh,
                           O->npv_pv_batt, O->nfev, O->tariff_final, O->switched, O->status,
                           O->cash_flow, O->cfev_pv, O->bill_w_pv, O->bill_wo_pv, O->cfev_batt,
                           O->bill_w_batt, O->bill_wo_batt};
    for (const void* p : req_o)
        if (!p) { set_err("dgen_size_agents: missing output column"); return DGEN_E_ARG; }
    // WO: the with-battery plane alone (float32 tiles; daily plan, no loss
    // model, no demand machinery): the model-year loop's export form
    const bool wo = O->baseline == nullptr && O->net_pvonly == nullptr && O->net_with_batt != nullptr;
    const bool hourly = O->baseline != nullptr;
    if (!wo && ((O->net_pvonly != nullptr) != hourly || (O->net_with_batt != nullptr) != hourly)) {
        set_err("dgen_size_agents: hourly planes must be all set, all NULL, or the with-battery plane alone");
        return DGEN_E_ARG;
    }
    if (wo && (O->hourly_f64 || c->cfg.batt_loss_model == 1 || c->cfg.batt_update_hours != 24)) {
        set_err("dgen_size_agents: the with-battery plane alone is float32, daily plan, no loss model");
        return DGEN_E_ARG;
    }
    // k_hourly_batt forms a 32-bit per-lane byte offset i x 16 into the hourly tiles
    if (n >= ((int64_t)1 << 29) || n_scratch >= ((int64_t)1 << 28) ||
        ((hourly || wo) && n >= ((int64_t)1 << (O->hourly_f64 ? 27 : 28)))) {
        set_err("dgen_size_agents: batch too large (n < 2^29, n < 2^28 with f32 hourly planes, "
                "2^27 with f64, n_scratch < 2^28 per call)");
        return DGEN_E_ARG;
    }
    if (!ws || ws_bytes < dgen_workspace_bytes(n, n_scratch)) {
        set_err("dgen_size_agents: workspace too small (%zu < %zu)", ws_bytes,
                dgen_workspace_bytes(n, n_scratch));
        return DGEN_E_ARG;
    }
    // the year-lane kernels keep the TOU demand peaks in the lane's LDS column
    // (4 x half slots): with demand charges billed it must hold DGEN_DCP
    dgen_tables Tk = *T;
    // the demand machinery also supplies the month peaks of kWh/kW tier units
    const bool dc = (c->cfg.skip_demand_charges == 0 && Tk.n_demand > 0) || (Tk.peak_units && Tk.n_demand > 0);
    if (wo && dc) {
        set_err("dgen_size_agents: the with-battery plane alone is not built with demand charges / kWh/kW tiers");
        return DGEN_E_ARG;
    }
    if (dc && 4 * lds_half(Tk.max_periods) < DCP) Tk.max_periods = (DCP + 3) / 4;
    // yl_bill_nb stages its entries and month sums in slots 2 half .. 2 half + 4
    if (n_scratch > 0 && lds_half(Tk.max_periods) < 3) Tk.max_periods = 3;
    T = &Tk;
    HIP_TRY(hipSetDevice(c->device));
    if (dc && (size_t)n * DCW_BYTES > c->dc_cap) {   // envelope storage (context-owned)
        if (c->dc_buf) HIP_TRY(hipFree(c->dc_buf));
        c->dc_buf = nullptr;
        c->dc_cap = 0;
        if (hipMalloc(&c->dc_buf, (size_t)n * DCW_BYTES) != hipSuccess) {
            c->dc_buf = nullptr;   // no envelopes: the kernels fall back to the hourly pass
            (void)hipGetLastError();
        } else {
            c->dc_cap = (size_t)n * DCW_BYTES;
        }
    }
    hipStream_t s = (hipStream_t)stream;
    // certified Brent paths: trace buffer, per-chunk lists
    const bool exact_on = c->exact != 0;
    if (exact_on) {
        if ((size_t)n * BT_MAX * sizeof(double) > c->bt_cap) {
            if (c->bt_buf) HIP_TRY(hipFree(c->bt_buf));
            c->bt_buf = nullptr;
            c->bt_cap = 0;
            HIP_TRY(hipMalloc(&c->bt_buf, (size_t)n * BT_MAX * sizeof(double)));
            c->bt_cap = (size_t)n * BT_MAX * sizeof(double);
        }
        if ((size_t)(n + dgen_ctx::MAXCH) * sizeof(int32_t) > c->ex_list_cap) {
            if (c->ex_list) HIP_TRY(hipFree(c->ex_list));
            c->ex_list = nullptr;
            c->ex_list_cap = 0;
            HIP_TRY(hipMalloc(&c->ex_list, (size_t)(n + dgen_ctx::MAXCH) * sizeof(int32_t)));
            c->ex_list_cap = (size_t)(n + dgen_ctx::MAXCH) * sizeof(int32_t);
        }
        if (!c->ex_next) HIP_TRY(hipMalloc(&c->ex_next, (size_t)dgen_ctx::MAXCH * sizeof(int32_t)));
    }
    // the exact re-run's per-block scratch (its bins sized by the table's
    // periods and the demand records)
    const bool ex_dcb = c->cfg.skip_demand_charges == 0 && T->n_demand > 0;
    const int ex_P = (T->max_periods > 0 && T->max_periods <= MAXP) ? T->max_periods : MAXP;
    const size_t ex_wsb = ex_ws_bytes(ex_P, ex_dcb);
    if (exact_on && (size_t)EX_BLOCKS * ex_wsb > c->ex_ws_cap) {
        if (c->ex_ws) HIP_TRY(hipFree(c->ex_ws));
        c->ex_ws = nullptr;
        c->ex_ws_cap = 0;
        HIP_TRY(hipMalloc(&c->ex_ws, (size_t)EX_BLOCKS * ex_wsb));
        c->ex_ws_cap = (size_t)EX_BLOCKS * ex_wsb;
    }
    const int ex_threads = EX_THREADS;
    // the bins in LDS when the batch's analysis years and the table's periods
    // fit the device's work-group LDS (the year bills then read LDS), else in
    // the block's global scratch
    const int ex_ny = (A->max_years >= 1 && A->max_years <= MAXY) ? A->max_years : MAXY;
    // (N + 1 years: the no-system year rides on lane N)
    const size_t ex_bins_lds = sizeof(double) * (size_t)(ex_ny + 1) * 12 * (size_t)ex_P * (3 + (ex_dcb ? (size_t)DCP : 0));
    const bool ex_lb = ex_lds_bytes() + ex_bins_lds + 16 <= (size_t)c->lds_max;   // (+ the kernel's static s_next)
    const size_t ex_lds = ex_lds_bytes() + (ex_lb ? ex_bins_lds : 0);
    if (exact_on && ex_lds > 65536)
        HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(k_size_exact),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)ex_lds));
    double* const bt = exact_on ? c->bt_buf : nullptr;
    // the re-run's grid: the blocks the device holds at once (work counter),
    // at most EX_BLOCKS scratch slots
    int ex_grid = EX_BLOCKS;
    if (exact_on && c->ex_dyn) {
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k_size_exact),
                                                         ex_threads, ex_lds) == hipSuccess && per_cu > 0) {
            const int64_t g = (int64_t)per_cu * c->n_cu;
            ex_grid = g < EX_BLOCKS ? (int)g : EX_BLOCKS;
        } else {
            (void)hipGetLastError();
        }
    }
    if (c->pending == dgen_ctx::RING) {   // fold the oldest record before reuse
        int r = fold_one(c, c->head);
        if (r) return r;
        c->pending--;
    }
    // chunk pipeline: k_size of chunk j+1 (fp64 VALU / latency bound) runs on
    // the caller's stream while k_hourly_batt + k_batt_finance of chunk j (HBM
    // bound) run on s2; chunk boundaries are multiples of BLOCK so every wave's
    // hour-row stores stay one contiguous 256 B segment.
    int nch = c->chunks;
    if (nch < 1) nch = 1;
    if (nch > dgen_ctx::MAXCH) nch = dgen_ctx::MAXCH;
    int64_t csz = (n + nch - 1) / nch;
    csz = ((csz + BLOCK - 1) / BLOCK) * BLOCK;
    nch = (int)((n + csz - 1) / csz);
    int slot = c->head;
    c->head = (c->head + 1) % dgen_ctx::RING;
    c->pending++;
    c->nch[slot] = nch;
    // k_hourly_batt: per-period bins [P][BLOCK] double2 (x2 with the net-billing
    // split: import and export sums) + the waves' day buffers
    // (the scan form doubles the bins; kept within 64 KB of dynamic LDS per
    // block, i.e. batches whose tariffs have at most 10 periods)
    // battery-case demand records (DcrRec) built in the scan for the finance
    // kernel's demand pass: demand-charge / kWh/kW batches with the daily plan
    // (the hourly re-plan keeps the staged pass over the plane), DCR_BYTES per
    // scratch slot, context-owned; their per-period maxima add [dc_nq][BLOCK]
    // double2 to the scan's LDS
    const int dc_nq = (T->max_dc_periods > 0 && T->max_dc_periods <= DCP) ? T->max_dc_periods : DCP;
    // the Li-ion loss model's scan has no record forms: its batches bill from the planes
    const bool loss = c->cfg.batt_loss_model == 1;
    bool dcr_on = dc && n_scratch > 0 && c->battery && c->cfg.batt_update_hours != 1 && c->dcr_enable && !loss;
    if (dcr_on && (size_t)n_scratch * DCR_BYTES > c->dcr_cap) {
        if (c->dcr_buf) HIP_TRY(hipFree(c->dcr_buf));
        c->dcr_buf = nullptr;
        c->dcr_cap = 0;
        if (hipMalloc(&c->dcr_buf, (size_t)n_scratch * DCR_BYTES) != hipSuccess) {
            c->dcr_buf = nullptr;   // no records: the staged pass over the plane
            (void)hipGetLastError();
        } else {
            c->dcr_cap = (size_t)n_scratch * DCR_BYTES;
        }
    }
    dcr_on = dcr_on && c->dcr_buf != nullptr;
    char* const dcr = dcr_on ? reinterpret_cast<char*>(c->dcr_buf) : nullptr;
    const size_t lds_dcr = dcr_on ? (size_t)16 * dc_nq * BLOCK : 0;
    const size_t lds_nb = sizeof(double) * 4 * (size_t)lds_half(T->max_periods) * BLOCK + lds_dcr +
                          (size_t)(BLOCK / 64) * HB_DAY_BYTES;
    const bool nb_scan = n_scratch > 0 && c->nb_scan && c->battery && lds_nb <= 65536 && !loss;
    const size_t lds = sizeof(double) * 2 * (size_t)lds_half(T->max_periods) * BLOCK * (nb_scan ? 2 : 1) +
                       lds_dcr + (size_t)(BLOCK / 64) * HB_DAY_BYTES;
    const int rep_mask = (nb_scan ? 1 : 0) | (dcr_on ? 2 : 0);
    // TS sell-rate agents' split built in a scan of their own (k_hourly_batt<TS>,
    // launched beside the NB scan over the rest; 12 KB more of day buffer per
    // wave, so it runs one wave per SIMD): batches with a wholesale table, no
    // demand charges or kWh/kW peaks, daily plan, hourly planes requested.  With the planes the
    // NB scan is clock-bound and the TS blocks fill in around it (national 200k:
    // 21.38 -> 20.22 ms per step, k_batt_finance 3.54 -> 1.11 ms); without them
    // (the model-year loop's sizing call) the one-wave form's latency shows
    // (C5 2.5M: k_hourly_batt 56 -> 98 ms against k_batt_finance 47 -> 15 ms),
    // and the plane pass stays; in the with-battery-plane call (WO) as well
    // (round 5: 63 -> 102 ms against 46.5 -> 14.7 ms, profiles/r05/loop_ts_wo)
    const size_t lds_ts = lds + (size_t)(BLOCK / 64) * HB_DAY_BYTES;
    // (not in batches with the demand machinery at all: whether their agents
    // take this form must not depend on the demand records being on)
    const bool ts_split = nb_scan && T->wholesale != nullptr && !dc && c->ts_scan && lds_ts <= 65536 &&
                          c->cfg.batt_update_hours != 1 && hourly;
    c->last_paths[0] = nb_scan ? 1 : 0;
    c->last_paths[1] = dcr_on ? 1 : 0;
    c->last_paths[2] = ts_split ? 1 : 0;
    c->last_paths[3] = dc ? 1 : 0;
    c->last_paths[4] = T->max_periods;
    c->last_paths[5] = dc_nq;
    // two agents per wave when every analysis period fits 32 lanes, unless the
    // build guard withdrew that kernel's 32-lane instantiation (DGEN_NO2_*)
    const bool fits32 = A->max_years >= 1 && A->max_years <= 32;
    const bool pk = dc && T->peak_units != 0;       // kWh/kW tiers: the PK instantiations
    const int lpa_s = (fits32 && !(pk ? DGEN_NO2_SIZE_PK : dc ? DGEN_NO2_SIZE_DC : DGEN_NO2_SIZE)) ? 32 : WAVE;
    const int lpa_f = (fits32 && !(pk ? DGEN_NO2_FIN_PK : dc ? DGEN_NO2_FIN_DC : DGEN_NO2_FIN)) ? 32 : WAVE;
    // the NEM-only (!dc, !net) instantiations' slimmer layout
    const size_t ylds_s_nem = ylds_bytes(lds_half(T->max_periods), lpa_s, false, YL_NEM);
    const size_t ylds_f_nem = ylds_bytes(lds_half(T->max_periods), lpa_f, false, YL_NEM);
    // the demand-charge instantiations without net billing (no PK: those bill net)
    const size_t ylds_s_dc = ylds_bytes(lds_half(T->max_periods), lpa_s, false, YL_DC) +
                             (size_t)(WAVE / lpa_s) * DCS_BYTES;
    const size_t ylds_f_dc = ylds_bytes(lds_half(T->max_periods), lpa_f, false, YL_DC) +
                             (size_t)(WAVE / lpa_f) * DEM_STAGE_BYTES;
    const size_t ylds_s = ylds_bytes(lds_half(T->max_periods), lpa_s, pk) +
                          (dc ? (size_t)(WAVE / lpa_s) * DCS_BYTES : 0);   // k_size's envelope stage
    // k_batt_finance's demand-charge instantiations stage hours per segment
    const size_t ylds_f = ylds_bytes(lds_half(T->max_periods), lpa_f, pk) +
                          (dc ? (size_t)(WAVE / lpa_f) * DEM_STAGE_BYTES : 0);
    hipStream_t s2 = c->s2;
    char* const nbws = n_scratch > 0 ? ws_nb(ws, n, n_scratch) : nullptr;
    // demand envelopes of the first-evaluation tariffs prebuilt (k_dc_env)
    const int dc_pre = (dc && c->dc_buf && c->dc_pre) ? 1 : 0;
    c->last_paths[6] = dc_pre;
    const int nb_pre = (n_scratch > 0 && c->nb_pre) ? 1 : 0;
    const int pre = dc_pre | (nb_pre << 1);     // k_size's view of the two prebuilds
    c->ex_last_nch = exact_on ? nch : 0;
    HIP_TRY(hipEventRecord(c->fork, s));
    HIP_TRY(hipStreamWaitEvent(s2, c->fork, 0));
    for (int j = 0; j < nch; j++) {
        const int64_t i0 = (int64_t)j * csz, i1 = (i0 + csz < n) ? i0 + csz : n, m = i1 - i0;
        hipEvent_t* e = c->ev[slot][j];
        HIP_TRY(hipEventRecord(e[0], s));
        // net-billing splits and demand envelopes of the initial tariffs
        // (counted in k_size's time)
        if (nb_pre) {
            // its agents all hold a scratch slot: the bins-only prefix is skipped
            const int64_t ja = (!dc && c->nem_hi > i0) ? (c->nem_hi < i1 ? c->nem_hi : i1) : i0;
            if (i1 > ja)
                hipLaunchKernelGGL((k_nb_env<32>), dim3((unsigned)((i1 - ja + 1) / 2)), dim3(WAVE),
                                   4 * WAVE * sizeof(double) + 2 * NBS_BYTES, s, *T, *A, ja, i1, nbws);
        }
        if (dc_pre) {
            const dim3 eg((unsigned)((m + DCE_WPB - 1) / DCE_WPB));
            if (dc_nq <= 2)
                hipLaunchKernelGGL((k_dc_env<2>), eg, dim3(WAVE * DCE_WPB), 0, s, *T, *A, c->cfg, i0, i1, c->dc_buf);
            else if (dc_nq <= 4)
                hipLaunchKernelGGL((k_dc_env<4>), eg, dim3(WAVE * DCE_WPB), 0, s, *T, *A, c->cfg, i0, i1, c->dc_buf);
            else
                hipLaunchKernelGGL((k_dc_env<DCP>), eg, dim3(WAVE * DCE_WPB), 0, s, *T, *A, c->cfg, i0, i1, c->dc_buf);
        }
        // agents per year-lane block: WAVE / lpa
        const dim3 ygrid_s((unsigned)((m + WAVE / lpa_s - 1) / (WAVE / lpa_s)));
        const dim3 ygrid_f((unsigned)((m + WAVE / lpa_f - 1) / (WAVE / lpa_f)));
        // net billing compiled in only when the batch has scratch slots (an
        // agent whose tariffs can bill net always gets one, assign_scratch)
        const bool net = n_scratch > 0;
        // demand-charge batches: the net-billing paths only when some tariff
        // of the table bills net (dgen_tables.no_net; registers: C4 k_size
        // spills 412 -> 200 B per lane without them)
        const bool dc_net = T->no_net == 0;
        // a net batch's leading rows without a scratch slot (dgen_set_nem_rows:
        // bins-only agents, profile_order puts them first) run the bins-only
        // instantiations: fewer registers and the slimmer LDS layout
        const int64_t nm = (net && !dc && c->nem_hi > i0) ? (c->nem_hi < i1 ? c->nem_hi : i1) : i0;
        const dim3 ygrid_sa((unsigned)((nm - i0 + WAVE / lpa_s - 1) / (WAVE / lpa_s)));
        const dim3 ygrid_sb((unsigned)((i1 - nm + WAVE / lpa_s - 1) / (WAVE / lpa_s)));
        if (lpa_s == 32 && !dc) {
#if !DGEN_NO2_SIZE
            if (net) {
                if (nm > i0)
                    hipLaunchKernelGGL((k_size_w<32, false, false, false>), ygrid_sa, dim3(WAVE), ylds_s_nem, s, *T, *A,
                                       *O, c->cfg, n, i0, nm, nullptr, nbws, pre, bt);
                if (i1 > nm)
                    hipLaunchKernelGGL((k_size_w<32, false, true, false>), ygrid_sb, dim3(WAVE), ylds_s, s, *T, *A, *O,
                                       c->cfg, n, nm, i1, nullptr, nbws, pre, bt);
            } else
                hipLaunchKernelGGL((k_size_w<32, false, false, false>), ygrid_s, dim3(WAVE), ylds_s_nem, s, *T, *A, *O,
                                   c->cfg, n, i0, i1, nullptr, nbws, pre, bt);
#endif
        } else if (lpa_s == 32 && !pk) {
#if !DGEN_NO2_SIZE_DC
            if (dc_net)
                hipLaunchKernelGGL((k_size_w<32, true, true, false>), ygrid_s, dim3(WAVE), ylds_s, s, *T, *A, *O,
                                   c->cfg, n, i0, i1, c->dc_buf, nbws, pre, bt);
            else
                hipLaunchKernelGGL((k_size_w<32, true, false, false>), ygrid_s, dim3(WAVE), ylds_s_dc, s, *T, *A, *O,
                                   c->cfg, n, i0, i1, c->dc_buf, nbws, pre, bt);
#endif
        } else if (lpa_s == 32) {
#if !DGEN_NO2_SIZE_PK
            hipLaunchKernelGGL((k_size_w<32, true, true, true>), ygrid_s, dim3(WAVE), ylds_s, s, *T, *A, *O,
                               c->cfg, n, i0, i1, c->dc_buf, nbws, pre, bt);
#endif
        } else if (!dc) {
            if (net) {
                if (nm > i0)
                    hipLaunchKernelGGL((k_size_w<WAVE, false, false, false>), ygrid_sa, dim3(WAVE), ylds_s_nem, s, *T,
                                       *A, *O, c->cfg, n, i0, nm, nullptr, nbws, pre, bt);
                if (i1 > nm)
                    hipLaunchKernelGGL((k_size_w<WAVE, false, true, false>), ygrid_sb, dim3(WAVE), ylds_s, s, *T, *A,
                                       *O, c->cfg, n, nm, i1, nullptr, nbws, pre, bt);
            } else
                hipLaunchKernelGGL((k_size_w<WAVE, false, false, false>), ygrid_s, dim3(WAVE), ylds_s_nem, s, *T, *A, *O,
                                   c->cfg, n, i0, i1, nullptr, nbws, pre, bt);
        } else if (!pk) {
            if (dc_net)
                hipLaunchKernelGGL((k_size_w<WAVE, true, true, false>), ygrid_s, dim3(WAVE), ylds_s, s, *T, *A, *O,
                                   c->cfg, n, i0, i1, c->dc_buf, nbws, pre, bt);
            else
                hipLaunchKernelGGL((k_size_w<WAVE, true, false, false>), ygrid_s, dim3(WAVE), ylds_s_dc, s, *T, *A, *O,
                                   c->cfg, n, i0, i1, c->dc_buf, nbws, pre, bt);
        } else {
            hipLaunchKernelGGL((k_size_w<WAVE, true, true, true>), ygrid_s, dim3(WAVE), ylds_s, s, *T, *A, *O,
                               c->cfg, n, i0, i1, c->dc_buf, nbws, pre, bt);
        }
        if (exact_on) {
            // the chunk's searches replayed against the oracle-difference
            // bound; the listed agents re-run in the oracle's arithmetic
            // (counted in k_size's time)
            int32_t* const lst = c->ex_list + i0 + j;
            c->ex_last_off[j] = i0 + j;
            HIP_TRY(hipMemsetAsync(lst, 0, sizeof(int32_t), s));
            int32_t* const nxt = c->ex_dyn ? c->ex_next + j : nullptr;
            if (nxt) HIP_TRY(hipMemsetAsync(nxt, 0, sizeof(int32_t), s));
            hipLaunchKernelGGL(k_brent_certify, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, *T, *A, *O,
                               c->cfg, i0, i1, bt, lst, c->exact);
            hipLaunchKernelGGL(k_size_exact, dim3((unsigned)(m < ex_grid ? m : ex_grid)), dim3(ex_threads),
                               ex_lds, s, *T, *A, *O, c->cfg, lst, c->ex_ws, (int64_t)ex_wsb, ex_lb ? ex_ny + 1 : 0,
                               nxt);
        }
        HIP_TRY(hipEventRecord(e[1], s));
        HIP_TRY(hipStreamWaitEvent(s2, e[1], 0));
        HIP_TRY(hipEventRecord(e[2], s2));
        const dim3 block(BLOCK);
        // hourly split (dgen_ctx::hb_split parts, default 2; DGEN_HB_SPLIT
        // overrides): the chunk's parts sweep their months on their own
        // streams, so one part's launch tails overlap the others' waves (C3
        // 1M: k_hourly_batt 24.26 -> 23.68 ms with 2 parts, profiles/r04/ab)
        int nparts = c->hb_split;
        while (nparts > 1 && m < (int64_t)nparts * 2 * BLOCK) nparts--;
        const int64_t psz = ((m + nparts - 1) / nparts + BLOCK - 1) / BLOCK * BLOCK;
        // no scratch slot in the batch: the bins-only scan (DGEN_HB_NEM=0 disables, A/B)
        const bool nem_only = n_scratch == 0 && c->hb_nem;
        for (int part = 1; part < nparts; part++) HIP_TRY(hipStreamWaitEvent(c->sx[part - 1], e[1], 0));
        // the TS agents' scans run on streams of their own beside the NB scans
        // (disjoint agents): their one-wave-per-SIMD blocks fill in around the
        // NB blocks instead of queueing behind them
        if (ts_split)
            for (int part = 0; part < nparts; part++) HIP_TRY(hipStreamWaitEvent(c->st[part], e[1], 0));
        for (int part = 0; part < nparts; part++) {
        const int64_t ha = i0 + part * psz < i1 ? i0 + part * psz : i1;
        const int64_t hb = part == nparts - 1 ? i1 : (ha + psz < i1 ? ha + psz : i1);
        hipStream_t hs = part == 0 ? s2 : c->sx[part - 1];
        hipStream_t hts = c->st[part];
        if (hb <= ha) continue;
        const dim3 hgrid((unsigned)((hb - ha + BLOCK - 1) / BLOCK));
        // the TS form's rows: the part's rows that can hold a TS-capable agent
        // (dgen_set_ts_rows), from a block boundary of the part
        const int64_t tsa = c->ts_lo > ha ? ha + (c->ts_lo - ha) / BLOCK * BLOCK : ha;
        const int64_t tsb = c->ts_hi < hb ? c->ts_hi : hb;
        const dim3 tsgrid((unsigned)(tsb > tsa ? (tsb - tsa + BLOCK - 1) / BLOCK : 1));
        for (int m0 = 0; m0 < 12; m0 += c->hb_months) {
            const int m1 = m0 + c->hb_months < 12 ? m0 + c->hb_months : 12;
#define DGEN_HB_LAUNCH_R(H, F, REP, R)                                                            \
    do {                                                                                          \
        if (nb_scan && !(REP) && dcr_on && !(R))                                                  \
            hipLaunchKernelGGL((k_hourly_batt<H, F, true, false, true>), hgrid, block, lds, hs, *T, *A, *O, \
                               c->cfg, n, ws, n_scratch, ha, hb, m0, m1, c->battery, c->nb_scan, 0, dcr, dc_nq, c->dcr_enable); \
        else if (nb_scan && !(REP) && ts_split && !(R)) {                                         \
            hipLaunchKernelGGL((k_hourly_batt<H, F, true, false, false>), hgrid, block, lds, hs, *T, *A, *O, \
                               c->cfg, n, ws, n_scratch, ha, hb, m0, m1, c->battery, c->nb_scan, 0, nullptr, 0, 0, 1); \
            if (tsb > tsa)                                                                        \
                hipLaunchKernelGGL((k_hourly_batt<H, F, true, false, false, false, false, true>), tsgrid, block, \
                                   lds_ts, hts, *T, *A, *O, c->cfg, n, ws, n_scratch, tsa, tsb, m0, m1, c->battery, \
                                   c->nb_scan, 0, nullptr, 0, 0, 2);                               \
        } else if (nb_scan && !(REP))                                                             \
            hipLaunchKernelGGL((k_hourly_batt<H, F, true, R, false>), hgrid, block, lds, hs, *T, *A, *O, c->cfg, \
                               n, ws, n_scratch, ha, hb, m0, m1, c->battery, c->nb_scan, 0, nullptr, 0, 0); \
        else if (!(REP) && dcr_on && !(R))                                                        \
            hipLaunchKernelGGL((k_hourly_batt<H, F, false, false, true>), hgrid, block, lds, hs, *T, *A, *O, \
                               c->cfg, n, ws, n_scratch, ha, hb, m0, m1, c->battery, 0, 0, dcr, dc_nq, c->dcr_enable); \
        else                                                                                      \
            hipLaunchKernelGGL((k_hourly_batt<H, F, false, R, false>), hgrid, block, lds, hs, *T, *A, *O, \
                               c->cfg, n, ws, n_scratch, ha, hb, m0, m1, c->battery, 0, (REP) ? rep_mask : 0, \
                               (REP) ? dcr : nullptr, 0, 0);                                                               \
    } while (0)
#define DGEN_HB_LAUNCH_LOSS(H, F, R)                                                              \
            hipLaunchKernelGGL((k_hourly_batt<H, F, false, R, false, true>), hgrid, block, lds, hs, *T, *A, *O, \
                               c->cfg, n, ws, n_scratch, ha, hb, m0, m1, c->battery, 0, 0, nullptr, 0, 0)
#define DGEN_HB_LAUNCH(H, F, REP)                                                                 \
    do {                                                                                          \
        if (nem_only && !loss && c->cfg.batt_update_hours != 1 && !(REP))                         \
            hipLaunchKernelGGL((k_hourly_batt<H, F, false, false, false, false, true>), hgrid, block, lds, hs, \
                               *T, *A, *O, c->cfg, n, ws, n_scratch, ha, hb, m0, m1, c->battery, 0, 0, nullptr, 0, 0); \
        else if (loss && c->cfg.batt_update_hours == 1) DGEN_HB_LAUNCH_LOSS(H, F, true);         \
        else if (loss) DGEN_HB_LAUNCH_LOSS(H, F, false);                                          \
        else if (c->cfg.batt_update_hours == 1) DGEN_HB_LAUNCH_R(H, F, REP, true);                \
        else DGEN_HB_LAUNCH_R(H, F, REP, false);                                                  \
    } while (0)
            if (wo) {
                if (nem_only)
                    hipLaunchKernelGGL((k_hourly_batt<true, false, false, false, false, false, true, false, false, true>),
                                       hgrid, block, lds, hs, *T, *A, *O, c->cfg, n, ws, n_scratch, ha, hb, m0, m1,
                                       c->battery, 0, 0, nullptr, 0, 0);
                else if (nb_scan)
                    hipLaunchKernelGGL((k_hourly_batt<true, false, true, false, false, false, false, false, false, true>),
                                       hgrid, block, lds, hs, *T, *A, *O, c->cfg, n, ws, n_scratch, ha, hb, m0, m1,
                                       c->battery, c->nb_scan, 0, nullptr, 0, 0);
                else
                    hipLaunchKernelGGL((k_hourly_batt<true, false, false, false, false, false, false, false, false, true>),
                                       hgrid, block, lds, hs, *T, *A, *O, c->cfg, n, ws, n_scratch, ha, hb, m0, m1,
                                       c->battery, 0, 0, nullptr, 0, 0);
            } else if (hourly && O->hourly_f64) DGEN_HB_LAUNCH(true, true, false);
            else if (hourly) DGEN_HB_LAUNCH(true, false, false);
            else DGEN_HB_LAUNCH(false, false, false);
        }
        }
        for (int part = 1; part < nparts; part++) {
            HIP_TRY(hipEventRecord(c->hb_join[part - 1], c->sx[part - 1]));
            HIP_TRY(hipStreamWaitEvent(s2, c->hb_join[part - 1], 0));
        }
        if (ts_split)
            for (int part = 0; part < nparts; part++) {
                HIP_TRY(hipEventRecord(c->ts_join[part], c->st[part]));
                HIP_TRY(hipStreamWaitEvent(s2, c->ts_join[part], 0));
            }
        // repair pass (agents whose scan-built split or demand record
        // overflowed: their plane), whole chunk on s2
        const int64_t ha = i0, hb = i1;
        hipStream_t hs = s2;
        hipStream_t hts = s2;           // (the repair pass never launches the TS form)
        const int64_t tsa = 0, tsb = 0;
        const dim3 tsgrid(1);
        (void)hts; (void)tsa; (void)tsb; (void)tsgrid;
        const dim3 hgrid((unsigned)((m + BLOCK - 1) / BLOCK));
        // one launch over the whole year: the pass runs only the agents whose
        // split or record overflowed (none in most calls), so a month-segmented
        // sweep's L2 reuse buys nothing and its 12 launches over the chunk's
        // rows cost ~8 us each (national 200k: 12 of them per step)
        for (int m0 = 0; rep_mask && m0 < 12; m0 += 12) {
            const int m1 = 12;
            if (hourly && O->hourly_f64) DGEN_HB_LAUNCH(true, true, true);
            else if (hourly) DGEN_HB_LAUNCH(true, false, true);
            else DGEN_HB_LAUNCH(false, false, true);
#undef DGEN_HB_LAUNCH
#undef DGEN_HB_LAUNCH_R
#undef DGEN_HB_LAUNCH_LOSS
        }
        HIP_TRY(hipEventRecord(e[3], s2));
        const dim3 ygrid_fa((unsigned)((nm - i0 + WAVE / lpa_f - 1) / (WAVE / lpa_f)));
        const dim3 ygrid_fb((unsigned)((i1 - nm + WAVE / lpa_f - 1) / (WAVE / lpa_f)));
        if (!c->battery) {
            // PV-only variant: no battery-case bill / cash flow
        } else if (lpa_f == 32 && !dc) {
#if !DGEN_NO2_FIN
            if (net) {
                if (nm > i0)
                    hipLaunchKernelGGL((k_batt_finance_w<32, false, false, false>), ygrid_fa, dim3(WAVE), ylds_f_nem, s2,
                                       *T, *A, *O, c->cfg, n, ws, n_scratch, i0, nm, nbws, (int)nb_scan, dcr, dc_nq);
                if (i1 > nm)
                    hipLaunchKernelGGL((k_batt_finance_w<32, false, true, false>), ygrid_fb, dim3(WAVE), ylds_f, s2, *T,
                                       *A, *O, c->cfg, n, ws, n_scratch, nm, i1, nbws, (int)nb_scan, dcr, dc_nq);
            } else
                hipLaunchKernelGGL((k_batt_finance_w<32, false, false, false>), ygrid_f, dim3(WAVE), ylds_f_nem, s2, *T, *A,
                                   *O, c->cfg, n, ws, n_scratch, i0, i1, nbws, (int)nb_scan, dcr, dc_nq);
#endif
        } else if (lpa_f == 32 && !pk) {
#if !DGEN_NO2_FIN_DC
            if (dc_net)
                hipLaunchKernelGGL((k_batt_finance_w<32, true, true, false>), ygrid_f, dim3(WAVE), ylds_f, s2, *T, *A,
                                   *O, c->cfg, n, ws, n_scratch, i0, i1, nbws, (int)nb_scan, dcr, dc_nq);
            else
                hipLaunchKernelGGL((k_batt_finance_w<32, true, false, false>), ygrid_f, dim3(WAVE), ylds_f_dc, s2, *T, *A,
                                   *O, c->cfg, n, ws, n_scratch, i0, i1, nbws, (int)nb_scan, dcr, dc_nq);
#endif
        } else if (lpa_f == 32) {
#if !DGEN_NO2_FIN_PK
            hipLaunchKernelGGL((k_batt_finance_w<32, true, true, true>), ygrid_f, dim3(WAVE), ylds_f, s2, *T, *A,
                               *O, c->cfg, n, ws, n_scratch, i0, i1, nbws, (int)nb_scan, dcr, dc_nq);
#endif
        } else if (!dc) {
            if (net) {
                if (nm > i0)
                    hipLaunchKernelGGL((k_batt_finance_w<WAVE, false, false, false>), ygrid_fa, dim3(WAVE), ylds_f_nem,
                                       s2, *T, *A, *O, c->cfg, n, ws, n_scratch, i0, nm, nbws, (int)nb_scan, dcr, dc_nq);
                if (i1 > nm)
                    hipLaunchKernelGGL((k_batt_finance_w<WAVE, false, true, false>), ygrid_fb, dim3(WAVE), ylds_f, s2,
                                       *T, *A, *O, c->cfg, n, ws, n_scratch, nm, i1, nbws, (int)nb_scan, dcr, dc_nq);
            } else
                hipLaunchKernelGGL((k_batt_finance_w<WAVE, false, false, false>), ygrid_f, dim3(WAVE), ylds_f_nem, s2, *T,
                                   *A, *O, c->cfg, n, ws, n_scratch, i0, i1, nbws, (int)nb_scan, dcr, dc_nq);
        } else if (!pk) {
            if (dc_net)
                hipLaunchKernelGGL((k_batt_finance_w<WAVE, true, true, false>), ygrid_f, dim3(WAVE), ylds_f, s2, *T,
                                   *A, *O, c->cfg, n, ws, n_scratch, i0, i1, nbws, (int)nb_scan, dcr, dc_nq);
            else
                hipLaunchKernelGGL((k_batt_finance_w<WAVE, true, false, false>), ygrid_f, dim3(WAVE), ylds_f_dc, s2, *T,
                                   *A, *O, c->cfg, n, ws, n_scratch, i0, i1, nbws, (int)nb_scan, dcr, dc_nq);
        } else {
            hipLaunchKernelGGL((k_batt_finance_w<WAVE, true, true, true>), ygrid_f, dim3(WAVE), ylds_f, s2, *T,
                               *A, *O, c->cfg, n, ws, n_scratch, i0, i1, nbws, (int)nb_scan, dcr, dc_nq);
        }
        HIP_TRY(hipEventRecord(e[4], s2));
    }
    HIP_TRY(hipEventRecord(c->join, s2));
    HIP_TRY(hipStreamWaitEvent(s, c->join, 0));
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

int32_t dgen_hourly_planes(dgen_ctx* c, const dgen_tables* T, const dgen_agents* A,
                           const dgen_outputs* O, int64_t n, void* ws, size_t ws_bytes,
                           int64_t n_scratch, void* stream) {
    if (!c || !T || !A || !O) { set_err("dgen_hourly_planes: null argument"); return DGEN_E_ARG; }
    if (n <= 0) return DGEN_OK;
    if (!O->baseline || !O->net_pvonly || !O->net_with_batt) {
        set_err("dgen_hourly_planes: the three hourly planes are required");
        return DGEN_E_ARG;
    }
    if (!T->shapes || !T->shape_sum || !T->cfs || !T->tariffs || T->n_tariffs <= 0 ||
        (T->n_demand > 0 && !T->demand)) {
        set_err("dgen_hourly_planes: incomplete tables");
        return DGEN_E_ARG;
    }
    if (n >= ((int64_t)1 << (O->hourly_f64 ? 27 : 28)) || n_scratch >= ((int64_t)1 << 28)) {
        set_err("dgen_hourly_planes: batch too large (n < 2^28 with f32 planes, 2^27 with f64)");
        return DGEN_E_ARG;
    }
    if (!ws || ws_bytes < dgen_workspace_bytes(n, n_scratch)) {
        set_err("dgen_hourly_planes: workspace too small (%zu < %zu)", ws_bytes,
                dgen_workspace_bytes(n, n_scratch));
        return DGEN_E_ARG;
    }
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    // the scan alone (no split or demand records: nothing reads them after it);
    // it re-derives the battery run from the sizing outputs, so every output it
    // writes besides the planes is the value the sizing call wrote
    const size_t lds = sizeof(double) * 2 * (size_t)lds_half(T->max_periods) * BLOCK +
                       (size_t)(BLOCK / 64) * HB_DAY_BYTES;
    const dim3 grid((unsigned)((n + BLOCK - 1) / BLOCK)), block(BLOCK);
    const bool roll = c->cfg.batt_update_hours == 1;
    for (int m0 = 0; m0 < 12; m0 += c->hb_months) {
        const int m1 = m0 + c->hb_months < 12 ? m0 + c->hb_months : 12;
#define DGEN_HP_LAUNCH(F, R, L)                                                                    \
        hipLaunchKernelGGL((k_hourly_batt<true, F, false, R, false, L>), grid, block, lds, s, *T, *A, *O, c->cfg, \
                           n, ws, n_scratch, (int64_t)0, n, m0, m1, c->battery, 0, 0, nullptr, 0, 0)
        if (c->cfg.batt_loss_model == 1) {
            if (O->hourly_f64) { if (roll) DGEN_HP_LAUNCH(true, true, true); else DGEN_HP_LAUNCH(true, false, true); }
            else { if (roll) DGEN_HP_LAUNCH(false, true, true); else DGEN_HP_LAUNCH(false, false, true); }
        } else if (roll) {
            if (O->hourly_f64) DGEN_HP_LAUNCH(true, true, false); else DGEN_HP_LAUNCH(false, true, false);
        } else {
            // the bins-only form (NEM): no agent's bill is needed here, so no
            // hour writes the battery case's f64 system-output plane or takes
            // the net-billing branch; the dispatch, and so every plane, is the
            // same
#define DGEN_HP_LAUNCH_NEM(F)                                                                      \
            hipLaunchKernelGGL((k_hourly_batt<true, F, false, false, false, false, true>), grid, block, lds, s, *T, *A, \
                               *O, c->cfg, n, ws, n_scratch, (int64_t)0, n, m0, m1, c->battery, 0, 0, nullptr, 0, 0)
            if (O->hourly_f64) DGEN_HP_LAUNCH_NEM(true); else DGEN_HP_LAUNCH_NEM(false);
#undef DGEN_HP_LAUNCH_NEM
        }
#undef DGEN_HP_LAUNCH
    }
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

int32_t dgen_export_plane(dgen_ctx* c, const dgen_tables* T, const dgen_agents* A, const dgen_outputs* O,
                          const double* w_pvo, const double* w_batt, const double* w_non, double* plane,
                          int64_t n, void* ws, size_t ws_bytes, int64_t n_scratch, void* stream) {
    if (!c || !T || !A || !O || !w_pvo || !w_batt || !w_non || !plane) {
        set_err("dgen_export_plane: null argument");
        return DGEN_E_ARG;
    }
    if (n <= 0) return DGEN_OK;
    if (c->cfg.batt_loss_model == 1 || c->cfg.batt_update_hours == 1) {
        set_err("dgen_export_plane: the loss model / hourly re-plan scans export through dgen_hourly_planes");
        return DGEN_E_ARG;
    }
    if (!T->shapes || !T->shape_sum || !T->cfs || !T->tariffs || T->n_tariffs <= 0 ||
        (T->n_demand > 0 && !T->demand)) {
        set_err("dgen_export_plane: incomplete tables");
        return DGEN_E_ARG;
    }
    if (n >= ((int64_t)1 << 27) || n_scratch >= ((int64_t)1 << 28)) {
        set_err("dgen_export_plane: batch too large (n < 2^27)");
        return DGEN_E_ARG;
    }
    if (!ws || ws_bytes < dgen_workspace_bytes(n, n_scratch)) {
        set_err("dgen_export_plane: workspace too small (%zu < %zu)", ws_bytes, dgen_workspace_bytes(n, n_scratch));
        return DGEN_E_ARG;
    }
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    // the bins-only scan (as dgen_hourly_planes) writing the combined plane
    const size_t lds = sizeof(double) * 2 * (size_t)lds_half(T->max_periods) * BLOCK +
                       (size_t)(BLOCK / 64) * HB_DAY_BYTES;
    const dim3 grid((unsigned)((n + BLOCK - 1) / BLOCK)), block(BLOCK);
    for (int m0 = 0; m0 < 12; m0 += c->hb_months) {
        const int m1 = m0 + c->hb_months < 12 ? m0 + c->hb_months : 12;
        hipLaunchKernelGGL((k_hourly_batt<true, false, false, false, false, false, true, false, true>), grid, block,
                           lds, s, *T, *A, *O, c->cfg, n, ws, n_scratch, (int64_t)0, n, m0, m1, c->battery, 0, 0,
                           nullptr, 0, 0, 0, w_pvo, w_batt, w_non, plane);
    }
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

int32_t dgen_set_hourly_segment(dgen_ctx* c, int32_t months) {
    if (!c || months < 1 || months > 12) {
        set_err("dgen_set_hourly_segment: months must be in [1, 12]");
        return DGEN_E_ARG;
    }
    c->hb_months = months;
    return DGEN_OK;
}

int32_t dgen_set_dc_records(dgen_ctx* c, int32_t cap) {
    if (!c || cap < 0 || cap > DCR_CAP) {
        set_err("dgen_set_dc_records: cap must be in [0, %d]", DCR_CAP);
        return DGEN_E_ARG;
    }
    c->dcr_enable = cap;
    if (cap == 0 && c->dcr_buf) {   // records off: release their HBM (n_scratch x DCR_BYTES)
        HIP_TRY(hipStreamSynchronize(c->s2));
        HIP_TRY(hipFree(c->dcr_buf));
        c->dcr_buf = nullptr;
        c->dcr_cap = 0;
    }
    return DGEN_OK;
}

int32_t dgen_set_exact(dgen_ctx* c, int32_t mode) {
    if (!c || mode < 0 || mode > 2) { set_err("dgen_set_exact: mode must be 0, 1 or 2"); return DGEN_E_ARG; }
    c->exact = mode;
    return DGEN_OK;
}

int32_t dgen_exact_count(dgen_ctx* c, int64_t* out) {
    if (!c || !out) { set_err("dgen_exact_count: null argument"); return DGEN_E_ARG; }
    *out = 0;
    if (c->ex_last_nch == 0 || !c->ex_list) return DGEN_OK;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    for (int j = 0; j < c->ex_last_nch; j++) {
        int32_t k = 0;
        HIP_TRY(hipMemcpy(&k, c->ex_list + c->ex_last_off[j], sizeof(int32_t), hipMemcpyDeviceToHost));
        *out += k;
    }
    return DGEN_OK;
}

int32_t dgen_set_battery(dgen_ctx* c, int32_t on) {
    if (!c || (on != 0 && on != 1)) {
        set_err("dgen_set_battery: on must be 0 or 1");
        return DGEN_E_ARG;
    }
    c->battery = on;
    return DGEN_OK;
}

int32_t dgen_set_nb_scan(dgen_ctx* c, int32_t cap) {
    if (!c || cap < 0 || cap > DGEN_NB_CAPM) {
        set_err("dgen_set_nb_scan: cap must be in [0, %d]", DGEN_NB_CAPM);
        return DGEN_E_ARG;
    }
    c->nb_scan = cap;
    return DGEN_OK;
}

int32_t dgen_set_ts_rows(dgen_ctx* c, int64_t lo, int64_t hi) {
    if (!c || lo < 0 || hi < lo) {
        set_err("dgen_set_ts_rows: need 0 <= lo <= hi");
        return DGEN_E_ARG;
    }
    c->ts_lo = lo;
    c->ts_hi = hi;
    return DGEN_OK;
}

int32_t dgen_set_nem_rows(dgen_ctx* c, int64_t hi) {
    if (!c || hi < 0) {
        set_err("dgen_set_nem_rows: need hi >= 0");
        return DGEN_E_ARG;
    }
    c->nem_hi = hi;
    return DGEN_OK;
}

int32_t dgen_set_pipeline(dgen_ctx* c, int32_t chunks) {
    if (!c || chunks < 1 || chunks > dgen_ctx::MAXCH) {
        set_err("dgen_set_pipeline: chunks must be in [1, %d]", dgen_ctx::MAXCH);
        return DGEN_E_ARG;
    }
    c->chunks = chunks;
    return DGEN_OK;
}

int32_t dgen_set_dc_prebuild(dgen_ctx* c, int32_t on) {
    if (!c || (on != 0 && on != 1)) { set_err("dgen_set_dc_prebuild: on must be 0 or 1"); return DGEN_E_ARG; }
    c->dc_pre = on;
    return DGEN_OK;
}

int32_t dgen_last_paths(dgen_ctx* c, int32_t* out, int32_t n_out) {
    if (!c || !out || n_out < 0) { set_err("dgen_last_paths: null argument"); return DGEN_E_ARG; }
    for (int k = 0; k < n_out && k < DGEN_PATHS_N; k++) out[k] = c->last_paths[k];
    return DGEN_PATHS_N;
}

int32_t dgen_kernel_times(dgen_ctx* c, double* ms_size, double* ms_hourly, double* ms_finance) {
    if (!c) { set_err("dgen_kernel_times: null ctx"); return DGEN_E_ARG; }
    HIP_TRY(hipSetDevice(c->device));
    int start = (c->head - c->pending + dgen_ctx::RING) % dgen_ctx::RING;
    for (int k = 0; k < c->pending; k++) {
        int r = fold_one(c, (start + k) % dgen_ctx::RING);
        if (r) return r;
    }
    c->pending = 0;
    double cnt = c->count > 0 ? (double)c->count : 1.0;
    if (ms_size) *ms_size = c->sum_ms[0] / cnt;
    if (ms_hourly) *ms_hourly = c->sum_ms[1] / cnt;
    if (ms_finance) *ms_finance = c->sum_ms[2] / cnt;
    int64_t got = c->count;
    c->sum_ms[0] = c->sum_ms[1] = c->sum_ms[2] = 0.0;
    c->count = 0;
    return (int32_t)got;
}

int32_t dgen_segment_sums(dgen_ctx* c, const void* v1, const double* w1, const void* v2,
                          const double* w2, int32_t values_f32, int32_t k, int64_t n,
                          const int64_t* seg_off, int64_t n_seg, double* out, void* stream) {
    if (!c || !v1 || !seg_off || !out || k <= 0 || n < 0 || n_seg < 0 || (v2 && !w2) ||
        k > 65535) {
        set_err("dgen_segment_sums: bad argument");
        return DGEN_E_ARG;
    }
    if (n_seg == 0) return DGEN_OK;
    HIP_TRY(hipSetDevice(c->device));
    dim3 grid((unsigned)n_seg, (unsigned)k), block(256);
    if (values_f32)
        hipLaunchKernelGGL(k_segment_sums<float>, grid, block, 0, (hipStream_t)stream,
                           (const float*)v1, w1, (const float*)v2, w2, k, n, seg_off, n_seg, out);
    else
        hipLaunchKernelGGL(k_segment_sums<double>, grid, block, 0, (hipStream_t)stream,
                           (const double*)v1, w1, (const double*)v2, w2, k, n, seg_off, n_seg, out);
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

int32_t dgen_rows_seq_sum(dgen_ctx* c, const double* in, int64_t k, const int64_t* seg_off, int64_t n_seg,
                          double* out, void* stream) {
    if (!c || !in || !seg_off || !out || k <= 0 || n_seg < 0 || n_seg > 65535) {
        set_err("dgen_rows_seq_sum: bad argument");
        return DGEN_E_ARG;
    }
    if (n_seg == 0) return DGEN_OK;
    HIP_TRY(hipSetDevice(c->device));
    dim3 grid((unsigned)((k + 255) / 256), (unsigned)n_seg), block(256);
    hipLaunchKernelGGL(k_rows_seq_sum, grid, block, 0, (hipStream_t)stream, in, k, seg_off, n_seg, out);
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

int32_t dgen_max_market_share(dgen_ctx* c, const dgen_mms_table* tb, const double* payback,
                              const int32_t* mms_row, int64_t n, double* bounded, int64_t* factor,
                              double* mms, void* stream) {
    if (!c || !tb || !tb->mms || !payback || !mms_row || !bounded || !factor || !mms || n < 0 ||
        tb->n_rows < 0 || tb->n_factors < 0) {
        set_err("dgen_max_market_share: bad argument");
        return DGEN_E_ARG;
    }
    if (n == 0) return DGEN_OK;
    HIP_TRY(hipSetDevice(c->device));
    hipLaunchKernelGGL(k_max_market_share, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, *tb, payback, mms_row, n, bounded, factor, mms);
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

int32_t dgen_diffusion(dgen_ctx* c, const dgen_diffusion_in* in, const dgen_diffusion_out* out,
                       int64_t n, int32_t is_first_year, void* stream) {
    if (!c || !in || !out || n < 0) { set_err("dgen_diffusion: bad argument"); return DGEN_E_ARG; }
    const void* req[] = {in->max_market_share, in->market_share_last_year, in->bass_p, in->bass_q,
                         in->teq_yr1, in->developable_agent_weight, in->system_kw,
                         in->system_capex_per_kw, in->adopters_cum_last_year,
                         in->market_value_last_year, in->system_kw_cum_last_year,
                         out->mms_fix_zeros, out->ratio, out->bass_params_teq, out->teq2, out->f,
                         out->new_adopt_fraction, out->bass_market_share,
                         out->diffusion_market_share, out->market_share, out->new_market_share,
                         out->new_adopters, out->new_market_value, out->new_system_kw,
                         out->number_of_adopters, out->market_value, out->system_kw_cum};
    for (const void* p : req)
        if (!p) { set_err("dgen_diffusion: missing column"); return DGEN_E_ARG; }
    if (n == 0) return DGEN_OK;
    HIP_TRY(hipSetDevice(c->device));
    hipLaunchKernelGGL(k_diffusion, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, *in, *out, n, (int)is_first_year);
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

int32_t dgen_brent_selftest(dgen_ctx* c, const double* lo, const double* hi, const double* xatol,
                            const double* c2, const double* x0, const double* c1, int64_t n,
                            double* xs, int32_t maxn, double* xopt, int32_t* nfev, void* stream) {
    if (!c || !lo || !hi || !xatol || !c2 || !x0 || !c1 || !xs || !xopt || !nfev || maxn <= 0) {
        set_err("dgen_brent_selftest: bad argument");
        return DGEN_E_ARG;
    }
    if (n <= 0) return DGEN_OK;
    HIP_TRY(hipSetDevice(c->device));
    hipLaunchKernelGGL(k_brent_selftest, dim3((unsigned)((n + 63) / 64)), dim3(64), 0,
                       (hipStream_t)stream, lo, hi, xatol, c2, x0, c1, n, xs, maxn, xopt, nfev);
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

int32_t dgen_batt_attach(dgen_ctx* c, const dgen_attach_in* in, const dgen_attach_out* out,
                         const int64_t* seg_off, const double* rate, int64_t n_seg, void* stream) {
    if (!c || !in || !out || !seg_off || !rate || n_seg < 0) {
        set_err("dgen_batt_attach: bad argument");
        return DGEN_E_ARG;
    }
    if (n_seg == 0) return DGEN_OK;                                 // nothing to allocate
    const void* req[] = {in->new_adopters, in->aid_rank, in->batt_kw, in->batt_kwh,
                         in->batt_kw_cum_last_year, in->batt_kwh_cum_last_year, out->added,
                         out->new_batt_kw, out->new_batt_kwh, out->batt_kw_cum, out->batt_kwh_cum};
    for (const void* p : req)
        if (!p) { set_err("dgen_batt_attach: missing column"); return DGEN_E_ARG; }
    HIP_TRY(hipSetDevice(c->device));
    hipLaunchKernelGGL(k_batt_attach, dim3((unsigned)n_seg), dim3(ATT_BLOCK), 0, (hipStream_t)stream,
                       *in, *out, seg_off, rate, n_seg);
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

int32_t dgen_export_weights(dgen_ctx* c, const double* customers_in_bin,
                            const double* number_of_adopters, const double* batt_kw_cum_last_year,
                            const double* batt_kw, const int64_t* added, int64_t n, double* w_pvo,
                            double* w_batt, double* w_non, void* stream) {
    if (!c || !customers_in_bin || !number_of_adopters || !batt_kw_cum_last_year || !batt_kw ||
        !added || !w_pvo || !w_batt || !w_non || n < 0) {
        set_err("dgen_export_weights: bad argument");
        return DGEN_E_ARG;
    }
    if (n == 0) return DGEN_OK;
    HIP_TRY(hipSetDevice(c->device));
    hipLaunchKernelGGL(k_export_weights, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, customers_in_bin, number_of_adopters,
                       batt_kw_cum_last_year, batt_kw, added, n, w_pvo, w_batt, w_non);
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

int32_t dgen_state_hourly(dgen_ctx* c, const void* baseline, const void* pvonly,
                          const void* with_batt, int32_t planes_f32, const double* w_pvo,
                          const double* w_batt, const double* w_non, const int64_t* idx, int64_t n,
                          int32_t n_hours, const int64_t* seg_off, int64_t n_seg, double* out,
                          void* stream) {
    const bool comb = planes_f32 == 3;        // dgen_export_plane's combined plane in `baseline`
    if (!c || !baseline || (!comb && (!pvonly || !with_batt || !w_pvo || !w_batt || !w_non)) || !seg_off ||
        !out || n < 0 || n_hours <= 0 || n_seg < 0 || n_seg > 0x7fffffff) {
        set_err("dgen_state_hourly: bad argument");
        return DGEN_E_ARG;
    }
    if (planes_f32 < 0 || planes_f32 > 3) {
        set_err("dgen_state_hourly: planes_f32 must be 0 (f64 [h][n]), 1 (f32 tiles), 2 (f64 tiles) "
                "or 3 (the combined f64 plane, tiles)");
        return DGEN_E_ARG;
    }
    if (planes_f32 && n_hours % 4 != 0) {
        set_err("dgen_state_hourly: f32 (hour-quad tiled) planes need n_hours %% 4 == 0");
        return DGEN_E_ARG;
    }
    if (n_seg == 0) return DGEN_OK;
    HIP_TRY(hipSetDevice(c->device));
    const dim3 grid((unsigned)n_seg, (unsigned)((n_hours + SH_TILE - 1) / SH_TILE));
    if (comb)
        hipLaunchKernelGGL((k_state_hourly<double, true, true>), grid, dim3(256), 0, (hipStream_t)stream,
                           (const double*)baseline, nullptr, nullptr, nullptr, nullptr, nullptr, idx, n,
                           (int)n_hours, seg_off, n_seg, out);
    else if (planes_f32 == 2)
        hipLaunchKernelGGL((k_state_hourly<double, true>), grid, dim3(256), 0, (hipStream_t)stream,
                           (const double*)baseline, (const double*)pvonly, (const double*)with_batt,
                           w_pvo, w_batt, w_non, idx, n, (int)n_hours, seg_off, n_seg, out);
    else if (planes_f32)
        hipLaunchKernelGGL((k_state_hourly<float, true>), grid, dim3(256), 0, (hipStream_t)stream,
                           (const float*)baseline, (const float*)pvonly, (const float*)with_batt,
                           w_pvo, w_batt, w_non, idx, n, (int)n_hours, seg_off, n_seg, out);
    else
        hipLaunchKernelGGL((k_state_hourly<double, false>), grid, dim3(256), 0, (hipStream_t)stream,
                           (const double*)baseline, (const double*)pvonly, (const double*)with_batt,
                           w_pvo, w_batt, w_non, idx, n, (int)n_hours, seg_off, n_seg, out);
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

int32_t dgen_state_hourly_rows(dgen_ctx* c, const dgen_tables* T, const dgen_agents* A, const dgen_outputs* O,
                               const float* with_batt, const double* w_pvo, const double* w_batt,
                               const double* w_non, const int64_t* idx, int64_t n, const int64_t* seg_off,
                               int64_t n_seg, double* out, void* stream) {
    if (!c || !T || !A || !O || !with_batt || !w_pvo || !w_batt || !w_non || !seg_off || !out || n < 0 ||
        n_seg < 0 || n_seg > 0x7fffffff || !A->load_row || !A->cf_row || !A->load_kwh || !O->x_last ||
        !O->status || !T->shapes || !T->cfs || !T->shape_sum) {
        set_err("dgen_state_hourly_rows: bad argument");
        return DGEN_E_ARG;
    }
    if (n_seg == 0) return DGEN_OK;
    HIP_TRY(hipSetDevice(c->device));
    if ((size_t)n * sizeof(double2) > c->rows_cap) {        // per-agent scalars (grown on demand)
        if (c->rows_buf) {       // an earlier call may still read it on another stream
            HIP_TRY(hipDeviceSynchronize());
            HIP_TRY(hipFree(c->rows_buf));
        }
        c->rows_buf = nullptr;
        c->rows_cap = 0;
        HIP_TRY(hipMalloc(&c->rows_buf, (size_t)(n > 0 ? n : 1) * sizeof(double2)));
        c->rows_cap = (size_t)(n > 0 ? n : 1) * sizeof(double2);
    }
    double2* const scal = reinterpret_cast<double2*>(c->rows_buf);
    if (n > 0)
        hipLaunchKernelGGL(k_state_rows_prep, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                           *T, *A, *O, n, scal);
    const dim3 grid((unsigned)n_seg, (unsigned)((NH + SH_TILE - 1) / SH_TILE));
    hipLaunchKernelGGL(k_state_hourly_rows, grid, dim3(256), 0, (hipStream_t)stream, *T, *A, scal, with_batt,
                       w_pvo, w_batt, w_non, idx, n, seg_off, n_seg, out);
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

int32_t dgen_year_inputs(dgen_ctx* c, const dgen_year_keys* K, const dgen_year_tables* T,
                         const dgen_year_out* O, int64_t n, void* stream) {
    if (!c || !K || !T || !O || n < 0) { set_err("dgen_year_inputs: bad argument"); return DGEN_E_ARG; }
    if (n == 0) return DGEN_OK;
    const void* req[] = {K->k_sector, K->k_sector_county, K->k_state_sector, K->is_res, K->load_kwh_initial,
                         K->customers_initial, K->load_in_bin_initial, O->load_kwh, O->price_mult,
                         O->escalator, O->inflation, O->pv_deg, O->capex, O->capex_combined,
                         O->batt_capex_kwh, O->itc_frac, O->down_payment, O->real_discount, O->tax_rate,
                         O->vor, O->econ_life, O->loan_term, O->customers_in_bin, O->load_kwh_in_bin};
    for (const void* p : req)
        if (!p) { set_err("dgen_year_inputs: missing column"); return DGEN_E_ARG; }
    if ((T->n_sector > 0 && !T->by_sector) || (T->n_sector_county > 0 && !T->by_sector_county) ||
        (T->n_state_sector > 0 && !T->by_state_sector) || (O->wholesale_row && !K->k_county)) {
        set_err("dgen_year_inputs: missing table");
        return DGEN_E_ARG;
    }
    HIP_TRY(hipSetDevice(c->device));
    hipLaunchKernelGGL(k_year_inputs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       *K, *T, *O, n);
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

int32_t dgen_initial_market_shares(dgen_ctx* c, const dgen_init_in* in, const dgen_init_out* out,
                                   const int64_t* idx, const int64_t* seg_off, const double* caps,
                                   int64_t n_seg, void* stream) {
    if (!c || !in || !out || !idx || !seg_off || !caps || n_seg < 0) {
        set_err("dgen_initial_market_shares: bad argument");
        return DGEN_E_ARG;
    }
    if (n_seg == 0) return DGEN_OK;
    const void* req[] = {in->developable_agent_weight, in->system_capex_per_kw, out->adopters_cum_last_year,
                         out->system_kw_cum_last_year, out->batt_kw_cum_last_year, out->batt_kwh_cum_last_year,
                         out->market_share_last_year, out->market_value_last_year,
                         out->initial_number_of_adopters, out->initial_pv_kw, out->initial_batt_kw,
                         out->initial_batt_kwh, out->initial_market_share, out->initial_market_value,
                         out->developable_customers_in_state, out->agent_count};
    for (const void* p : req)
        if (!p) { set_err("dgen_initial_market_shares: missing column"); return DGEN_E_ARG; }
    if (n_seg > 0x7fffffff) { set_err("dgen_initial_market_shares: too many groups"); return DGEN_E_ARG; }
    HIP_TRY(hipSetDevice(c->device));
    hipLaunchKernelGGL(k_initial_shares, dim3((unsigned)n_seg), dim3(256), 0, (hipStream_t)stream, *in, *out,
                       idx, seg_off, caps, n_seg);
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

int32_t dgen_finance_series(dgen_ctx* c, const dgen_outputs* O, const int32_t* list_len, int64_t n,
                            double* out, void* stream) {
    if (!c || !O || !list_len || !out || n < 0) {
        set_err("dgen_finance_series: bad argument");
        return DGEN_E_ARG;
    }
    if (n == 0) return DGEN_OK;
    Series6 src = {{O->cfev_pv, O->bill_w_pv, O->bill_wo_pv, O->cfev_batt, O->bill_w_batt,
                    O->bill_wo_batt}};
    for (const double* p : src.p)
        if (!p) { set_err("dgen_finance_series: missing yearly output"); return DGEN_E_ARG; }
    HIP_TRY(hipSetDevice(c->device));
    const int64_t total = 6 * n * NORM25;
    hipLaunchKernelGGL(k_finance_series, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, src, list_len, n, (int32_t)(MAXY + 1), out);
    HIP_TRY(hipGetLastError());
    return DGEN_OK;
}

}  // extern "C"
#endif  // DGEN_TU_SEARCH
