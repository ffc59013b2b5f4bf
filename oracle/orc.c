/*
 * orc.c -- CPU oracle (TEST INFRASTRUCTURE ONLY; see orc.h for the contract).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp -shared).
 * Every function cites the reference code it restates.  SSC-side semantics
 * (Utilityrate5 / Cashloan / Battery) follow SAM's published methodology and
 * are parity-unpinned; DESIGN.md lists each modelling choice.
 */
#include "orc.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static const int kDaysInMonth[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};

/* ------------------------------------------------------------------------- */
/* numpy summation                                                            */
/* ------------------------------------------------------------------------- */

/* numpy/_core/src/umath/loops_utils.h.src  <TYPE>_pairwise_sum: blocks of <=128
 * with 8 interleaved accumulators, halving split rounded down to a multiple of 8. */
double orc_pairwise_sum(const double* a, int64_t n) {
    if (n < 8) {
        double res = 0.0;
        for (int64_t i = 0; i < n; i++) res += a[i];
        return res;
    }
    if (n <= 128) {
        double r[8];
        int64_t i;
        for (int j = 0; j < 8; j++) r[j] = a[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return orc_pairwise_sum(a, n2) + orc_pairwise_sum(a + n2, n - n2);
}

/* np.add.reduce on a 1-D contiguous float64 array: the buffered reduction
 * iterator feeds the pairwise inner loop 8192 elements at a time into an output
 * seeded with 0 (verified bit-exact against numpy 2.2.6 in tests/test_oracle.py). */
double orc_np_sum(const double* a, int64_t n) {
    double res = 0.0;
    for (int64_t s = 0; s < n; s += 8192) {
        int64_t m = n - s < 8192 ? n - s : 8192;
        res += orc_pairwise_sum(a + s, m);
    }
    return res;
}

/* np.round(x, 1) for float64: y = x * 10; rint(y) / 10 (round-half-even). */
double orc_np_round1(double x) {
    double y = x * 10.0;
    return nearbyint(y) / 10.0;
}

/* exact-order integer power used for every escalation factor (documented
 * replacement for SSC's pow(): sequential multiplication, identical on device) */
static double pow_int(double b, int e) {
    double r = 1.0;
    for (int i = 0; i < e; i++) r = r * b;
    return r;
}

/* ------------------------------------------------------------------------- */
/* tariff                                                                     */
/* ------------------------------------------------------------------------- */

/* Consume the fields process_tariff() writes (financial_functions.py:617-622):
 * ur_ec_tou_mat rows [period, tier, max_usage, unit, buy, sell] and the 12x24
 * schedules.  normalize_tariff (ff:962-1007) has already made periods 1..P
 * contiguous, tiers equal per period and caps single-valued per tier. */
int orc_tariff_from_mat(orc_tariff* t, const double* mat, int nrows, int mo, double fixed,
                        const int32_t* wk, const int32_t* we) {
    memset(t, 0, sizeof(*t));
    t->mo = mo;
    t->fixed = fixed;
    if (nrows <= 0) { /* empty matrix: no energy charges (status flagged by caller) */
        t->P = 1; t->T = 1; t->cap[0] = 1e38;
    } else {
        int P = 0, T = 0;
        for (int i = 0; i < nrows; i++) {
            int p = (int)mat[i * 6 + 0], k = (int)mat[i * 6 + 1];
            if (p > P) P = p;
            if (k > T) T = k;
        }
        if (P < 1 || T < 1 || P > ORC_MAXP || T > ORC_MAXT) return -1;
        if (nrows != P * T) return -2;
        t->P = P; t->T = T;
        t->unit = (int)mat[3];
        for (int i = 0; i < nrows; i++) {
            int p = (int)mat[i * 6 + 0] - 1, k = (int)mat[i * 6 + 1] - 1;
            if (p < 0 || k < 0) return -3;
            t->cap[k] = mat[i * 6 + 2];
            t->buy[p][k] = mat[i * 6 + 4];
            t->sell[p][k] = mat[i * 6 + 5];
        }
    }
    for (int m = 0; m < 12; m++)
        for (int h = 0; h < 24; h++) {
            int a = wk ? wk[m * 24 + h] : 1, b = we ? we[m * 24 + h] : 1;
            if (a < 1 || a > t->P) a = 1;
            if (b < 1 || b > t->P) b = 1;
            t->wkday[m][h] = (uint8_t)(a - 1);
            t->wkend[m][h] = (uint8_t)(b - 1);
        }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Utilityrate5 subset                                                        */
/* ------------------------------------------------------------------------- */

/* Hour -> (month, period).  SSC util::translate_schedule: the year starts on a
 * Monday, hours (i % 168) >= 120 are weekend. */
static void hour_calendar(const orc_tariff* t, int* month_of, int* period_of) {
    int i = 0;
    for (int m = 0; m < 12; m++)
        for (int d = 0; d < kDaysInMonth[m]; d++)
            for (int h = 0; h < 24; h++, i++) {
                int weekend = (i % 168) >= 120;
                month_of[i] = m;
                period_of[i] = weekend ? t->wkend[m][h] : t->wkday[m][h];
            }
}

/* Energy charge for one month: tier amounts from total monthly usage U, each
 * period billed its share u_p/U of every tier at its own price.  One tier:
 * every period's kWh at its own price, sum_p u_p * buy_p (the same quantity
 * without the share / re-multiplication round trip). */
/* Tier caps per usage unit (the compile's code, ff:778-779, harmonised to one
 * code per tariff, ff:939-956): 0 kWh, 2 kWh daily (x days in month), 1 kWh/kW
 * (x the month's peak demand: the largest hourly grid import of the billed
 * case, kW; SSC's billing demand with ur_enable_billing_demand = 0, ff:614),
 * 3 kWh/kW daily (x peak x days).  Parity unpinned (SSC restatement). */
static double month_energy_charge(const orc_tariff* t, int m, const double* u, double peak) {
    double U = 0.0;
    for (int p = 0; p < t->P; p++) U += u[p];
    if (!(U > 0.0)) return 0.0;
    if (t->T == 1) {
        double charge = 0.0;
        for (int p = 0; p < t->P; p++) charge += u[p] * t->buy[p][0];
        return charge;
    }
    const double days = (double)kDaysInMonth[m];
    double scale = (t->unit == 2) ? days : (t->unit == 1) ? peak : (t->unit == 3) ? peak * days : 1.0;
    double charge = 0.0, prev = 0.0;
    for (int k = 0; k < t->T; k++) {
        double hi = (k == t->T - 1) ? INFINITY : t->cap[k] * scale;
        double top = U < hi ? U : hi;
        double amt = top - prev;
        if (amt < 0.0) amt = 0.0;
        if (hi > prev) prev = hi;
        for (int p = 0; p < t->P; p++) charge += (u[p] / U) * amt * t->buy[p][k];
    }
    return charge;
}

/* One year's bill (undiscounted, before the escalation factor), by metering
 * option (SAM's enumeration; the reference passes the tariff's value through,
 * ff:586-588, 970-971; only 0 and 2 have the reference's semantics pinned by
 * its own code paths, all of them are SSC restatements, parity unpinned):
 *   0  net metering, kWh credits: monthly net kWh per period, surplus kWh
 *      carried per period, December true-up at ur_nm_yearend_sell_rate;
 *   1  net metering, $ credits: monthly net kWh per period, imports billed,
 *      surplus kWh credited at the period's tier-1 sell rate; the month's
 *      energy bill floors at 0 with the excess $ carried to the next month
 *      (lost at year end);
 *   2  net billing: hourly imports billed, hourly exports credited at the
 *      period's tier-1 sell rate or the 8760 TS sell rate;
 *   3  net billing with carryover: as 2, the month's energy bill floors at 0
 *      and the excess $ carries to the next month (lost at year end);
 *   4  buy all / sell all: all load billed, all generation credited at the
 *      period's tier-1 sell rate.
 * Fixed charges are always billed. */
static double year_bill(const orc_tariff* t, const orc_cfg* cfg, const double* net /*[12][P]*/,
                        const double* imp, const double* exv /*[12][P] $ or kWh*/, const double* lbin,
                        const double* gbin, const double* peak /*[12]*/, int ts) {
    double total = 0.0, carry = 0.0;
    double credit[ORC_MAXP];
    for (int p = 0; p < ORC_MAXP; p++) credit[p] = 0.0;
    for (int m = 0; m < 12; m++) {
        double u[ORC_MAXP];
        double bill = t->fixed;
        if (t->mo == 0) {
            for (int p = 0; p < t->P; p++) {
                double n = net[m * ORC_MAXP + p];
                if (n >= 0.0) {
                    double use = n < credit[p] ? n : credit[p];
                    u[p] = n - use;
                    credit[p] -= use;
                } else {
                    u[p] = 0.0;
                    credit[p] += -n;
                }
            }
            bill += month_energy_charge(t, m, u, peak[m]);
            if (m == 11) {
                double c = 0.0;
                for (int p = 0; p < t->P; p++) c += credit[p];
                bill -= c * cfg->nm_yearend_sell_rate;
            }
        } else if (t->mo == 1) {
            double cr = 0.0;
            for (int p = 0; p < t->P; p++) {
                double n = net[m * ORC_MAXP + p];
                u[p] = n > 0.0 ? n : 0.0;
                cr += (n < 0.0 ? -n : 0.0) * t->sell[p][0];
            }
            double e = month_energy_charge(t, m, u, peak[m]) - cr - carry;
            carry = e < 0.0 ? -e : 0.0;
            bill += e < 0.0 ? 0.0 : e;
        } else if (t->mo == 4) {
            double cr = 0.0;
            for (int p = 0; p < t->P; p++) {
                u[p] = lbin[m * ORC_MAXP + p];
                cr += gbin[m * ORC_MAXP + p] * t->sell[p][0];
            }
            bill += month_energy_charge(t, m, u, peak[m]) - cr;
        } else {
            double cr = 0.0;
            for (int p = 0; p < t->P; p++) u[p] = imp[m * ORC_MAXP + p];
            double charge = month_energy_charge(t, m, u, peak[m]);
            if (ts) {
                for (int p = 0; p < t->P; p++) cr += exv[m * ORC_MAXP + p];
            } else {
                for (int p = 0; p < t->P; p++) cr += exv[m * ORC_MAXP + p] * t->sell[p][0];
            }
            if (t->mo == 3) {
                double e = charge - cr - carry;
                carry = e < 0.0 ? -e : 0.0;
                bill += e < 0.0 ? 0.0 : e;
            } else {
                bill += charge;
                bill -= cr;
            }
        }
        total += bill;
    }
    return total;
}

/* Bins one year: gen scaled by s (degradation), hour by hour in time order;
 * peak[m] = the month's largest hourly grid import (0 without import). */
static void bin_year(const orc_tariff* t, const int* mon, const int* per, const double* gen,
                     const double* load, const double* ts, double s, double* net, double* imp,
                     double* exv, double* lbin, double* gbin, double* peak) {
    for (int i = 0; i < 12 * ORC_MAXP; i++) net[i] = imp[i] = exv[i] = lbin[i] = gbin[i] = 0.0;
    for (int m = 0; m < 12; m++) peak[m] = 0.0;
    for (int h = 0; h < ORC_NH; h++) {
        double g = gen ? gen[h] * s : 0.0;
        double d = load[h] - g;            /* > 0: import */
        int b = mon[h] * ORC_MAXP + per[h];
        if (d > peak[mon[h]]) peak[mon[h]] = d;
        net[b] += d;
        lbin[b] += load[h];
        gbin[b] += g;
        if (d > 0.0) {
            imp[b] += d;
        } else {
            double e = -d;
            exv[b] += ts ? e * ts[h] : e;
        }
    }
}

/* Demand charge of one tier table: the last tier is unbounded above. */
static double dc_tier_charge(double peak, const double* cap, const double* price, int nt) {
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

/* One year's demand charges (extension mode, parity unpinned): per month the
 * flat peak = max hourly grid import, and per TOU demand period the max over
 * that period's hours; no import -> peak 0.  Hours in time order, the calendar
 * of hour_calendar.  Month charge = flat tiers, then periods 0..ORC_DCP-1. */
static double year_demand(const orc_tariff* t, const double* gen, const double* load, double s) {
    double total = 0.0;
    int i = 0;
    for (int m = 0; m < 12; m++) {
        double flat = 0.0, pk[ORC_DCP];
        for (int p = 0; p < ORC_DCP; p++) pk[p] = 0.0;
        for (int d = 0; d < kDaysInMonth[m]; d++)
            for (int h = 0; h < 24; h++, i++) {
                int weekend = (i % 168) >= 120;
                int p = weekend ? t->dc_wkend[m][h] : t->dc_wkday[m][h];
                double g = gen ? gen[i] * s : 0.0;
                double imp = load[i] - g;
                if (imp > flat) flat = imp;
                if (imp > pk[p]) pk[p] = imp;
            }
        double c = dc_tier_charge(flat, t->dc_flat_cap[m], t->dc_flat_price[m], t->dc_flat_nt[m]);
        for (int p = 0; p < ORC_DCP; p++)
            c += dc_tier_charge(pk[p], t->dc_tou_cap[p], t->dc_tou_price[p], t->dc_tou_nt[p]);
        total += c;
    }
    return total;
}

/* cmod_utilityrate5 as driven at ff:364-368,258-270: analysis_period years,
 * system_use_lifetime_output = 0, degradation (%/yr, compounding),
 * rate escalation (1 + inflation + escalation)^i, outputs index 0 = 0. */
int orc_ur5(const orc_tariff* t, const orc_cfg* cfg, const double* gen, const double* load,
            const double* ts_sell, int nyears, double inflation_pct, double escal_pct,
            double degr_pct, double* bill_w, double* bill_wo, double* aev, double* e_fromgrid) {
    if (nyears < 1 || nyears > ORC_MAXY) return -1;
    int mon[ORC_NH], per[ORC_NH];
    hour_calendar(t, mon, per);
    int ts = (t->mo == 2) && ts_sell != NULL;
    const double* tsp = ts ? ts_sell : NULL;
    double net[12 * ORC_MAXP], imp[12 * ORC_MAXP], exv[12 * ORC_MAXP];
    double lbin[12 * ORC_MAXP], gbin[12 * ORC_MAXP], peak[12];
    double rate_base = 1.0 + inflation_pct * 0.01 + escal_pct * 0.01;
    double sys_base = 1.0 - degr_pct * 0.01;

    bin_year(t, mon, per, NULL, load, tsp, 1.0, net, imp, exv, lbin, gbin, peak);
    double wo1 = year_bill(t, cfg, net, imp, exv, lbin, gbin, peak, ts);
    if (t->dc_on) wo1 += year_demand(t, NULL, load, 1.0);
    bill_w[0] = bill_wo[0] = aev[0] = 0.0;
    for (int i = 0; i < nyears; i++) {
        double r = pow_int(rate_base, i);
        double s = pow_int(sys_base, i);
        bin_year(t, mon, per, gen, load, tsp, s, net, imp, exv, lbin, gbin, peak);
        double wb = year_bill(t, cfg, net, imp, exv, lbin, gbin, peak, ts);
        if (t->dc_on) wb += year_demand(t, gen, load, s);
        double w = wb * r;
        double wo = wo1 * r;
        bill_w[i + 1] = w;
        bill_wo[i + 1] = wo;
        aev[i + 1] = wo - w;
    }
    if (e_fromgrid) {
        for (int h = 0; h < ORC_NH; h++) {
            double d = load[h] - (gen ? gen[h] : 0.0);
            e_fromgrid[h] = d > 0.0 ? d : 0.0;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Cashloan subset                                                            */
/* ------------------------------------------------------------------------- */

static double depr_frac(int type, int year, int sl_years) {
    static const double macrs5[6] = {0.20, 0.32, 0.192, 0.1152, 0.1152, 0.0576};
    if (type == 1) return (year >= 1 && year <= 6) ? macrs5[year - 1] : 0.0;
    if (type == 2) return (year >= 1 && year <= sl_years) ? 1.0 / (double)sl_years : 0.0;
    return 0.0;
}

/* cmod_cashloan as driven at ff:272-288,385-421: after-tax cash flows, NPV at
 * the nominal discount rate (Horner form of SSC libfin::npv), payback from the
 * cumulative cf_payback_with_expenses (SSC compute_payback, 1e99 if none). */
/* NPV association (diagnostics only): 0 = SSC's libfin::npv order (default) */
int orc_npv_order = 0;
void orc_set_npv_order(int k) { orc_npv_order = k; }

int orc_cashloan(const orc_loan_in* in, const orc_cfg* cfg, const double* aev, double* npv,
                 double* payback, double* cf_payback, double* cf_energy_value) {
    int N = in->nyears;
    if (N < 1 || N > ORC_MAXY) return -1;
    double C = in->total_cost;
    double infl = in->inflation_pct * 0.01;
    double real = in->real_disc_pct * 0.01;
    double nom = (1.0 + real) * (1.0 + infl) - 1.0;
    double fed = in->fed_tax_pct * 0.01, sta = in->sta_tax_pct * 0.01;
    double debt = in->debt_fraction_pct * 0.01 * C;
    double r = cfg->loan_rate_pct * 0.01;
    int term = in->loan_term;
    double pmt = 0.0;
    if (term > 0 && debt != 0.0) {
        if (r != 0.0) {
            double f = pow_int(1.0 + r, term);
            pmt = debt * r / (1.0 - 1.0 / f);
        } else {
            pmt = debt / (double)term;
        }
    }
    double itc = in->itc_fed_pct * 0.01 * C;
    if (itc > cfg->itc_fed_max) itc = cfg->itc_fed_max;
    double basis = C - 0.5 * itc;
    double ins = cfg->insurance_rate_pct * 0.01 * C;

    double atcf[ORC_MAXY + 1];
    double balance = debt;
    atcf[0] = -(C - debt);
    cf_payback[0] = -C;
    cf_energy_value[0] = 0.0;
    for (int i = 1; i <= N; i++) {
        double ev = aev[i];
        double oe = ins * pow_int(1.0 + infl, i - 1);
        double interest = 0.0, payment = 0.0;
        if (i <= term && pmt != 0.0) {
            interest = balance * r;
            payment = pmt;
            balance = balance - (pmt - interest);
        }
        double itc_i = (i == 1) ? itc : 0.0;
        double sta_tax_i = 0.0, fed_tax_i = 0.0;
        if (in->market != 0) {
            double dep_s = depr_frac(in->depr_sta_type, i, cfg->depr_sl_years) * basis;
            double dep_f = depr_frac(in->depr_fed_type, i, cfg->depr_sl_years) * basis;
            sta_tax_i = sta * (ev - oe - interest - dep_s);
            fed_tax_i = fed * (ev - oe - interest - dep_f - sta_tax_i);
        }
        double taxsav = itc_i - sta_tax_i - fed_tax_i;
        atcf[i] = ev - oe - payment + taxsav;
        cf_payback[i] = ev - oe + taxsav;
        cf_energy_value[i] = ev;
    }
    double rr = 1.0 / (1.0 + nom);
    double acc = 0.0;
    if (orc_npv_order == 1) {
        /* diagnostics only: the association of a 32/64-lane xor butterfly
         * over atcf_y rr^y (the device's round-4 form) */
        int W = N <= 32 ? 32 : 64;
        double v[64];
        for (int k = 0; k < W; k++) {
            double df = 1.0;
            for (int j = 0; j <= k; j++) df *= rr;
            v[k] = (k < N) ? atcf[k + 1] * df : 0.0;
        }
        for (int o = W / 2; o > 0; o >>= 1) {
            double t[64];
            for (int k = 0; k < W; k++) t[k] = v[k] + v[k ^ o];
            for (int k = 0; k < W; k++) v[k] = t[k];
        }
        *npv = -(C - debt) + v[0];
    } else {
        for (int i = N; i > 0; i--) acc = rr * acc + atcf[i];
        *npv = atcf[0] + acc * rr;
    }

    double cum = cf_payback[0];
    double pb = 1e99;
    for (int i = 1; i <= N; i++) {
        cum += cf_payback[i];
        if (cum > 0.0) {
            pb = (cf_payback[i] != 0.0) ? (double)i - cum / cf_payback[i] : (double)i - 0.5;
            break;
        }
    }
    *payback = pb;
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Battery subset                                                             */
/* ------------------------------------------------------------------------- */

/* PySAM.BatteryTools.battery_model_sizing (ff:140-147): cells in series to reach
 * the voltage, strings to reach the capacity, C-rate preserved for power. */
void orc_batt_size(double desired_kw, double desired_kwh, double desired_v, const orc_cfg* cfg,
                   double* bank_kwh, double* power_kw) {
    if (!(desired_kwh > 0.0)) { *bank_kwh = 0.0; *power_kw = 0.0; return; }
    double series = ceil(desired_v / cfg->batt_v_nom);
    double strings = floor(desired_kwh * 1000.0 / (cfg->batt_q_full * cfg->batt_v_nom * series) + 0.5);
    if (strings < 1.0) strings = 1.0;
    double bank = cfg->batt_q_full * cfg->batt_v_nom * series * strings * 0.001;
    *bank_kwh = bank;
    *power_kw = bank * (desired_kw / desired_kwh);
}

/* Peak-shaving target with perfect 24 h look-ahead: the smallest grid
 * import level T >= 0 such that holding imports at T needs no more than the
 * energy stored at the start of the day:
 *     f(T) = sum_h min(max(d_h - T, 0), P) <= E,   d_h = max(load_h - pv_h, 0).
 * f is continuous, non-increasing and piecewise linear with breakpoints at d_h
 * and d_h - P.  If no d_h exceeds P, f is convex and Newton from T = 0 is
 * exact in a few steps.  Otherwise bisect [0, max d] until no breakpoint lies
 * inside the bracket (the counts a = #{d > T} and b = #{d - P >= T} agree at
 * both ends), then solve the linear piece exactly (slope -(a - b)). */
/* Daily peak-shaving target: smallest T >= 0 with
 * f(T) = sum_h min(max(d_h - T, 0), P) <= E over the day's deficits
 * d_h = max(load_h - pv_h, 0), evaluated on the deficits sorted descending
 * (s[0] = max; every sum below runs in that order, as on the device).
 * No saturated hour (s[0] <= P): f(T) = max_k (S_k - k T), S_k the sum of the
 * k largest, so T = (S_K - E) / K for the largest K with S_K - K s[K-1] <= E.
 * Otherwise bisection until no breakpoint (s_k, s_k - P) lies inside the
 * bracket, then the exact linear piece. */
/* The window is hours h0 .. h0 + 23; past the last hour of the year it wraps
 * to the first (a typical year repeats: the forecast for January 1 of the next
 * year is this year's January 1).  Only the hourly re-plan reaches past 8759. */
static double day_target(const double* load, const double* pv, int h0, double power, double avail) {
    double s[24];
    for (int k = 0; k < 24; k++) {
        const int h = (h0 + k) % ORC_NH;
        double v = load[h] - pv[h];
        s[k] = v > 0.0 ? v : 0.0;
    }
    for (int i = 1; i < 24; i++) {          /* insertion sort, descending */
        double x = s[i];
        int j = i - 1;
        while (j >= 0 && s[j] < x) { s[j + 1] = s[j]; j--; }
        s[j + 1] = x;
    }
    double need0 = 0.0;
    for (int k = 0; k < 24; k++) need0 += s[k] < power ? s[k] : power;
    if (need0 <= avail) return 0.0;
    if (s[0] <= power) {
        double S = 0.0, SK = s[0];
        int K = 1;
        for (int k = 1; k <= 24; k++) {
            S += s[k - 1];
            if (S - (double)k * s[k - 1] <= avail) { K = k; SK = S; }
        }
        return (SK - avail) / (double)K;
    }
    int a_lo = 0, b_lo = 0;
    for (int k = 0; k < 24; k++) {
        a_lo += s[k] > 0.0;
        b_lo += (s[k] - power) >= 0.0;
    }
    double lo = 0.0, hi = s[0], f_hi = 0.0;
    int a_hi = 0, b_hi = 0;
    for (int it = 0; it < 48; it++) {
        if (a_lo == a_hi && b_lo == b_hi) break;
        double mid = 0.5 * (lo + hi);
        double f = 0.0;
        int am = 0, bm = 0;
        for (int k = 0; k < 24; k++) {
            double e = s[k] - mid;
            am += e > 0.0;
            bm += (e - power) >= 0.0;
            if (e < 0.0) e = 0.0;
            f += e < power ? e : power;
        }
        if (f <= avail) { hi = mid; f_hi = f; a_hi = am; b_hi = bm; }
        else { lo = mid; a_lo = am; b_lo = bm; }
    }
    int k = a_hi - b_hi;
    if (k <= 0) return hi;
    double t = hi - (avail - f_hi) / (double)k;
    if (t < lo) t = lo;
    if (t > hi) t = hi;
    return t;
}

/* BTM dispatch (bdh:59-98): peak shaving with 24 h look-ahead, charge only from
 * PV surplus, no grid charging, discharge whenever imports exceed the target.
 * Re-plan interval (cfg->batt_update_hours):
 *   24  one plan per calendar day, made at its first hour from the energy
 *       stored then over that day's 24 hours (SSC's BTM peak-shaving update);
 *    1  a plan every hour from the energy stored at that hour over the next 24
 *       hours (bdh:86-87 read literally: batt_look_ahead_hours = 24,
 *       batt_dispatch_update_frequency_hours = 1).  A plan only matters in an
 *       hour that can discharge (net load > 0, energy stored > 0), so the
 *       hourly rule forms it only there; the result is the same.            */
/* Li-ion loss model (cfg->batt_loss_model = 1): converters of efficiency
 * batt_conv_eff each way, and the cells' I^2 R at the bank's open-circuit
 * voltage.  With s cells in series and p strings (battery_model_sizing) the
 * bank has V(soc) = s (v_e + (v_f - v_e) soc) and R = s r / p, so a DC power x
 * (kW) loses k x^2 with k = 1000 R / V^2 = r q v_nom / (bank_kwh v(soc)^2)
 * (s p = 1000 bank_kwh / (q v_nom)).  k is taken at the hour's starting SOC.
 * Charging c kW (AC) stores x - k x^2, x = c eta; discharging d kW (AC) draws
 * y + k y^2, y = d / eta.  The limits are the roots of those quadratics,
 * in their cancellation-free forms:
 *   room:  x_max = 2 E_room / (1 + sqrt(1 - 4 k E_room))  (x up to 1 / 2k)
 *   avail: y_max = 2 E_av / (1 + sqrt(1 + 4 k E_av))
 * The day's plan uses the deliverable energy without the cell losses,
 * E_av eta (the per-hour limits are exact). */
static double loss_k(const orc_cfg* cfg, double soc, double bank_kwh) {
    const double v = cfg->batt_v_cell_empty + (cfg->batt_v_cell_full - cfg->batt_v_cell_empty) * soc;
    return cfg->batt_r_cell * cfg->batt_q_full * cfg->batt_v_nom / (bank_kwh * (v * v));
}

void orc_batt_dispatch(const double* load, const double* pv, double bank_kwh, double power_kw,
                       const orc_cfg* cfg, double* sysgen, double* grid_to_load) {
    double soc = cfg->batt_init_soc;
    double target = 0.0;
    const int hourly = cfg->batt_update_hours == 1;
    /* per-step constants (multiplications instead of divisions in the scan) */
    const double inv_eta_in = 1.0 / cfg->batt_eta_in;
    const double in_per_bank = bank_kwh > 0.0 ? cfg->batt_eta_in / bank_kwh : 0.0;
    const double out_per_bank = bank_kwh > 0.0 ? 1.0 / (cfg->batt_eta_out * bank_kwh) : 0.0;
    const int loss = cfg->batt_loss_model == 1;
    const double eta = cfg->batt_conv_eff;
    /* monthly target floor (cfg->batt_month_floor): a plan's target is raised
     * to the largest target planned earlier in the month, and raises it */
    const int mfl = cfg->batt_month_floor == 1;
    double floor_t = 0.0;
    int month = 0, next_month_h = kDaysInMonth[0] * 24;
    for (int h = 0; h < ORC_NH; h++) {
        double n = load[h] - pv[h];
        if (h == next_month_h) {
            month++;
            next_month_h += kDaysInMonth[month] * 24;
            floor_t = 0.0;
        }
        if (!(bank_kwh > 0.0)) {
            sysgen[h] = pv[h];
            grid_to_load[h] = n > 0.0 ? n : 0.0;
            continue;
        }
        if (loss) {
            if (h % 24 == 0 || hourly) {
                double e_av = (soc - cfg->batt_min_soc) * bank_kwh;
                if (e_av < 0.0) e_av = 0.0;
                if (!hourly) target = day_target(load, pv, h, power_kw, e_av * eta);
                else target = (n > 0.0 && e_av > 0.0) ? day_target(load, pv, h, power_kw, e_av * eta) : 0.0;
                if (mfl && (!hourly || (n > 0.0 && e_av > 0.0))) {
                    if (target < floor_t) target = floor_t;
                    else floor_t = target;
                }
            }
            const double k = loss_k(cfg, soc, bank_kwh);
            if (n < 0.0) {
                double e_room = (cfg->batt_max_soc - soc) * bank_kwh;
                if (e_room < 0.0) e_room = 0.0;
                const double disc = 1.0 - 4.0 * k * e_room;
                const double x_max = disc > 0.0 ? 2.0 * e_room / (1.0 + sqrt(disc)) : 0.5 / k;
                double c = -n;
                if (c > power_kw) c = power_kw;
                if (c > x_max / eta) c = x_max / eta;
                const double x = c * eta;
                soc = soc + (x - k * (x * x)) / bank_kwh;
                sysgen[h] = pv[h] - c;
                grid_to_load[h] = 0.0;
            } else {
                double e_av = (soc - cfg->batt_min_soc) * bank_kwh;
                if (e_av < 0.0) e_av = 0.0;
                const double y_max = 2.0 * e_av / (1.0 + sqrt(1.0 + 4.0 * k * e_av));
                double d = n - target;
                if (d < 0.0) d = 0.0;
                if (d > power_kw) d = power_kw;
                if (d > y_max * eta) d = y_max * eta;
                const double y = d / eta;
                soc = soc - (y + k * (y * y)) / bank_kwh;
                sysgen[h] = pv[h] + d;
                grid_to_load[h] = n - d;
            }
            continue;
        }
        if (!hourly && h % 24 == 0) {
            double avail = (soc - cfg->batt_min_soc) * bank_kwh * cfg->batt_eta_out;
            if (avail < 0.0) avail = 0.0;
            target = day_target(load, pv, h, power_kw, avail);
            if (mfl) {
                if (target < floor_t) target = floor_t;
                else floor_t = target;
            }
        }
        if (n < 0.0) {
            double room = (cfg->batt_max_soc - soc) * bank_kwh * inv_eta_in;
            if (room < 0.0) room = 0.0;
            double c = -n;
            if (c > power_kw) c = power_kw;
            if (c > room) c = room;
            soc = soc + c * in_per_bank;
            sysgen[h] = pv[h] - c;
            grid_to_load[h] = 0.0;
        } else {
            double avail = (soc - cfg->batt_min_soc) * bank_kwh * cfg->batt_eta_out;
            if (avail < 0.0) avail = 0.0;
            if (hourly) {
                target = (n > 0.0 && avail > 0.0) ? day_target(load, pv, h, power_kw, avail) : 0.0;
                if (mfl && n > 0.0 && avail > 0.0) {
                    if (target < floor_t) target = floor_t;
                    else floor_t = target;
                }
            }
            double d = n - target;
            if (d < 0.0) d = 0.0;
            if (d > power_kw) d = power_kw;
            if (d > avail) d = avail;
            soc = soc - d * out_per_bank;
            sysgen[h] = pv[h] + d;
            grid_to_load[h] = n - d;
        }
    }
}

/* ------------------------------------------------------------------------- */
/* scipy 1.15.3 _minimize_scalar_bounded (scipy/optimize/_optimize.py:2251)   */
/* ------------------------------------------------------------------------- */

typedef double (*orc_obj_fn)(double x, void* ctx);

static double np_sign(double v) { return (v > 0.0) ? 1.0 : ((v < 0.0) ? -1.0 : 0.0); }

/* Optional evaluation trace (diagnostics only, this thread): (x, f) pairs of
 * every bounded-Brent evaluation, set with orc_set_trace(buf, max). */
static __thread double* orc_trace_buf = 0;
static __thread int orc_trace_max = 0, orc_trace_n = 0;
void orc_set_trace(double* buf, int max) { orc_trace_buf = buf; orc_trace_max = max; orc_trace_n = 0; }
int orc_trace_count(void) { return orc_trace_n; }
static double traced(orc_obj_fn f, void* ctx, double x) {
    double v = f(x, ctx);
    if (orc_trace_buf && orc_trace_n < orc_trace_max) {
        orc_trace_buf[2 * orc_trace_n] = x;
        orc_trace_buf[2 * orc_trace_n + 1] = v;
    }
    if (orc_trace_buf) orc_trace_n++;
    return v;
}

static double brent_bounded(orc_obj_fn f, void* ctx, double x1, double x2, double xatol,
                            int maxfun, int* nfev) {
    const double sqrt_eps = sqrt(2.2e-16);
    const double golden_mean = 0.5 * (3.0 - sqrt(5.0));
    double a = x1, b = x2;
    double fulc = a + golden_mean * (b - a);
    double nfc = fulc, xf = fulc;
    double rat = 0.0, e = 0.0;
    double x = xf;
    double fx = traced(f, ctx, x);
    int num = 1;
    double ffulc = fx, fnfc = fx;
    double xm = 0.5 * (a + b);
    double tol1 = sqrt_eps * fabs(xf) + xatol / 3.0;
    double tol2 = 2.0 * tol1;
    while (fabs(xf - xm) > (tol2 - 0.5 * (b - a))) {
        int golden = 1;
        if (fabs(e) > tol1) {
            golden = 0;
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
                golden = 1;
            }
        }
        if (golden) {
            if (xf >= xm) e = a - xf; else e = b - xf;
            rat = golden_mean * e;
        }
        double si = np_sign(rat) + ((rat == 0.0) ? 1.0 : 0.0);
        double ar = fabs(rat);
        x = xf + si * (ar > tol1 ? ar : tol1);   /* np.maximum(|rat|, tol1) */
        double fu = traced(f, ctx, x);
        num += 1;
        if (fu <= fx) {
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
        xm = 0.5 * (a + b);
        tol1 = sqrt_eps * fabs(xf) + xatol / 3.0;
        tol2 = 2.0 * tol1;
        if (num >= maxfun) break;
    }
    *nfev = num;
    return xf;
}

typedef struct { double c2, x0, c1; double* xs; int maxn, n; } quad_ctx;
static double quad_obj(double x, void* p) {
    quad_ctx* q = (quad_ctx*)p;
    if (q->n < q->maxn) q->xs[q->n] = x;
    q->n++;
    double d = x - q->x0;
    return q->c2 * d * d + q->c1 * x;
}

int orc_brent_quadratic(double lo, double hi, double xatol, double c2, double x0, double c1,
                        double* xs, int maxn, double* xopt) {
    quad_ctx q = {c2, x0, c1, xs, maxn, 0};
    int nfev = 0;
    *xopt = brent_bounded(quad_obj, &q, lo, hi, xatol, 500, &nfev);
    return nfev;
}

/* ------------------------------------------------------------------------- */
/* per-agent driver                                                           */
/* ------------------------------------------------------------------------- */

typedef struct {
    const orc_agent* a;
    const orc_tariff* tariffs;
    int n_tariffs;
    const orc_cfg* cfg;
    const double* load;       /* cons (8760)                                  */
    const double* gpk;        /* gen_per_kw (8760)                            */
    const double* ts;         /* f32-rounded TS sell or NULL                  */
    double* gen;              /* scratch (8760)                               */
    int tariff;               /* sticky state (elec.py:852-855)               */
    int switched;
    int status;
    double x_last;
    /* last PV-only evaluation capture (ff:449-474) */
    double npv, payback, bill_w1, bill_wo1;
    double aev[ORC_MAXY + 1], bw[ORC_MAXY + 1], bwo[ORC_MAXY + 1];
    double cfpb[ORC_MAXY + 1], cfev[ORC_MAXY + 1];
} drv_ctx;

/* apply_rate_switch (elec.py:838-863): exactly one candidate row with
 * min_kw <= size < max_kw and size > 0 switches the agent's tariff in place. */
static double rate_switch(drv_ctx* c, const orc_switch* rows, int n, double size) {
    int hit = -1, cnt = 0;
    for (int i = 0; i < n; i++)
        if (rows[i].min_kw <= size && rows[i].max_kw > size) { cnt++; hit = i; }
    if (size > 0.0 && cnt == 1) {
        c->tariff = rows[hit].tariff;
        c->switched = 1;
        return rows[hit].one_time_charge;
    }
    return 0.0;
}

static void loan_inputs(const orc_agent* a, double total, orc_loan_in* li) {
    li->nyears = a->econ_life;
    li->market = a->is_res ? 0 : 1;
    li->loan_term = a->loan_term;
    li->depr_fed_type = a->is_res ? 0 : 2;
    li->depr_sta_type = a->is_res ? 0 : 2;
    li->pad = 0;
    li->debt_fraction_pct = 100.0 - (a->down_payment * 100.0);
    li->fed_tax_pct = (a->tax_rate * 100.0) * 0.7;
    li->sta_tax_pct = (a->tax_rate * 100.0) * 0.3;
    li->real_disc_pct = a->real_discount * 100.0;
    li->inflation_pct = a->inflation * 100.0;
    li->itc_fed_pct = a->itc_frac;        /* ff:285 passes the fraction as percent */
    li->total_cost = total;
}

/* diagnostics only: objective noise of +-k ulps (sensitivity of the Brent path) */
static int orc_obj_noise_ulps = 0;
static __thread unsigned long long orc_noise_state = 1;
void orc_set_obj_noise(int ulps, unsigned long long seed) { orc_obj_noise_ulps = ulps; orc_noise_state = seed; }

/* calc_system_performance(..., en_batt=False) (ff:96-288 PV-only branch). */
static double perf_no_batt(double kw, void* p) {
    drv_ctx* c = (drv_ctx*)p;
    const orc_agent* a = c->a;
    c->x_last = kw;
    for (int h = 0; h < ORC_NH; h++) c->gen[h] = (((c->gpk[h] * kw) * 1000.0) * 0.96) / 1000.0;
    double otc = 0.0;
    if (kw > 0.0) otc = rate_switch(c, a->sw_solar, a->n_sw_solar, kw);
    const orc_tariff* t = &c->tariffs[c->tariff];
    const double* ts = (t->mo == 2 && !a->is_ca) ? c->ts : NULL;
    int N = a->econ_life;
    if (orc_ur5(t, c->cfg, c->gen, c->load, ts, N, a->inflation * 100.0, a->escalator * 100.0,
                a->pv_deg * 100.0, c->bw, c->bwo, c->aev, NULL) != 0)
        c->status = -10;
    double total = ((a->capex * kw + 0.0) * a->ccm) + 0.0 + otc;
    orc_loan_in li;
    loan_inputs(a, total, &li);
    if (orc_cashloan(&li, c->cfg, c->aev, &c->npv, &c->payback, c->cfpb, c->cfev) != 0)
        c->status = -11;
    c->bill_w1 = c->bw[1];
    c->bill_wo1 = c->bwo[1];
    if (orc_obj_noise_ulps > 0) {        /* diagnostics only: +-k ulp of the objective */
        orc_noise_state = orc_noise_state * 6364136223846793005ull + 1442695040888963407ull;
        int k = (int)((orc_noise_state >> 33) % (2 * orc_obj_noise_ulps + 1)) - orc_obj_noise_ulps;
        double v = -c->npv;
        for (; k > 0; k--) v = nextafter(v, INFINITY);
        for (; k < 0; k++) v = nextafter(v, -INFINITY);
        return v;
    }
    return -c->npv;
}

/* forced (test infrastructure, orc_eval_at): {kw_star, x_last, search tariff,
 * switched} replace the bounded Brent search -- the PV-only outputs come from
 * one evaluation at x_last with that sticky tariff state, the PV+battery run
 * from kw_star, as ff:449-565 post-processes a finished search. */
static int size_agent_impl(const orc_agent* a, const orc_tariff* tariffs, int n_tariffs,
                           const orc_cfg* cfg, orc_result* r, const double* forced) {
    double* buf = (double*)malloc(sizeof(double) * ORC_NH * 8);
    if (!buf) return -1;
    double *hourly = buf, *load = buf + ORC_NH, *gpk = buf + 2 * ORC_NH, *gen = buf + 3 * ORC_NH;
    double *ts = buf + 4 * ORC_NH, *pv = buf + 5 * ORC_NH, *sysgen = buf + 6 * ORC_NH;
    double* g2l = buf + 7 * ORC_NH;
    int N = a->econ_life;
    memset(r->cash_flow, 0, sizeof(double) * (ORC_MAXY + 1) * 7);
    r->status = 0;
    if (N < 1 || N > ORC_MAXY || a->tariff0 < 0 || a->tariff0 >= n_tariffs) {
        free(buf);
        r->status = -2;
        return -2;
    }

    /* elec.py:571-577 scale_array_sum: hourly / hourly.sum() * load_kwh */
    for (int h = 0; h < ORC_NH; h++) hourly[h] = (double)a->shape[h];
    double S = orc_np_sum(hourly, ORC_NH);
    for (int h = 0; h < ORC_NH; h++) load[h] = (hourly[h] / S) * a->load_kwh;
    /* ff:350-351 gen_per_kw = cf / 1e6, naep = gen_per_kw.sum() */
    for (int h = 0; h < ORC_NH; h++) gpk[h] = (double)a->cf[h] / 1e6;
    double naep0 = orc_np_sum(gpk, ORC_NH);
    /* ff:182,246,372 wholesale * multiplier, then _list1d_8760's float32 cast */
    int has_ts = 0;
    if (a->wholesale) {
        has_ts = 1;
        for (int h = 0; h < ORC_NH; h++) {
            float v = (float)(a->wholesale[h] * a->price_mult);
            ts[h] = (double)v;
            if (!isfinite(ts[h])) has_ts = 0;
        }
    }

    drv_ctx c;
    memset(&c, 0, sizeof(c));
    c.a = a; c.tariffs = tariffs; c.n_tariffs = n_tariffs; c.cfg = cfg;
    c.load = load; c.gpk = gpk; c.ts = has_ts ? ts : NULL; c.gen = gen;
    c.tariff = a->tariff0;

    /* ff:440-447 bracket, xatol, bounded Brent */
    double max_load = a->load_kwh / naep0;
    double low = max_load * 0.8, high = max_load * 1.25;
    double span = high - low;
    double tl = (span > 1.0 ? span : 1.0) * 1e-3;
    double tol = 2.0;
    if (tl >= 3.0) tol = floor(tl);        /* max(2, int(...)), int() truncates */
    if (!isfinite(low) || !isfinite(high) || low > high) {
        free(buf);
        r->status = -3;
        return -3;
    }
    int nfev = 0;
    double kw_star;
    if (forced) {
        int ts = (int)forced[2];
        if (ts < 0 || ts >= n_tariffs) {
            free(buf);
            r->status = -4;
            return -4;
        }
        c.tariff = ts;
        c.switched = (int)forced[3];
        (void)perf_no_batt(forced[1], &c);
        kw_star = forced[0];
    } else {
        kw_star = brent_bounded(perf_no_batt, &c, low, high, tol, 500, &nfev);
    }

    /* ff:449-474: PV-only outputs come from the LAST evaluation (x_last),
     * system_kw from res.x (kw_star). */
    double x_last = c.x_last;
    for (int h = 0; h < ORC_NH; h++) gen[h] = (((gpk[h] * x_last) * 1000.0) * 0.96) / 1000.0;
    double annual = orc_np_sum(gen, ORC_NH);             /* np.nansum, ff:452 */
    r->system_kw = kw_star;
    r->x_last = x_last;
    r->nfev = nfev;
    r->annual_kwh = annual;
    double den = kw_star > 1e-9 ? kw_star : 1e-9;
    r->naep = annual / den;
    r->capacity_factor = r->naep / 8760.0;
    r->first_with = c.bill_w1;
    r->first_without = c.bill_wo1;
    r->price_per_kwh = c.bill_wo1 / a->load_kwh;
    r->npv = c.npv;
    r->payback_raw = c.payback;
    r->payback_period = orc_np_round1(isfinite(c.payback) ? c.payback : 30.1);
    for (int i = 0; i <= N; i++) {
        r->cash_flow[i] = c.cfpb[i];
        r->cf_energy_value_pv_only[i] = c.cfev[i];
        r->bill_w_pv_only[i] = c.bw[i];
        r->bill_wo_pv_only[i] = c.bwo[i];
    }
    if (r->baseline)
        for (int h = 0; h < ORC_NH; h++) r->baseline[h] = load[h];
    if (r->net_pvonly)
        for (int h = 0; h < ORC_NH; h++) {
            double d = load[h] - gen[h];
            r->net_pvonly[h] = d > 0.0 ? d : 0.0;
        }

    /* ff:479, ff:130-220: one PV+battery forward run at kw_star. */
    for (int h = 0; h < ORC_NH; h++) pv[h] = (((gpk[h] * kw_star) * 1000.0) * 0.96) / 1000.0;
    double desired_kwh = kw_star / 0.8, desired_kw = desired_kwh / 2.0;
    double bank = 0.0, power = 0.0;
    orc_batt_size(desired_kw, desired_kwh, a->is_res ? 240.0 : 500.0, cfg, &bank, &power);
    orc_batt_dispatch(load, pv, bank, power, cfg, sysgen, g2l);
    double otc = 0.0;
    if (bank > 0.0) otc = rate_switch(&c, a->sw_storage, a->n_sw_storage, bank);
    const orc_tariff* t = &tariffs[c.tariff];
    const double* tsp = (t->mo == 2 && !a->is_ca && has_ts) ? ts : NULL;
    double aev[ORC_MAXY + 1], bw[ORC_MAXY + 1], bwo[ORC_MAXY + 1];
    if (orc_ur5(t, cfg, sysgen, load, tsp, N, a->inflation * 100.0, a->escalator * 100.0,
                a->pv_deg * 100.0, bw, bwo, aev, NULL) != 0)
        c.status = -12;
    double system_costs = (kw_star > 0.0) ? a->capex_combined * kw_star : a->capex * kw_star;
    double batt_costs = a->batt_capex_kwh_combined * bank * 0.7;
    for (int i = 0; i <= N; i++) aev[i] = aev[i] + a->vor;    /* ff:275 (index 0 too) */
    orc_loan_in li;
    loan_inputs(a, ((system_costs + batt_costs) * a->ccm) + 0.0 + otc, &li);
    double npv_b = 0.0, pb_b = 0.0, cfpb_b[ORC_MAXY + 1], cfev_b[ORC_MAXY + 1];
    if (orc_cashloan(&li, cfg, aev, &npv_b, &pb_b, cfpb_b, cfev_b) != 0) c.status = -13;
    r->npv_pv_batt = npv_b;
    r->batt_kw = power;
    r->batt_kwh = bank;
    for (int i = 0; i <= N; i++) {
        r->cf_energy_value_pv_batt[i] = cfev_b[i];
        r->bill_w_pv_batt[i] = bw[i];
        r->bill_wo_pv_batt[i] = bwo[i];
    }
    if (r->net_with_batt)
        for (int h = 0; h < ORC_NH; h++) r->net_with_batt[h] = g2l[h];
    r->tariff_final = c.tariff;
    r->switched = c.switched;
    r->status = c.status;
    free(buf);
    return c.status;
}

int orc_size_agent(const orc_agent* a, const orc_tariff* tariffs, int n_tariffs, const orc_cfg* cfg,
                   orc_result* r) {
    return size_agent_impl(a, tariffs, n_tariffs, cfg, r, NULL);
}

/* The driver's outputs for a search that ended at (kw_star, x_last) with the
 * given sticky tariff state (test infrastructure: checks a device agent whose
 * Brent path left the oracle's at a knife edge). */
int orc_eval_at(const orc_agent* a, const orc_tariff* tariffs, int n_tariffs, const orc_cfg* cfg,
                double kw_star, double x_last, int tariff, int switched, orc_result* r) {
    const double forced[4] = {kw_star, x_last, (double)tariff, (double)switched};
    return size_agent_impl(a, tariffs, n_tariffs, cfg, r, forced);
}

int orc_size_batch(const orc_agent* agents, int64_t n, const orc_tariff* tariffs, int n_tariffs,
                   const orc_cfg* cfg, orc_result* results, int threads) {
    int bad = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : bad)
#endif
    for (int64_t i = 0; i < n; i++) {
        if (orc_size_agent(&agents[i], tariffs, n_tariffs, cfg, &results[i]) != 0) bad++;
    }
    (void)threads;
    return bad;
}
