/*
 * orc.h -- CPU ORACLE for the dGen sizing & economics hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under dgen_amd/ links, loads or calls this
 * library; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may use it, and only as the checker / the timed CPU baseline ("kind": "port").
 *
 * What it restates (plain C, fp64, sequential, compiled with -ffp-contract=off):
 *   - numpy's pairwise float64 summation (np.sum / np.nansum as used at
 *     financial_functions.py:351,452 and agent_mutation/elec.py:571-577);
 *   - scipy 1.15.3 optimize._minimize_scalar_bounded, op for op
 *     (driven at financial_functions.py:440-447);
 *   - the per-agent driver calc_system_size_and_performance
 *     (financial_functions.py:291-568) incl. the sticky rate switch
 *     (agent_mutation/elec.py:838-863) and last-evaluation output capture;
 *   - the PySAM/SSC engines it drives (nrel-pysam==7.1.0, dgen_os/python/dg3n.yml:24)
 *     -- Utilityrate5, Cashloan, Battery -- restated from SAM's published
 *     methodology.  SSC is NOT in /root/reference and PySAM is not installed:
 *     the SSC-side semantics are PARITY UNPINNED (see DESIGN.md "SSC subset").
 *
 * Pinning: tests/golden/ fixtures were produced by running the reference's own
 * Python driver (stub import, tests/golden/make_golden.py) with fake PySAM
 * modules whose execute() calls the primitives below.  So the Python-side
 * semantics (bracket/xatol, Brent path, rate-switch stickiness, last-eval
 * capture, naep mixing, payback rounding, tariff compile) are pinned to the
 * reference; the SSC arithmetic is pinned only to this restatement.
 */
#ifndef DGEN_ORACLE_ORC_H
#define DGEN_ORACLE_ORC_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_NH    8760
#define ORC_MAXP  12
#define ORC_MAXT  6
#define ORC_MAXY  50
#define ORC_DCP   8     /* demand-charge TOU periods (extension mode) */
#define ORC_DCT   4     /* demand-charge tiers                        */

/* Compiled tariff: what process_tariff() (financial_functions.py:575-648) leaves
 * in Utilityrate5.ElectricityRates for the energy-charge path.               */
typedef struct {
    int32_t P, T;            /* periods (1..P), tiers (1..T)                   */
    int32_t mo;              /* ur_metering_option: 0 NEM, 2 net billing       */
    int32_t unit;            /* usage unit code: 0 kWh/month, 2 kWh/day         */
    double  fixed;           /* ur_monthly_fixed_charge                        */
    double  cap[ORC_MAXT];   /* tier upper bound (harmonised, ff:919-960)      */
    double  buy[ORC_MAXP][ORC_MAXT];
    double  sell[ORC_MAXP][ORC_MAXT];
    uint8_t wkday[12][24];   /* 0-based period id                              */
    uint8_t wkend[12][24];
    /* demand charges (extension mode; the reference keeps them off, ff:35):
     * monthly flat and TOU peaks of hourly grid import, tiered per month /
     * period, the last tier unbounded.  dc_on = 0: no demand charge.        */
    int32_t dc_on;
    int32_t dc_tou_nt[ORC_DCP];      /* tiers per TOU period (0 = no charge)  */
    int32_t dc_flat_nt[12];          /* tiers per month (0 = no charge)       */
    double  dc_tou_cap[ORC_DCP][ORC_DCT], dc_tou_price[ORC_DCP][ORC_DCT];
    double  dc_flat_cap[12][ORC_DCT], dc_flat_price[12][ORC_DCT];
    uint8_t dc_wkday[12][24];        /* 0-based demand period                 */
    uint8_t dc_wkend[12][24];
} orc_tariff;

/* PySAM config defaults the reference never sets (parity unpinned). */
typedef struct {
    double nm_yearend_sell_rate;   /* $/kWh, Utilityrate5 ur_nm_yearend_sell_rate */
    double loan_rate_pct;          /* Cashloan loan_rate (%)                      */
    double insurance_rate_pct;     /* Cashloan insurance_rate (%)                 */
    double itc_fed_max;            /* itc_fed_percent_maxvalue ($)                */
    int32_t depr_sl_years;         /* straight-line depreciation years (type 2)   */
    double batt_v_nom;             /* cell nominal voltage (V)                    */
    double batt_q_full;            /* cell capacity (Ah)                          */
    double batt_min_soc;           /* fraction                                    */
    double batt_max_soc;           /* fraction                                    */
    double batt_init_soc;          /* fraction (ff:151: 30 %)                     */
    double batt_eta_in;            /* AC->stored efficiency                       */
    double batt_eta_out;           /* stored->AC efficiency                       */
    int32_t batt_update_hours;     /* 24: daily plan, 1: re-planned every hour    */
    int32_t batt_loss_model;       /* 0: constant efficiencies, 1: Li-ion losses  */
    double batt_r_cell;            /* cell internal resistance (ohm)              */
    double batt_conv_eff;          /* converter efficiency each way               */
    double batt_v_cell_empty;      /* open-circuit voltage at SOC 0 (V)           */
    double batt_v_cell_full;       /* open-circuit voltage at SOC 1 (V)           */
    int32_t batt_month_floor;      /* 1: targets floored at the month's earlier   */
} orc_cfg;

/* One row of the rate-switch table, already filtered to (tech, eia_id, res_com). */
typedef struct {
    double  min_kw, max_kw, one_time_charge;
    int32_t tariff;              /* index into the tariff table                 */
    int32_t pad;
} orc_switch;

typedef struct {
    const float*   shape;        /* 8760 raw load profile values (DB array)    */
    const int32_t* cf;           /* 8760 solar CF x 1e6 (elec.py:545)          */
    const double*  wholesale;    /* 8760 $/kWh or NULL                          */
    double load_kwh, price_mult;
    int32_t is_res, is_ca, econ_life, loan_term;
    double inflation, pv_deg, escalator, down_payment, tax_rate, real_discount, itc_frac;
    double capex, capex_combined, batt_capex_kwh_combined, ccm, vor;
    int32_t tariff0;
    int32_t n_sw_solar, n_sw_storage;
    const orc_switch* sw_solar;
    const orc_switch* sw_storage;
} orc_agent;

typedef struct {
    double system_kw, x_last, annual_kwh, naep, capacity_factor, price_per_kwh;
    double npv, payback_raw, payback_period, first_with, first_without;
    double batt_kw, batt_kwh, npv_pv_batt;
    int32_t nfev, tariff_final, switched, status;
    double cash_flow[ORC_MAXY + 1];
    double cf_energy_value_pv_only[ORC_MAXY + 1];
    double bill_w_pv_only[ORC_MAXY + 1];
    double bill_wo_pv_only[ORC_MAXY + 1];
    double cf_energy_value_pv_batt[ORC_MAXY + 1];
    double bill_w_pv_batt[ORC_MAXY + 1];
    double bill_wo_pv_batt[ORC_MAXY + 1];
    double* baseline;            /* 8760 outputs (caller-owned, may be NULL)   */
    double* net_pvonly;
    double* net_with_batt;
} orc_result;

/* ---- primitives --------------------------------------------------------- */
double orc_pairwise_sum(const double* a, int64_t n);      /* numpy pairwise      */
double orc_np_sum(const double* a, int64_t n);            /* np.sum(a) (1-D)     */
double orc_np_round1(double x);                           /* np.round(x, 1)      */

/* Build a compiled tariff from PySAM-style fields: rows [period,tier,cap,unit,buy,sell]
 * (1-based), schedules 12x24 1-based.  Returns 0 or a negative error.            */
int orc_tariff_from_mat(orc_tariff* t, const double* mat, int nrows, int mo,
                        double fixed, const int32_t* wk, const int32_t* we);

/* Utilityrate5 subset.  gen/load: 8760 kWh.  ts_sell: 8760 or NULL.
 * Outputs of length nyears+1 (index 0 = 0).  e_fromgrid: 8760 or NULL.      */
int orc_ur5(const orc_tariff* t, const orc_cfg* cfg, const double* gen, const double* load,
            const double* ts_sell, int nyears, double inflation_pct, double escal_pct,
            double degr_pct, double* bill_w, double* bill_wo, double* aev,
            double* e_fromgrid);

/* Cashloan subset.  aev: nyears+1 (index 0 ignored).  Percent inputs as PySAM. */
typedef struct {
    int32_t nyears, market, loan_term, depr_fed_type, depr_sta_type, pad;
    double debt_fraction_pct, fed_tax_pct, sta_tax_pct, real_disc_pct, inflation_pct;
    double itc_fed_pct, total_cost;
} orc_loan_in;
int orc_cashloan(const orc_loan_in* in, const orc_cfg* cfg, const double* aev,
                 double* npv, double* payback, double* cf_payback, double* cf_energy_value);

/* Battery subset (BatteryTools.battery_model_sizing + BTM peak-shaving dispatch). */
void orc_batt_size(double desired_kw, double desired_kwh, double desired_v,
                   const orc_cfg* cfg, double* bank_kwh, double* power_kw);
void orc_batt_dispatch(const double* load, const double* pv, double bank_kwh,
                       double power_kw, const orc_cfg* cfg, double* sysgen,
                       double* grid_to_load);

/* scipy bounded Brent on a closed-form objective (tests the search in isolation):
 * f(x) = c2*(x-x0)^2 + c1*x.  Writes the evaluated x sequence.               */
int orc_brent_quadratic(double lo, double hi, double xatol, double c2, double x0,
                        double c1, double* xs, int maxn, double* xopt);

/* Full per-agent driver (financial_functions.py:291-568). */
int orc_size_agent(const orc_agent* a, const orc_tariff* tariffs, int n_tariffs,
                   const orc_cfg* cfg, orc_result* r);

/* Parallel batch driver over host threads (OpenMP); used as the CPU baseline. */
int orc_size_batch(const orc_agent* agents, int64_t n, const orc_tariff* tariffs,
                   int n_tariffs, const orc_cfg* cfg, orc_result* results, int threads);

#ifdef __cplusplus
}
#endif
#endif
