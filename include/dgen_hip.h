/*
 * dgen_hip.h -- C-ABI of libdgen_hip.so, the MI355X (gfx950) sizing & economics
 * engine that replaces dGen's per-agent hot path.
 *
 * Reference interface replaced (tsgsteele/dgen @ 2025-09-19, /root/reference):
 *   financial_functions.calc_system_size_and_performance   dgen_os/python/financial_functions.py:291-568
 *   financial_functions.calc_system_performance (objective) dgen_os/python/financial_functions.py:96-288
 *   financial_functions.size_chunk (worker loop)            dgen_os/python/financial_functions.py:1136-1218
 *   agent_mutation.elec.get_and_apply_agent_load_profiles   dgen_os/python/agent_mutation/elec.py:508-532
 *   agent_mutation.elec.get_and_apply_normalized_hourly_resource_solar  elec.py:535-558
 *   agent_mutation.elec.apply_rate_switch                    dgen_os/python/agent_mutation/elec.py:838-863
 *   PySAM Utilityrate5 / Cashloan / Battery .execute()       financial_functions.py:164,270,287
 *   scipy.optimize.minimize_scalar(method='bounded')         financial_functions.py:445-447
 *
 * Conventions
 *   - Plain C types only; every pointer in dgen_tables / dgen_agents /
 *     dgen_outputs is a DEVICE pointer owned by the caller (the Python host keeps
 *     them in torch-ROCm tensors) and borrowed for the duration of a call.
 *   - Every entry point returns 0 on success or a negative DGEN_E_* code; the
 *     message is available from dgen_last_error().  No exception crosses the ABI.
 *   - Per-agent problems are reported in dgen_outputs.status (DGEN_ST_* bits);
 *     the host raises like the reference's abort-the-year behaviour
 *     (dgen_model.py:382).
 *   - Calls are stream-ordered on the given hipStream_t (NULL = default stream)
 *     and asynchronous unless stated otherwise.
 *   - Yearly array outputs are agent-major: value (agent, y) at
 *     [agent * (DGEN_MAXY + 1) + y]; hourly outputs are time-major in
 *     hour-quad tiles: (hour, agent) at [((hour / 4) * n + agent) * 4 + hour % 4]
 *     (a [2190][n][4] array: each agent's 4 consecutive hours are 16 B, so a
 *     wave writes 1 KB contiguous per plane every 4 hours).
 */
#ifndef DGEN_HIP_H
#define DGEN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DGEN_ABI_VERSION 14
#define DGEN_DEFAULT_CHUNKS 1  /* dgen_size_agents pipeline depth (dgen_set_pipeline) */
#define DGEN_DEFAULT_HOURLY_MONTHS 1  /* months per k_hourly_batt launch (dgen_set_hourly_segment) */
#define DGEN_DEFAULT_HOURLY_SPLIT 2   /* parts of a chunk's hourly scan, each on its own stream */
#define DGEN_NH    8760   /* hours per year                                    */
#define DGEN_NSLOT 576    /* 12 months x {weekday, weekend} x 24 hours         */
#define DGEN_MAXP  12     /* TOU periods                                        */
#define DGEN_MAXT  6      /* tiers                                              */
#define DGEN_MAXY  50     /* analysis years                                     */
#define DGEN_DCP   8      /* demand-charge TOU periods (extension mode)         */
#define DGEN_DCR_CAP 1024 /* kept hours per battery-case demand record          */
#define DGEN_DCT   4      /* demand-charge tiers (extension mode)               */

/* error codes */
#define DGEN_OK            0
#define DGEN_E_ARG        -1
#define DGEN_E_HIP        -2
#define DGEN_E_UNSUPPORTED -3

/* per-agent status bits */
#define DGEN_ST_BOUNDS       0x01  /* non-finite Brent bracket (scipy raises)       */
#define DGEN_ST_TARIFF       0x02  /* tariff index out of range / malformed          */
#define DGEN_ST_EMPTY_EC     0x04  /* tariff has no energy-charge matrix              */
#define DGEN_ST_UNIT         0x08  /* unsupported usage unit code (1, 3)              */
#define DGEN_ST_YEARS        0x10  /* analysis period outside 1..DGEN_MAXY            */
#define DGEN_ST_SCRATCH      0x20  /* mo=2 battery run without a scratch slot         */
#define DGEN_ST_ZERO_LOAD    0x40  /* load_kwh == 0: reference divides by zero (ff:549)*/
#define DGEN_ST_DEMAND       0x80  /* demand-charge mat outside SSC's / the record's   */
                                   /* limits (month, period, tier numbering)          */

/* Engine configuration: the PySAM config defaults the reference never sets
 * (CustomGenerationBattery{Residential,Commercial}, ff:59-80) plus the
 * reference's module switches (ff:35,38).                                     */
typedef struct {
    int32_t skip_demand_charges;   /* 1 = the reference (ff:35 SKIP_DEMAND_CHARGES  */
                                   /* = True): tariffs' demand records are ignored; */
                                   /* 0 = extension mode: they are billed           */
    int32_t force_net_billing;     /* ff:38; applied by the host tariff compiler    */
    double  nm_yearend_sell_rate;  /* $/kWh, Utilityrate5 ur_nm_yearend_sell_rate  */
    double  loan_rate_pct;         /* Cashloan loan_rate (%)                        */
    double  insurance_rate_pct;    /* Cashloan insurance_rate (%)                   */
    double  itc_fed_max;           /* Cashloan itc_fed_percent_maxvalue ($)         */
    int32_t depr_sl_years;         /* straight-line depreciation years (type 2)     */
    int32_t pad0;
    double  batt_v_nom;            /* Li-ion cell nominal voltage (V)               */
    double  batt_q_full;           /* cell capacity (Ah)                            */
    double  batt_min_soc;          /* fraction                                      */
    double  batt_max_soc;          /* fraction                                      */
    double  batt_init_soc;         /* fraction (ff:151: 30 %)                       */
    double  batt_eta_in;           /* AC -> stored                                  */
    double  batt_eta_out;          /* stored -> AC                                  */
    int32_t batt_update_hours;     /* peak-shaving re-plan interval: 24 = one 24-h  */
                                   /* plan per calendar day (SSC's BTM peak-shaving */
                                   /* update), 1 = a 24-h look-ahead plan every     */
                                   /* hour (bdh:86-87 read literally); DESIGN.md 3  */
    int32_t batt_loss_model;       /* 0: constant efficiencies batt_eta_in / _out   */
                                   /* (default); 1: Li-ion loss model (ABI 9):      */
                                   /* converters batt_conv_eff each way + cell I^2 R */
                                   /* with an open-circuit voltage linear in SOC     */
                                   /* (parameters are guesses)  */
    double  batt_r_cell;           /* cell internal resistance (ohm)                */
    double  batt_conv_eff;         /* AC-DC and DC-AC converter efficiency          */
    double  batt_v_cell_empty;     /* cell open-circuit voltage at SOC 0 (V)        */
    double  batt_v_cell_full;      /* cell open-circuit voltage at SOC 1 (V)        */
    int32_t batt_month_floor;      /* 1: a plan's target never falls below the     */
                                   /* month's earlier targets (SSC's monthly peak-  */
                                   /* shaving target, as we read it; ABI 9); 0: off */
    int32_t pad1;
} dgen_cfg;

/* Compiled tariff = the Utilityrate5.ElectricityRates energy fields that
 * process_tariff (ff:575-648) writes, after normalize_tariff (ff:962-1007).
 * Built on the host, bit-exact to the reference compile (tests/golden).      */
typedef struct {
    int32_t P, T;                  /* periods, tiers                               */
    int32_t mo;                    /* ur_metering_option (0 or 2)                  */
    int32_t unit;                  /* usage unit code: 0 kWh/mo, 1 kWh/kW, 2 kWh    */
                                   /* daily, 3 kWh/kW daily (ff:778-779, one code   */
                                   /* per tariff, ff:939-956); 1 and 3 scale the tier*/
                                   /* caps by the month's peak import (kW), which the*/
                                   /* kernels take from the record `dc` points to    */
                                   /* (its flat peak; a zero-charge one-period record*/
                                   /* when the tariff has no demand charges)         */
    double  fixed;                 /* ur_monthly_fixed_charge ($/month)            */
    double  cap[DGEN_MAXT];        /* tier upper bounds (single cap per tier)      */
    double  buy[DGEN_MAXP][DGEN_MAXT];
    double  sell[DGEN_MAXP][DGEN_MAXT];
    uint8_t wkday[12][24];         /* 0-based period per (month, hour)             */
    uint8_t wkend[12][24];
    int32_t flags;                 /* DGEN_ST_EMPTY_EC / _UNIT / _DEMAND if so      */
    int32_t dc;                    /* 1 + index into dgen_tables.demand; 0 = none  */
                                   /* (charges billed in extension mode only; the   */
                                   /* peaks of units 1 / 3 are read in both modes)  */
} dgen_tariff;

/* Demand charges of one tariff (extension mode): the ur_dc_flat_mat /
 * ur_dc_tou_mat / ur_dc_sched_* fields process_tariff writes when
 * SKIP_DEMAND_CHARGES is off (ff:604-615), packed on the host.  Per month the
 * flat peak is the max hourly grid import (kW = kWh per hour; 0 without
 * import) and each TOU peak the max over that period's hours; each peak is
 * billed through its tier table (tier upper bounds in kW, the last tier
 * unbounded above), escalated with the energy charges.  SSC semantics
 * restated from SAM's published methodology: parity unpinned.                */
typedef struct {
    int32_t tou_nt[DGEN_DCP];      /* tiers per TOU period (0 = no charge)          */
    int32_t flat_nt[12];           /* tiers per month (0 = no charge)               */
    int32_t flags;                 /* DGEN_ST_DEMAND when the mats were out of range*/
    int32_t pad;
    double  tou_cap[DGEN_DCP][DGEN_DCT];
    double  tou_price[DGEN_DCP][DGEN_DCT];   /* $/kW                              */
    double  flat_cap[12][DGEN_DCT];
    double  flat_price[12][DGEN_DCT];
    uint8_t wkday[12][24];         /* 0-based demand period per (month, hour)       */
    uint8_t wkend[12][24];
} dgen_demand;

/* One row of diffusion_shared.rate_switch_lkup_2020 (elec.py:828-836), already
 * filtered to one agent's (tech, eia_id, res_com) on the host.                */
typedef struct {
    double  min_kw, max_kw, one_time_charge;
    int32_t tariff;                /* index into dgen_tables.tariffs                */
    int32_t pad;
} dgen_switch;

/* Resident tables (device pointers). */
typedef struct {
    const float*   shapes;         /* [n_shapes][8760] kwh_load_profile rows        */
    const double*  shape_sum;      /* [n_shapes]   np.sum of the row (numpy order)  */
    const double*  shape_slots;    /* [n_shapes][576] slot sums of the row          */
    const int32_t* cfs;            /* [n_cfs][8760] solar cf x 1e6                  */
    const double*  cf_naep;        /* [n_cfs]      np.sum(cf / 1e6)                 */
    const double*  cf_slots;       /* [n_cfs][576] slot sums of cf / 1e6            */
    const double*  wholesale;      /* [n_wholesale][8760] $/kWh (may be NULL)       */
    const dgen_tariff* tariffs;
    const dgen_switch* switches;
    int64_t n_shapes, n_cfs, n_wholesale, n_switches;
    int32_t n_tariffs;
    int32_t max_periods;           /* max P over tariffs (sizes LDS; 0 = DGEN_MAXP) */
    const dgen_demand* demand;     /* [n_demand] (may be NULL when n_demand == 0)   */
    int32_t n_demand;
    int32_t peak_units;            /* 1: some tariff bills its tiers in kWh/kW (unit */
                                   /* codes 1, 3): the year-lane kernels keep month  */
                                   /* peaks per lane (see dgen_tariff.unit)          */
    int32_t max_dc_periods;        /* 1 + the largest period in the demand records' */
                                   /* schedules (sizes LDS; 0 = DGEN_DCP)           */
    int32_t no_net;                /* 1: no agent of the call can bill net hourly   */
                                   /* (metering options 2, 3: initial tariff and    */
                                   /* every rate-switch candidate): the demand-     */
                                   /* charge kernels run their instantiations       */
                                   /* without the net-billing paths (fewer          */
                                   /* registers); 0: some may (ABI 12)              */
    int32_t pad_t;
    /* Bounds of the certified Brent paths (ABI 14, dgen_set_exact; each may be   */
    /* NULL: the agents that would need it take the exact re-run instead):        */
    const double*  bt_tariff;      /* [n_tariffs][3]: max |buy|, |sell| ($/kWh);   */
                                   /* demand prices, max over months of the flat   */
                                   /* tier price + the TOU periods' ($/kW); the     */
                                   /* kWh/kW tier caps' peak sensitivity ($/kW)     */
    const double*  bt_shape_max;   /* [n_shapes] max |shape| of the row             */
    const double*  bt_cf_max;      /* [n_cfs]    max |cf| of the row (x 1e6)        */
    const double*  bt_ts_max;      /* [n_wholesale] max |wholesale| of the row      */
} dgen_tables;

/* Agent batch, structure of arrays (device pointers, length n).  Column
 * meaning follows the agent row read by the reference. */
typedef struct {
    const int32_t* load_row;       /* row of shapes  <- (bldg_id, sector, state)     */
    const int32_t* cf_row;         /* row of cfs     <- (gid, tilt, azimuth)         */
    const int32_t* wholesale_row;  /* row of wholesale or -1 (no finite 8760 series) */
    const int32_t* tariff0;        /* initial tariff (tariff_dict)                   */
    const int32_t* sw_solar_off;   /* rate-switch candidates, tech = 'solar'          */
    const int32_t* sw_solar_cnt;
    const int32_t* sw_storage_off; /* rate-switch candidates, tech = 'storage'        */
    const int32_t* sw_storage_cnt;
    const int32_t* scratch_slot;   /* hourly scratch slot for mo=2 or demand-charge   */
                                   /* battery runs, or -1                             */
    const uint8_t* flags;          /* bit0 sector_abbr == 'res', bit1 state == 'CA'  */
    const int32_t* econ_life;      /* economic_lifetime_yrs                           */
    const int32_t* loan_term;      /* loan_term_yrs                                   */
    const double* load_kwh;        /* load_kwh_per_customer_in_bin                    */
    const double* price_mult;      /* elec_price_multiplier                           */
    const double* inflation;       /* inflation_rate (fraction)                       */
    const double* pv_deg;          /* pv_degradation_factor                           */
    const double* escalator;       /* elec_price_escalator                            */
    const double* down_payment;    /* down_payment_fraction                           */
    const double* tax_rate;        /* tax_rate                                        */
    const double* real_discount;   /* real_discount_rate                              */
    const double* itc_frac;        /* itc_fraction_of_capex                           */
    const double* capex;           /* system_capex_per_kw                             */
    const double* capex_combined;  /* system_capex_per_kw_combined                    */
    const double* batt_capex_kwh;  /* batt_capex_per_kwh_combined                     */
    const double* ccm;             /* cap_cost_multiplier                             */
    const double* vor;             /* value_of_resiliency_usd                         */
    int32_t max_years;             /* max econ_life over the batch: <= 32 runs two    */
                                   /* agents per wave in the year-lane kernels; 0 or  */
                                   /* > 32 runs one (agents above 32 lanes then fail  */
                                   /* with DGEN_ST_YEARS instead of being truncated)  */
} dgen_agents;

/* Outputs (device pointers).  Hourly planes may be NULL (on-device reduction
 * mode: nothing hourly is materialised).                                     */
typedef struct {
    double* system_kw;             /* res.x                                           */
    double* x_last;                /* last evaluated x (source of PV-only outputs)    */
    double* annual_kwh;            /* annual_energy_production_kwh                    */
    double* naep;                  /* annual / max(system_kw, 1e-9)                   */
    double* capacity_factor;
    double* price_per_kwh;
    double* npv;
    double* payback_raw;           /* Cashloan payback                                */
    double* payback_period;        /* np.round(payback if finite else 30.1, 1)        */
    double* first_with;            /* utility_bill_w_sys_year1                        */
    double* first_without;         /* utility_bill_wo_sys_year1                       */
    double* batt_kw;               /* batt_power_discharge_max_kwdc                   */
    double* batt_kwh;              /* batt_bank_installed_capacity                    */
    double* npv_pv_batt;           /* NPV of the PV+battery run (not in the ref row)  */
    int32_t* nfev;                 /* PV-only objective evaluations                   */
    int32_t* tariff_final;         /* sticky tariff state after both runs             */
    int32_t* switched;             /* any rate switch happened (nem limit -> 1e6)     */
    int32_t* status;               /* DGEN_ST_* bits                                  */
    double* cash_flow;             /* [n][MAXY+1] cf_payback_with_expenses            */
    double* cfev_pv;               /* [n][MAXY+1] cf_energy_value_pv_only             */
    double* bill_w_pv;             /* [n][MAXY+1] utility_bill_w_sys_pv_only          */
    double* bill_wo_pv;            /* [n][MAXY+1] utility_bill_wo_sys_pv_only         */
    double* cfev_batt;             /* [n][MAXY+1] cf_energy_value_pv_batt             */
    double* bill_w_batt;           /* [n][MAXY+1] utility_bill_w_sys_pv_batt          */
    double* bill_wo_batt;          /* [n][MAXY+1] utility_bill_wo_sys_pv_batt         */
    void*   baseline;              /* [2190][n][4] baseline_net_hourly (may be NULL)  */
    void*   net_pvonly;            /* [2190][n][4] adopter_net_hourly_pvonly          */
    void*   net_with_batt;         /* [2190][n][4] adopter_net_hourly_with_batt       */
    int32_t hourly_f64;            /* plane element type: 0 float (default), 1 double */
                                   /* (the reference's fp64 lists, bit-for-bit the    */
                                   /* values the kernels compute; 2 x the bytes)      */
    int32_t pad_;
} dgen_outputs;

typedef struct dgen_ctx dgen_ctx;

/* Version / build info. */
int32_t dgen_abi_version(void);

/* Copy the last error message of this thread into buf (NUL-terminated). */
int32_t dgen_last_error(char* buf, size_t n);

/* Open an engine on HIP device `device` with configuration `cfg`. */
int32_t dgen_open(int32_t device, const dgen_cfg* cfg, dgen_ctx** out);
int32_t dgen_close(dgen_ctx* ctx);

/* Profile-table preparation (replaces the per-agent SQL fetch + scaling of
 * elec.py:508-558, done once per table load instead of once per agent):
 * row sums in numpy's exact pairwise order and 576 slot sums per row.        */
int32_t dgen_prep_shapes(dgen_ctx* ctx, const float* shapes, int64_t n_rows, double* row_sum,
                         double* row_slots, void* stream);
int32_t dgen_prep_cfs(dgen_ctx* ctx, const int32_t* cfs, int64_t n_rows, double* row_naep,
                      double* row_slots, void* stream);

/* Workspace bytes for a batch of n agents with n_scratch scratch slots (agents
 * whose tariffs can bill net or carry demand charges):
 *   8 x (4 x 144 n + n + 8760 n_scratch)   bins, carries, battery output plane
 *   + DGEN_NB_BYTES x n_scratch             net-billing split records (k_size,
 *                                           k_batt_finance): per (month, period)
 *                                           4 f64 sums, 12 counts, 12 x 192
 *                                           mixed-hour entries of 24 B       */
#define DGEN_NB_BYTES 59968
#define DGEN_NB_CAPM 192     /* mixed hours per month a net-billing split record holds */
size_t dgen_workspace_bytes(int64_t n, int64_t n_scratch);

/* Size a batch: Brent over PV kW with 25-year bills + cash flow per
 * evaluation, then one PV+battery forward run at kW*, all on device.         */
int32_t dgen_size_agents(dgen_ctx* ctx, const dgen_tables* tables, const dgen_agents* agents,
                         const dgen_outputs* out, int64_t n, void* workspace, size_t ws_bytes,
                         int64_t n_scratch, void* stream);

/* Test entry: the device Brent on f(x) = c2 (x - x0)^2 + c1 x per lane,
 * recording up to maxn evaluated x per lane (xs: [lane][maxn]).              */
int32_t dgen_brent_selftest(dgen_ctx* ctx, const double* lo, const double* hi,
                            const double* xatol, const double* c2, const double* x0,
                            const double* c1, int64_t n, double* xs, int32_t maxn,
                            double* xopt, int32_t* nfev, void* stream);

/* Deterministic weighted segmented sums over contiguous agent ranges, for the
 * per-(state, sector) totals and per-state 8760-h net sums that feed diffusion
 * (replaces size_chunk's running net_sum, ff:1173-1188, and the per-state
 * hourly export, attachment_rate_functions.py:151-206):
 *   out[s * k + j] = sum_{i in [seg_off[s], seg_off[s+1])}
 *                      w1[i] * v1[j * n + i] + w2[i] * v2[j * n + i]
 * v1/v2 are k planes of n agents (plane-major, float32 or float64 by
 * `values_f32`); v2/w2 may be NULL, w1 NULL means weight 1.  Fixed summation
 * order (256-thread strided partials + LDS tree) => run-to-run identical.     */
int32_t dgen_segment_sums(dgen_ctx* ctx, const void* v1, const double* w1, const void* v2,
                          const double* w2, int32_t values_f32, int32_t k, int64_t n,
                          const int64_t* seg_off, int64_t n_seg, double* out, void* stream);

/* Sequential sum of row segments (ABI 9): out[s * k + j] = the rows
 * r in [seg_off[s], seg_off[s+1]) of in[r * k + j] added in row order
 * (((r0 + r1) + r2) + ...).  The model-year loop forms each state's totals and
 * 8760-h rows as the sum of fixed-size member chunks' partials in chunk order
 * (dgen_amd/partition.py), so a state split across ranks sums to the same bits
 * as on one rank.  n_seg <= 65535.                                           */
int32_t dgen_rows_seq_sum(dgen_ctx* ctx, const double* in, int64_t k, const int64_t* seg_off,
                          int64_t n_seg, double* out, void* stream);

/* ------------------------------------------------------------------------
 * Diffusion step: the per-agent arithmetic of
 *   financial_functions.calc_max_market_share      ff:1264-1310 (payback -> max market share)
 *   diffusion_functions_elec.calc_diffusion_solar   diffusion_functions_elec.py:24-156
 *     (calc_equiv_time :343-372, calc_diffusion_market_share :251-292,
 *      bass_diffusion :323-338).
 * The pandas merges (bass p/q/teq_yr1 by state x sector, table keys) stay on
 * the host; every per-agent number is computed here.
 * ---------------------------------------------------------------------- */

/* max_market_curves_to_model (metric 'payback_period', business model
 * 'host_owned') as a dense table: value(row, factor) at
 * mms[row * n_factors + (factor - factor_min)], factor = round(100 * payback)
 * on the 0.1-year grid; NaN = no curve point (left-merge miss).              */
typedef struct {
    const double* mms;
    int32_t n_rows, n_factors, factor_min, pad;
    double min_pb, max_pb;          /* clip range (min / max over the curve)    */
} dgen_mms_table;

/* payback_period_bounded, payback_period_as_factor, max_market_share.
 * mms_row: curve row of the agent's sector (-1: no curve -> NaN).            */
int32_t dgen_max_market_share(dgen_ctx* ctx, const dgen_mms_table* table, const double* payback,
                              const int32_t* mms_row, int64_t n, double* payback_bounded,
                              int64_t* factor, double* max_market_share, void* stream);

typedef struct {
    const double* max_market_share;
    const double* market_share_last_year;
    const double* bass_p;
    const double* bass_q;
    const double* teq_yr1;
    const double* developable_agent_weight;
    const double* system_kw;
    const double* system_capex_per_kw;
    const double* adopters_cum_last_year;
    const double* market_value_last_year;
    const double* system_kw_cum_last_year;
} dgen_diffusion_in;

typedef struct {
    double *mms_fix_zeros, *ratio, *bass_params_teq, *teq2, *f, *new_adopt_fraction;
    double *bass_market_share, *diffusion_market_share, *market_share, *new_market_share;
    double *new_adopters, *new_market_value, *new_system_kw, *number_of_adopters;
    double *market_value, *system_kw_cum;
} dgen_diffusion_out;

/* One Bass diffusion step for every agent (is_first_year selects teq_yr1). */
int32_t dgen_diffusion(dgen_ctx* ctx, const dgen_diffusion_in* in, const dgen_diffusion_out* out,
                       int64_t n, int32_t is_first_year, void* stream);

/* ------------------------------------------------------------------------
 * Battery attachment and the per-state hourly export:
 *   attachment_rate_functions._allocate_battery_adopters_integer  :58-138
 *   attachment_rate_functions.export_state_hourly_with_storage_mix :141-206
 * ---------------------------------------------------------------------- */
typedef struct {
    const double* new_adopters;           /* diffusion's new_adopters (float)     */
    const int64_t* aid_rank;              /* rank of str(agent_id), unique        */
    const double* batt_kw;
    const double* batt_kwh;
    const double* batt_kw_cum_last_year;
    const double* batt_kwh_cum_last_year;
} dgen_attach_in;

typedef struct {
    int64_t* added;                       /* batt_adopters_added_this_year        */
    double *new_batt_kw, *new_batt_kwh, *batt_kw_cum, *batt_kwh_cum;
} dgen_attach_out;

/* Largest-remainder allocation per group: agents of group g are
 * [seg_off[g], seg_off[g+1]) in the reference's row order (its n.sum() is
 * numpy-pairwise in that order); rate[g] = the group's storage_attachment_rate.
 * Tie-break among equal fractional parts: ascending str(agent_id) (aid_rank).
 * Replaces the per-group pandas sort (:105-129).  Integer results bit-exact. */
int32_t dgen_batt_attach(dgen_ctx* ctx, const dgen_attach_in* in, const dgen_attach_out* out,
                         const int64_t* seg_off, const double* rate, int64_t n_seg, void* stream);

/* Per-agent multipliers of the state export (:181-190): w_pvo = pvo_cum,
 * w_batt = batt_cum (integers as doubles), w_non = max(n_cust - n_adopt, 0). */
int32_t dgen_export_weights(dgen_ctx* ctx, const double* customers_in_bin,
                            const double* number_of_adopters, const double* batt_kw_cum_last_year,
                            const double* batt_kw, const int64_t* added, int64_t n, double* w_pvo,
                            double* w_batt, double* w_non, void* stream);

/* Per-state hourly net sums in MW (:179-198) from the three hourly planes
 * (planes_f32 = 1: float32 in dgen_size_agents' hour-quad tiles
 * [n_hours / 4][n][4], its hourly outputs in place, n_hours % 4 == 0;
 * 2: the same tiles in float64 (dgen_outputs.hourly_f64); 0: float64
 * [n_hours][n]; 3: dgen_export_plane's combined float64 plane in tiles, in
 * `baseline`, pvonly / with_batt / weights unused) and the per-column weights:
 * out[s * n_hours + h].  Members of state s are the plane columns
 * idx[seg_off[s] .. seg_off[s+1]) (idx NULL: columns seg_off[s] ..
 * seg_off[s+1]).  Fixed summation order (deterministic); the reference's
 * sequential iterrows sum is matched to fp64 rounding, not bit for bit.    */
int32_t dgen_state_hourly(dgen_ctx* ctx, const void* baseline, const void* pvonly,
                          const void* with_batt, int32_t planes_f32, const double* w_pvo,
                          const double* w_batt, const double* w_non, const int64_t* idx, int64_t n,
                          int32_t n_hours, const int64_t* seg_off, int64_t n_seg, double* out,
                          void* stream);

/* ------------------------------------------------------------------------
 * Per-year agent attributes: the elec.apply_* merges that
 * dgen_model.py:252-292 runs on the agent frame every model year, as device
 * gathers over per-year tables compiled on the host (dgen_amd/market.py,
 * the reference's own expressions per table row):
 *   apply_load_growth                         elec.py:398-411
 *   apply_elec_price_multiplier_and_escalator elec.py:29-82
 *   apply_pv_tech_performance / apply_pv_prices / apply_pv_plus_batt_prices
 *   apply_financial_params (financing + ITC)  elec.py:135-394
 *   apply_value_of_resiliency                 elec.py:284-314
 *   apply_wholesale_elec_prices               elec.py:608-616
 *   calculate_developable_customers_and_load  elec.py:414-423
 * A left merge that finds no row gives NaN (reals) or -1 (ints); -1 keys do
 * the same.  by_sector rows carry DGEN_YS_COLS columns in this order:       */
enum {
    DGEN_YS_CAPEX = 0,          /* system_capex_per_kw                        */
    DGEN_YS_CAPEX_COMBINED,     /* system_capex_per_kw_combined               */
    DGEN_YS_BATT_CAPEX_KWH,     /* batt_capex_per_kwh_combined                */
    DGEN_YS_PV_DEG,             /* pv_degradation_factor                      */
    DGEN_YS_ITC,                /* itc_fraction_of_capex (tech 'solar')       */
    DGEN_YS_ECON_LIFE,          /* economic_lifetime_yrs                      */
    DGEN_YS_LOAN_TERM,          /* loan_term_yrs                              */
    DGEN_YS_DOWN_PAYMENT,       /* down_payment_fraction                      */
    DGEN_YS_REAL_DISCOUNT,      /* real_discount_rate                         */
    DGEN_YS_TAX_RATE,           /* tax_rate                                   */
    DGEN_YS_COLS
};
/* by_sector_county rows: load_multiplier, elec_price_multiplier,
 * elec_price_escalator (DGEN_YC_COLS); by_state_sector: value_of_resiliency_usd. */
enum { DGEN_YC_LOAD_MULT = 0, DGEN_YC_PRICE_MULT, DGEN_YC_ESCALATOR, DGEN_YC_COLS };

typedef struct {
    const int32_t* k_sector;          /* row of by_sector (-1: none)            */
    const int32_t* k_sector_county;   /* row of by_sector_county                 */
    const int32_t* k_state_sector;    /* row of by_state_sector                  */
    const int32_t* k_county;          /* row of wholesale_row                    */
    const uint8_t* is_res;            /* sector_abbr == 'res' (load growth rule) */
    const double* load_kwh_initial;   /* load_kwh_per_customer_in_bin_initial    */
    const double* customers_initial;  /* customers_in_bin_initial                */
    const double* load_in_bin_initial;/* load_kwh_in_bin_initial                 */
} dgen_year_keys;

typedef struct {
    const double* by_sector;          /* [n_sector][DGEN_YS_COLS]                */
    const double* by_sector_county;   /* [n_sector_county][DGEN_YC_COLS]         */
    const double* by_state_sector;    /* [n_state_sector]                        */
    const int32_t* wholesale_row;     /* [n_county]: this year's wholesale row   */
    int64_t n_sector, n_sector_county, n_state_sector, n_county;
    double inflation_rate;            /* apply_financial_params' scalar          */
} dgen_year_tables;

typedef struct {                      /* the dgen_agents columns it rewrites +   */
    double *load_kwh, *price_mult, *escalator, *inflation, *pv_deg, *capex, *capex_combined;
    double *batt_capex_kwh, *itc_frac, *down_payment, *real_discount, *tax_rate, *vor;
    int32_t *econ_life, *loan_term, *wholesale_row;
    double *customers_in_bin, *load_kwh_in_bin;   /* the loop's developable weight / load */
} dgen_year_out;

int32_t dgen_year_inputs(dgen_ctx* ctx, const dgen_year_keys* keys, const dgen_year_tables* tables,
                         const dgen_year_out* out, int64_t n, void* stream);

/* First-model-year market seeding, elec.estimate_initial_market_shares
 * (elec.py:701-765): per (state, sector, tech) group the developable
 * customers (pandas' Kahan-compensated group sum, rows in frame order) and the
 * agent count, then each agent's portion of the state's starting capacities
 * (caps[g * 5 + {system_mw, batt_mw, batt_mwh, pv_systems_count,
 * batt_systems_count}], NaN when the state has no row) and the
 * *_last_year / initial_* columns, NaN -> 0 (fillna).  Group g's members are
 * rows idx[seg_off[g] .. seg_off[g+1]) in frame order.                      */
typedef struct {
    const double* developable_agent_weight;
    const double* system_capex_per_kw;
} dgen_init_in;

typedef struct {
    double *adopters_cum_last_year, *system_kw_cum_last_year, *batt_kw_cum_last_year;
    double *batt_kwh_cum_last_year, *market_share_last_year, *market_value_last_year;
    double *initial_number_of_adopters, *initial_pv_kw, *initial_batt_kw, *initial_batt_kwh;
    double *initial_market_share, *initial_market_value;
    double *developable_customers_in_state;   /* per group, [n_seg]          */
    int64_t *agent_count;                     /* per group, [n_seg]          */
} dgen_init_out;

int32_t dgen_initial_market_shares(dgen_ctx* ctx, const dgen_init_in* in, const dgen_init_out* out,
                                   const int64_t* idx, const int64_t* seg_off, const double* caps,
                                   int64_t n_seg, void* stream);

/* ------------------------------------------------------------------------
 * Finance-series export, finance_series_export.py:9-81:
 * _norm25 of the six yearly arrays the export writes per agent, in the
 * reference's column order -- cf_energy_value / utility_bill_w_sys /
 * utility_bill_wo_sys of the pv_only case, then of the pv_batt case (O's
 * cfev_pv, bill_w_pv, bill_wo_pv, cfev_batt, bill_w_batt, bill_wo_batt).
 * Entry k of agent i = O.<series>[i * (DGEN_MAXY + 1) + k] for k < list_len[i]
 * (the agent's list length, economic life + 1), 0 otherwise; first 25 entries
 * (the 26-long lists are truncated); non-finite -> 0.  out: [6][n][25] f64.
 * ---------------------------------------------------------------------- */
int32_t dgen_finance_series(dgen_ctx* ctx, const dgen_outputs* O, const int32_t* list_len, int64_t n,
                            double* out, void* stream);

/* Average per-call kernel time (ms) of the dgen_size_agents calls since the
 * previous query: k_size, k_hourly_batt, k_batt_finance, each summed over the
 * call's chunks (HIP events recorded on the stream each kernel runs on).
 * Returns the number of calls averaged (>= 0) or an error code.              */
int32_t dgen_kernel_times(dgen_ctx* ctx, double* ms_size, double* ms_hourly, double* ms_finance);

/* The record forms the last dgen_size_agents call on ctx took, as the call
 * decided them from its tables, settings and LDS limits (ABI 11): out[0] the
 * battery case's net-billing split built in the scan (dgen_set_nb_scan),
 * out[1] battery-case demand records (dgen_set_dc_records), out[2] the TS
 * sell-rate agents' own split scan, out[3] the demand machinery on (demand
 * charges billed or kWh/kW tier peaks), out[4] the period count the kernels'
 * LDS is laid out for (the tables' max_periods after the call's adjustments),
 * out[5] the demand periods per record, out[6] the demand envelopes of the
 * first-evaluation tariffs prebuilt by their own kernel (k_dc_env).  Writes
 * min(n_out, DGEN_PATHS_N) values; returns DGEN_PATHS_N.  For byte
 * accounting (bench.py); replaces nothing in the reference.                 */
#define DGEN_PATHS_N 7
int32_t dgen_last_paths(dgen_ctx* ctx, int32_t* out, int32_t n_out);

/* Demand envelopes (the PV-only search's per-(month, demand period) import
 * lines, demand-charge and kWh/kW-tier batches) of every agent's
 * first-evaluation tariff prebuilt by their own kernel ahead of the search
 * (1, default; k_dc_env: day lanes, coalesced 16-B profile loads) or built by
 * the search kernel at the first evaluation that bills the tariff (0; the
 * DGEN_DC_PREBUILD=0 environment setting at dgen_open does the same).  The
 * kept lines are the same set either way and an evaluation takes their max,
 * so results are bit-identical (ABI 11).  Replaces nothing in the reference. */
int32_t dgen_set_dc_prebuild(dgen_ctx* ctx, int32_t on);

/* Rows [0, hi) of the next dgen_size_agents batches hold only agents without a
 * scratch slot (scratch_slot < 0: bins-only billing, no net-billing or demand
 * path; engine.profile_order puts them first).  A batch that has scratch slots
 * then sizes those rows with the bins-only instantiations of k_size /
 * k_batt_finance (fewer registers, slimmer LDS) and skips them in the split
 * prebuild; results are bit-identical (the same bills on the same path).  0
 * (default): the whole batch takes the batch's form.  A row in [0, hi) that
 * does hold a scratch slot would be flagged DGEN_ST_SCRATCH, so the caller
 * must only cover true bins-only rows (ABI 13).  Replaces nothing in the
 * reference. */
int32_t dgen_set_nem_rows(dgen_ctx* ctx, int64_t hi);

/* Pipeline depth of dgen_size_agents: the batch is cut into `chunks` pieces;
 * k_size of piece j+1 runs on the caller's stream while k_hourly_batt and
 * k_batt_finance of piece j run on a context-owned second stream (forked from
 * and joined back into the caller's stream, so stream order is unchanged for
 * the caller).  1 = no overlap.  Range [1, 16]; default DGEN_DEFAULT_CHUNKS.
 * Replaces nothing in the reference (its per-agent loop is serial, ff:1149). */
int32_t dgen_set_pipeline(dgen_ctx* ctx, int32_t chunks);

/* The hourly planes of a batch already sized by dgen_size_agents (same ctx
 * settings, same tables / agents / workspace), without re-sizing it: the
 * 8760-h scan alone, re-deriving the battery run from O's sizing outputs
 * (system_kw, x_last, tariff_final, switched, status); every other output it
 * writes gets the value the sizing call wrote.  For shards whose planes do not
 * fit beside the batch (dgen_amd.year_loop's chunked per-state export): size
 * the whole shard without planes, then call this per chunk of agents with the
 * chunk's slices of O and a plane buffer.  Replaces nothing in the reference
 * (its lists come out of the one sizing call, ff:505-539).                  */
int32_t dgen_hourly_planes(dgen_ctx* ctx, const dgen_tables* tables, const dgen_agents* agents,
                           const dgen_outputs* outputs, int64_t n, void* workspace, size_t workspace_bytes,
                           int64_t n_scratch, void* stream);

/* The per-state export's combined plane of a batch already sized by
 * dgen_size_agents (same ctx settings, tables, agents, workspace; as
 * dgen_hourly_planes, the scan alone): per agent-hour the f64 value
 * dgen_state_hourly adds from the three float32 planes,
 *   ((double)pvo * w_pvo + (double)wbt * w_batt) + (double)base * w_non,
 * in hour-quad tiles ((h, i) at ((h / 4) * n + i) * 4 + h % 4), from the
 * weights of dgen_export_weights.  dgen_state_hourly with planes_f32 = 3 sums
 * it (baseline = the plane; pvonly / with_batt / weights unused): the same
 * per-state rows, bit for bit, from 8 B per agent-hour written and read
 * instead of 12.  Daily plan without the loss model only (DGEN_E_ARG
 * otherwise: use dgen_hourly_planes).  n < 2^27.  Replaces nothing in the
 * reference (attachment_rate_functions.py:151-206 sums the frame's lists).   */
int32_t dgen_export_plane(dgen_ctx* ctx, const dgen_tables* tables, const dgen_agents* agents,
                          const dgen_outputs* outputs, const double* w_pvo, const double* w_batt,
                          const double* w_non, double* plane, int64_t n, void* workspace,
                          size_t workspace_bytes, int64_t n_scratch, void* stream);

/* The per-state export from the with-battery plane alone (ABI 11): a batch
 * sized by dgen_size_agents with only outputs.net_with_batt set (float32
 * hour-quad tiles; daily plan, no loss model, no demand charges / kWh/kW
 * tiers) -- the load and PV-only net load of each agent-hour are recomputed
 * from the profile rows (agents' load_row / cf_row / load_kwh, outputs'
 * x_last / status) as the scan forms them, so out (per segment, 8760 rows,
 * MW) equals dgen_state_hourly over the three float32 planes bit for bit,
 * from 4 B of plane per agent-hour.  idx / seg_off as dgen_state_hourly.
 * Replaces nothing in the reference (attachment_rate_functions.py:151-206
 * sums the frame's hourly lists).  The per-agent scalars live in a buffer
 * the ctx owns and grows on demand (after a device-wide sync): calls on one
 * ctx must be serialised, as for every other entry point.                 */
int32_t dgen_state_hourly_rows(dgen_ctx* ctx, const dgen_tables* tables, const dgen_agents* agents,
                               const dgen_outputs* outputs, const float* with_batt, const double* w_pvo,
                               const double* w_batt, const double* w_non, const int64_t* idx, int64_t n,
                               const int64_t* seg_off, int64_t n_seg, double* out, void* stream);

/* Months of the year per k_hourly_batt launch (the sequential 8760-h scan of
 * dgen_size_agents): the year is swept in ceil(12 / months) launches, SOC and
 * the annual PV sum carried between them in the workspace, so that all
 * resident waves read the same weeks of the shared profile rows and those
 * slices stay cache-resident.  Results do not depend on it.  Range [1, 12];
 * default DGEN_DEFAULT_HOURLY_MONTHS.  Replaces nothing in the reference.   */
int32_t dgen_set_hourly_segment(dgen_ctx* ctx, int32_t months);

/* PV+battery forward run on (1, default: the reference, which always runs it
 * at ff:479) or off (0: the PV-only variant of SURVEY 8(d)).  Off: no battery
 * sizing, storage rate switch or dispatch (batt_kw = batt_kwh = 0, the
 * with-battery plane is the PV-only net load at kW*), k_batt_finance is not
 * launched: npv_pv_batt is NaN and the three battery-case yearly arrays are
 * left untouched.                                                          */
int32_t dgen_set_battery(dgen_ctx* ctx, int32_t on);

/* Where the battery case's net-billing split is built for agents that bill
 * net without a TS sell rate: cap > 0 (default DGEN_NB_CAPM) in
 * k_hourly_batt's scan, as the system output is produced, holding at most cap
 * mixed hours per month -- k_batt_finance then bills from the record and the
 * system-output plane is not written for agents without demand charges; an
 * agent whose split overflows gets its plane from a repair pass and is billed
 * as with 0 -- or 0: in k_batt_finance from the plane.  Results are equal up
 * to the rounding of the re-associated sums (bit-identical for an overflowing
 * agent).  The scan form pays its classification in every wave that holds
 * such an agent, so a batch where few agents qualify is faster with 0 (the
 * Python engine decides per batch: Engine.upload_agents).  Applies to
 * batches whose tariffs have at most 10 periods (the scan form's doubled
 * bins then fit 64 KB of LDS per block); others build in k_batt_finance.
 * Range [0, DGEN_NB_CAPM].  Replaces nothing in the reference.            */
int32_t dgen_set_nb_scan(dgen_ctx* ctx, int32_t cap);

/* The batch rows [lo, hi) that hold every agent able to bill the hourly TS
 * sell rate (a scratch slot and a wholesale row, non-CA): the TS agents' own
 * split scan (k_hourly_batt<TS>, batches with hourly planes and a wholesale
 * table, no demand charges) is launched over those rows only; lo == hi: none.
 * Default [0, INT64_MAX): the whole batch.  Results do not depend on it as
 * long as the range covers those agents (the Python engine sets it from the
 * device order, Engine.upload_agents).  Replaces nothing in the reference.  */
int32_t dgen_set_ts_rows(dgen_ctx* ctx, int64_t lo, int64_t hi);

/* Battery-case demand records holding at most cap kept hours per agent
 * (default and maximum DGEN_DCR_CAP), or none (0).  With demand charges
 * billed (or kWh/kW tier peaks) and the daily plan, k_hourly_batt's scan keeps
 * per (month, demand period) the max load and a lower bound of every analysis
 * year's peak import, and the hours that can raise some year's peak above it
 * (a context-owned buffer per scratch slot); k_batt_finance's battery-case
 * demand pass then stages those hours only, instead of all 8760 hours of the
 * system-output plane.  Results are bit-identical (peaks are maxima of the
 * same values).  An agent whose kept hours overflow the record falls back to
 * the plane.  Replaces nothing in the reference.                            */
int32_t dgen_set_dc_records(dgen_ctx* ctx, int32_t cap);

/* Certified Brent paths (ABI 14).  The search bills from re-associated sums
 * (slot sums, net-billing split), a few ulps from the reference's hour order,
 * and scipy's bounded Brent can turn such a difference into another search
 * path (ff:440-447).  mode 1 (default): every search traces its objective
 * values; a replay with a bound on |device - reference| carried through every
 * Brent state variable lists the agents with a decision that bound does not
 * settle, and those agents' searches re-run in the reference's arithmetic
 * (hours in time order: Utilityrate5 bins, bill, Cashloan, op for op), so every
 * agent takes the reference's path.  mode 2: every searched agent re-runs
 * (test mode).  mode 0: off (k_size's search alone).  Replaces nothing in the
 * reference (its one path is the hour-order one).                            */
int32_t dgen_set_exact(dgen_ctx* ctx, int32_t mode);

/* Agents the last dgen_size_agents call re-ran in the reference's arithmetic
 * (synchronises the ctx's stream work of that call).                         */
int32_t dgen_exact_count(dgen_ctx* ctx, int64_t* out);

#ifdef __cplusplus
}
#endif
#endif /* DGEN_HIP_H */
