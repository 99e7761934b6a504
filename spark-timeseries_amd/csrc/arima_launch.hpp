// arima_launch.hpp — host-side launchers of the HIP kernels (internal; the public ABI is include/sparkts_arima.h)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sts {

int launch_difference(const double *in, int64_t ld_in, double *out, int64_t ld_out, int64_t N, int T, int d,
                      int drop, hipStream_t s);
int launch_search_init(double *best_aic, int32_t *order, double *coef, int64_t N, hipStream_t s);
constexpr int kSearchMaxLanes = 32;
struct SearchBests {               // the order search's per-lane best candidates (by value into k_search_merge)
    const double *aic[kSearchMaxLanes];
    const int32_t *order[kSearchMaxLanes];
    const double *coef[kSearchMaxLanes];
};
int launch_search_merge(const SearchBests &b, int lanes, int64_t N, double *best_aic, int32_t *order, double *coef,
                        hipStream_t s);
int launch_search_select(const double *cand_coef, const double *cand_ll, const int32_t *cand_status,
                         const uint8_t *cand_flags, int64_t N, int p, int d, int q, int I,
                         const unsigned long long *fit_ctl, double *best_aic, int32_t *order, double *coef,
                         hipStream_t s);
int launch_forecast(const double *ts, int64_t ld_in, const double *coef, int k, double *out, int64_t ld_out,
                    int64_t N, int T, int p, int d, int q, int I, int n_future, hipStream_t s);
int launch_inverse_difference(const double *in, int64_t ld_in, double *out, int64_t ld_out, int64_t N, int T,
                              int d, hipStream_t s);
// The fit kernel's counter words (ctl) and express-ring ready words are initialised by the kernel that runs before it
// on the same stream (k_hr_init, else k_fit_prep): ctl[] = 0 except ctl[15] = ~0 and the option words 19, 44-47;
// xready[0 .. xready_words) = 0. ctl == nullptr / xready_words == 0: nothing to prepare.
constexpr int kFitCtlWords = 48;
struct FitPrep {
    unsigned long long *ctl = nullptr;
    unsigned *xready = nullptr;
    int64_t xready_words = 0;
    unsigned long long v19 = 0, v44 = 0, v45 = 0, v46 = 0, v47 = 0;
};
int launch_fit_prep(const FitPrep &prep, hipStream_t s);
// hr_grid > 0: that many single-wave workgroups stride over the series (bounds the rows in flight, so the 2(C_A + C_B)
// passes over a row can hit the Infinity Cache); 0: one lane per series in 256-lane workgroups.
// dd (here and in the fit launchers): 1 = y holds the RAW rows of a d = 1 fit and every pass differences them on the
// fly (arima_device.hpp stream_row); 0 = y holds the differenced rows.
int launch_hr_init(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, double *init_out,
                   int32_t *status_out, hipStream_t s, int hr_grid = 0, int dd = 0, const FitPrep &prep = FitPrep{});
int launch_ar_fit(const double *y, int64_t ld, int n, int64_t N, int p, int I, double *coef_out, double *ll_out,
                  int32_t *status_out, int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out,
                  hipStream_t s, int dd = 0);
int launch_cg_fit(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, int smear,
                  const double *init, const int32_t *init_status, double *coef_out, double *ll_out,
                  int32_t *status_out, int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out,
                  unsigned long long *ctl, int grid_blocks, int express_blocks, unsigned char *xq, unsigned *xready,
                  int join_express, hipStream_t s, int dd = 0);
constexpr int kExpressRingEntries = 32768;      // k_cg_fit's express hand-offs per launch (entries never reused)
constexpr int kExpressRingBytes = kExpressRingEntries * 512;   // x kExpressEntryBytes
constexpr int kExpressReadyBytes = kExpressRingEntries * 4;
int launch_css_loglik(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, const double *coef,
                      double *ll_out, hipStream_t s);
int launch_css_grad(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, int smear,
                    const double *coef, double *g_out, hipStream_t s);
int launch_model_flags(const double *coef, int64_t N, int p, int q, int I, uint8_t *flags_out, hipStream_t s);
// base_host: I + p + q host doubles (passed to the kernel by value)
int launch_sample(double *out, int64_t ld, int64_t N, int T, int p, int d, int q, int I, const double *base_host,
                  double jitter, uint64_t seed, int64_t first, hipStream_t s);
int cg_fit_series_per_block(int p, int q, int I);   // optimizer slots of one fit workgroup
// k_cg_fit workgroups are single waves (4 per CU, one per SIMD, each with a quarter of the LDS): a wave that has
// finished its series leaves the CU at once, so the next fit's waves take its SIMD and LDS share while the other
// waves of the CU still run their slowest series (pipelined fits)
constexpr int kFitBlockWaves = 1;            // waves per k_cg_fit workgroup
constexpr int kFitWavesPerCU = 4;            // resident k_cg_fit waves per CU (one per SIMD)
constexpr int kFitBlocksPerCU = kFitWavesPerCU / kFitBlockWaves;

constexpr int kMergeLiveDefault = 16;        // k_cg_fit's drain merge threshold (option "merge_live"; 0 = off)

// ---- ARIMA.autoFit (arima_autofit.hip) ----
// candidate (p, q, intercept) orders the stepwise walk can meet: p <= max(max_p, 2), q <= 2 (combo (p * 3 + q) * 2 + I;
// max_p <= kAfMaxP: its css-bobyqa retries have at most 11 parameters, the dimensions arima_bobyqa.hip compiles)
constexpr int kAfMaxP = 8;
constexpr int kAfCombosMax = (kAfMaxP + 1) * 6;
inline int af_combos(int max_p) { return ((max_p > 2 ? max_p : 2) + 1) * 6; }
constexpr int kAfMaxCand = 4;      // distinct candidates of one round of one series
struct AfSeries {                  // one series' walk state (findBestARMAModel's locals, ARIMA.scala:321-375)
    double best_aic;               // curBestAIC
    unsigned long long seen;       // pastParams, one bit per (p, q, intercept)
    int32_t dsel;                  // d chosen by the KPSS search (-1: none)
    int32_t status;                // ARIMA_ST_*
    int32_t best;                  // packed p | q << 4 | I << 8 of curBestModel, -1 = null
    int32_t n_fits;                // candidate fits run so far
    int32_t ncand;                 // candidates of the current round (0: the walk is over)
    int32_t cand[kAfMaxCand];      // nextParams, packed, deduplicated in first-appearance order
    int32_t slot[kAfMaxCand];      // each candidate's row in its order's list this round
};
int launch_kpss_c(const double *w, int64_t ld, int n, int64_t N, int d, int32_t *dsel, double *stat_out, hipStream_t s);
int kpss_lag_host(int n);
int kpss_lag_max();
int launch_difference_sel(const double *in, int64_t ld_in, double *out, int64_t ld_out, int64_t N, int T,
                          const int32_t *dsel, int d, hipStream_t s);
int launch_af_init(int64_t N, const int32_t *dsel, AfSeries *st, int32_t kpss_status, hipStream_t s);
int launch_af_plan(int64_t N, AfSeries *st, unsigned *counts, int32_t *lists, hipStream_t s);
int launch_gather_rows(const double *in, int64_t ld, const int32_t *list, int64_t count, int T, double *out,
                       hipStream_t s);
int launch_af_update(int64_t N, AfSeries *st, const int64_t *off, const double *res_coef, const double *res_ll,
                     const int32_t *res_status, const uint8_t *res_flags, double *best_coef, int max_p, int max_q,
                     hipStream_t s);
int launch_af_finish(int64_t N, const AfSeries *st, const double *best_coef, int32_t *order_out, double *coef_out,
                     double *aic_out, int32_t *status_out, int32_t *n_fits_out, hipStream_t s);

// css-bobyqa (arima_bobyqa.hip): one lane per series after the initial parameters; refit_status (optional): only the
// series whose css-cgd status there is an optimizer exception (autoFit's fitTryBothStrategies) are refitted in place
int launch_bobyqa_fit(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, const double *init,
                      const int32_t *init_status, const int32_t *refit_status, double *coef_out, double *ll_out,
                      int32_t *status_out, int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out, bool wave,
                      hipStream_t s);

// autoFit: the css-bobyqa retries of a whole round (every order's rows whose css-cgd fit threw in the optimizer), one
// launch; rows = the differenced series (ld), lists / off = the round's per-order lists and row offsets, init /
// init_status = each row's Hannan-Rissanen init (k-strided from off[cb] * 11) and status; list / count: workspace
// (the list, bucketed by dimension k = p + q + intercept -- bucket k at list[k * stride ..], counts[k] rows -- then
// one kernel per dimension present, each on its own stream; ncombos orders in the round's layout, coefficient rows
// kc-strided from off[cb] * kc)
constexpr int kBqRefitBuckets = 12;
int launch_bobyqa_refit_list(const int64_t *off, int ncombos, int64_t total, const int32_t *status, int32_t *list,
                             int64_t stride, unsigned *counts, hipStream_t s);
int launch_bobyqa_refit_dim(int k, const double *rows_, int64_t ld, int n, const int32_t *lists, int64_t N,
                            const int64_t *off, int ncombos, int kc, const int32_t *list, const unsigned *counts,
                            int64_t rows, const double *init, const int32_t *init_status, double *coef, double *ll,
                            int32_t *status, uint8_t *flags, bool wave, hipStream_t s);

int hr_shape_status_host(int n, int p, int q, int I);
int ar_shape_status_host(int n, int p, int I);

// ---- the runtime-order path (arima_generic.hip): p or q above the compiled orders (5), up to kGenMaxOrder ----
constexpr int kFastMaxOrder = 5;   // orders the compile-time kernels cover
constexpr int kGenMaxOrder = 20;   // p, q <= 20
constexpr int kGenMaxK = 2 * kGenMaxOrder + 1;
inline bool gen_order(int p, int q) { return p > kFastMaxOrder || q > kFastMaxOrder; }
// Fused differencing pays where the fused Householder init keeps its registers (k_hr_init<P, Q, I, true>): C2's
// (2,1,2)+c gains 7 % from it, C4's (5,1,5)+c loses 6-16 % (profiles/r06/d_ab, p_c4fuse, q_fuse); the compiled orders
// with p + q <= 6 fuse, the others take the k_difference copy. The runtime-order kernels always fuse.
inline bool fuse_pays(int p, int q) { return gen_order(p, q) || p + q <= 6; }
bool gen_orders_ok(int p, int q);
int launch_gen_hr_init(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, double *init_out,
                       int32_t *status_out, int dd, const FitPrep &prep, hipStream_t s);
int launch_gen_ar_fit(const double *y, int64_t ld, int n, int64_t N, int p, int I, double *coef_out, double *ll_out,
                      int32_t *status_out, int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out, int dd,
                      hipStream_t s);
int launch_gen_fit(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, int smear, const double *init,
                   const int32_t *init_status, double *coef_out, double *ll_out, int32_t *status_out,
                   int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out, unsigned long long *ctl, int dd,
                   hipStream_t s);
int launch_gen_css_loglik(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, const double *coef,
                          double *ll_out, hipStream_t s);
int launch_gen_css_grad(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, int smear,
                        const double *coef, double *g_out, hipStream_t s);
int launch_gen_model_flags(const double *coef, int64_t N, int p, int q, int I, uint8_t *flags_out, hipStream_t s);
int64_t gen_forecast_ws_doubles(int T, int p, int d, int q, int n_future);
int launch_gen_forecast(const double *ts, int64_t ld_in, const double *coef, int k, double *out, int64_t ld_out,
                        int64_t N, int T, int p, int d, int q, int I, int n_future, double *ws, int64_t ws_stride,
                        hipStream_t s);

}  // namespace sts
