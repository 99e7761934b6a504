/*
 * sparkts_arima.h — C ABI of the MI355X-native batched ARIMA (CSS-CGD) engine.
 *
 * This library is a drop-in for ONE hot path of spark-ts (dhmodi/spark-timeseries, sparkts 0.4.0-SNAPSHOT):
 *
 *     ARIMA.fitModel(p, d, q, ts, includeIntercept, method = "css-cgd", userInitParams)
 *         src/main/scala/com/cloudera/sparkts/models/ARIMA.scala:79-116
 *
 * called once per series inside TimeSeriesRDD.mapSeries (TimeSeriesRDD.scala:249-260). The JVM binding
 * a maintainer adds on the reference side (JNI / Panama) is shown in INTEGRATION.md; the Python mirror of
 * python/sparkts/models/ARIMA.py lives in spark-timeseries_amd/sparkts_amd/.
 *
 * Conventions
 *   - Plain C types only. Host-buffer entry points take caller-owned host memory; the library never keeps a
 *     pointer after return. `*_device` entry points take device (HBM) pointers and a hipStream_t passed as
 *     `void*` (NULL = the handle's own stream) and are asynchronous w.r.t. the host: they enqueue their work
 *     and return (results are valid once that stream reaches the call's end). Calls on one handle are also
 *     ordered on the device whichever streams they use, because they share the handle's workspaces --
 *     except fit calls under the "fit_pipeline" option (arima_set_option; default 3): consecutive
 *     arima_fit_batch_device calls rotate over P fit contexts and may run concurrently -- unless a call's
 *     buffers overlap an in-flight call's (it reads that call's outputs, writes its inputs, or writes the same
 *     outputs): then it waits for that call, whatever fit_pipeline is set to when it is issued, so results always
 *     equal fit_pipeline 1's. Every non-fit call
 *     still waits for all earlier calls. arima_get_last_stats waits for the last call's device work.
 *     Host-buffer entry points block (arima_fit_batch pipelines its own chunks internally: "host_chunk",
 *     "host_pipeline").
 *   - A batch is N series of equal length T, series-major: element t of series i is series[i*ld + t]
 *     (ld == T for the host-buffer entry points). One call = one Spark partition bucketed by length.
 *   - Coefficient layout per series is the reference's: [c?, phi_1..phi_p, theta_1..theta_q]
 *     (ARIMA.scala:74-77, 406); k = arima_num_params(p, q, include_intercept).
 *   - Return value: ARIMA_OK or a negative ARIMA_E_* (API misuse / device failure only). Per-series
 *     outcomes are reported in status_out (ARIMA_ST_*), one code per exception the reference can throw on
 *     this path; a failed series never aborts the batch and its coefficients are NaN.
 */
#ifndef SPARKTS_ARIMA_H
#define SPARKTS_ARIMA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- call-level return codes ---------------------------------------------------------------------- */
#define ARIMA_OK              0
#define ARIMA_E_INVALID_ARG  (-1)
#define ARIMA_E_UNSUPPORTED  (-2)
#define ARIMA_E_DEVICE       (-3)
#define ARIMA_E_OOM          (-4)

/* ---- per-series status: one code per reference outcome ----------------- */
#define ARIMA_ST_OK                  0  /* fit returned normally                                             */
#define ARIMA_ST_MAX_EVAL            1  /* commons TooManyEvaluationsException, MaxEval(10000) ARIMA.scala:196 */
#define ARIMA_ST_BRACKET_MAX_EVAL    2  /* commons BracketFinder's own 500-evaluation cap                    */
#define ARIMA_ST_MAX_ITER            3  /* commons TooManyIterationsException, MaxIter(10000) ARIMA.scala:195 */
#define ARIMA_ST_SINGULAR            4  /* commons SingularMatrixException (QR rDiag == 0), ARIMA.scala:240   */
#define ARIMA_ST_NOT_ENOUGH_DATA     5  /* MathIllegalArgumentException: rows < predictors + 1               */
#define ARIMA_ST_NO_DATA             6  /* NoDataException: zero rows, or zero columns without intercept     */
#define ARIMA_ST_BAD_INTERVAL        7  /* NumberIsTooLarge / OutOfRange from SearchInterval (line search)   */
#define ARIMA_ST_ZERO_PARAMS         8  /* k == 0 parameters (ArithmeticException / index error)             */
#define ARIMA_ST_UNSUPPORTED_METHOD  9  /* UnsupportedOperationException, ARIMA.scala:108 (unknown method)    */
#define ARIMA_ST_SERIES_TOO_SHORT   10  /* negative lag-matrix size (NegativeArraySize / IndexOutOfBounds)    */
/* ARIMA.autoFit outcomes (ARIMA.scala:280-375), arima_autofit_batch* only */
#define ARIMA_ST_NOT_STATIONARY     11  /* no d <= max_d passes the KPSS test: "stationarity not achieved", :293-296 */
#define ARIMA_ST_NO_MODEL           12  /* no candidate qualified: curBestModel stays null (NullPointerException)  */
/* 13 and 15 are retired: they reported BOBYQA's RESCUE branch before it was restated (round 6); never returned */
/* css-bobyqa outcomes (ARIMA.fitWithCSSBOBYQA, ARIMA.scala:130-160) */
#define ARIMA_ST_TOO_FEW_PARAMS     14  /* BOBYQAOptimizer needs >= 2 parameters (NumberIsTooSmallException)    */

/* ---- fit methods (ARIMA.scala:105-109) -------------------------------------------------------------- */
#define ARIMA_METHOD_CSS_CGD     0
#define ARIMA_METHOD_CSS_BOBYQA  1      /* commons BOBYQAOptimizer as ARIMA.fitWithCSSBOBYQA configures it (ARIMA.scala:130-160) */

/* ---- stationarity / invertibility flags (ARIMAModel.isStationary / isInvertible, ARIMA.scala:777-815) - */
#define ARIMA_FLAG_STATIONARY  1u
#define ARIMA_FLAG_INVERTIBLE  2u

typedef struct arima_handle arima_handle;

/* Aggregate counters of the last fit call on a handle (for roofline accounting). */
typedef struct arima_fit_stats {
    int64_t n_series;
    int64_t f_passes;        /* objective (CSS) passes actually executed over a series            */
    int64_t g_passes;        /* gradient passes actually executed over a series (each also yields CSS) */
    int64_t hr_passes;       /* Hannan-Rissanen streaming-QR passes executed                       */
    int64_t n_eval;          /* objective evaluations as counted by the reference (incl. memoised)  */
    int64_t n_grad;          /* gradient evaluations as counted by the reference                    */
    double  flops;           /* algorithmic flops of all passes executed (SURVEY.md 8(d) formula)   */
    double  ms_difference;   /* device time of each kernel of the last call (HIP events, ms)        */
    double  ms_hr_init;
    double  ms_cg_fit;
    double  ms_total;
    int64_t wave_f_passes;   /* wave-level objective-only passes of the fit kernel                   */
    int64_t wave_g_passes;   /* wave-level passes that included the gradient recursion               */
    int64_t grid_blocks;     /* workgroups of the persistent fit kernel                               */
    int64_t spec_hits;       /* objective evaluations answered by a speculative line-search point     */
    int64_t wave_multi_passes; /* wave-level objective passes that carried speculative points          */
    int64_t spec_chains;     /* objective chains evaluated by lane F passes (primary + speculative)    */
    int64_t express_blocks;  /* CUs of express workgroups in the fit kernel (long-running series) */
    int64_t express_series;  /* series finished on the express path                                    */
    int64_t express_f_passes; /* objective / gradient passes run on the express path                    */
    int64_t express_g_passes;
    int64_t fault;           /* != 0: the fit kernel's hand-off watchdog fired (1 = stall, 2 = lost request, 3 = merge stall);
                                the call also returns ARIMA_E_DEVICE from arima_synchronize / blocking entry points */
    int64_t fault_info[5];   /* the kernel's record of the first fault (ticket, fills, bulk waves done, ...)      */
    int64_t diag[6];         /* diagnostics of builds with -DSTS_TIMING; else 0                       */
    int64_t ride_passes;     /* objective requests served by gradient passes (counted in g_passes)    */
    int64_t series_done;     /* series whose result the fit kernels wrote (== n_series unless a fault dropped some) */
    int64_t express_pit_passes;  /* express objective passes run parallel in time (all lanes on one series)   */
    int64_t express_pit_sweeps;  /* block sweeps of the parallel-in-time passes (objective and gradient)     */
    int64_t express_pit_g_passes;    /* express gradient passes run parallel in time                        */
    int64_t wave_chains;         /* objective chains the bulk objective passes computed (64 x chains per pass) */
    int64_t low_util_passes;     /* bulk wave passes that served fewer than 32 lanes                         */
    int64_t diag_step_cycles;    /* STS_TIMING builds: optimizer-step cycles, and refill cycles (within diag[2]) */
    int64_t diag_refill_cycles;
    int64_t merge_series;        /* series the drain merge moved between bulk waves (option "merge_live")    */
    int64_t merge_waves;         /* bulk waves that handed their last series over and left                   */
} arima_fit_stats;

/* ---- lifecycle ------------------------------------------------------------------------------------- */
/* One handle per device. Calls on one handle are serialised internally (thread-safe). arima_get_last_stats
 * waits for the device work of the last fit on the handle (the fit calls themselves do not). */
int         arima_create(int device, arima_handle **out);
int         arima_destroy(arima_handle *h);
const char *arima_last_error(const arima_handle *h);
const char *arima_status_name(int status);
int         arima_num_params(int p, int q, int include_intercept);
int         arima_get_last_stats(const arima_handle *h, arima_fit_stats *out);
/* Blocks until the device work of every call issued on the handle so far has finished. */
int         arima_synchronize(arima_handle *h);
/* Orders: p, q <= 5 run the order-specialised kernels, 5 < p, q <= 20 the runtime-order path (arima_generic.hip: the
 * same results, not tuned); p or q > 20 return ARIMA_E_UNSUPPORTED, and so do css-bobyqa fits of more than 11
 * parameters (the dimensions its kernels compile) and autoFit with max_p > 8 (its css-bobyqa retries).
 * Tuning knobs (not part of the reference contract): "smear" (Breeze reading at ARIMA.scala:526, default 1),
 * "fit_pipeline" (fit contexts in rotation for *_device fits, 1..8, default 3), "host_chunk" / "host_pipeline"
 * (series per chunk and contexts of the chunked host path: 131072 / 6 when GPU_MAX_HW_QUEUES >= 8 at arima_create, else
 * 262144 / 3), "host_tail" (1: the host path halves its last chunks), "express_blocks",
 * "grid_blocks", "search_lanes" (in-kernel scheduler and order-search concurrency), "hr_grid" (k_hr_init grid:
 * 0 = a lane per series, > 0 = that
 * many single-wave workgroups, -1 = 1024 for pipelined fits else 0), "fit_slice_bytes"
 * (differenced workspace of one slice of a large device fit), "express_ring" (express hand-offs per launch),
 * "row_pad" (doubles added to the stride of the differenced-row workspaces, whole 128-B lines, default 0),
 * "merge_live" (k_cg_fit drain merge: after the batch's work counter ran out, a wave with at most this many live
 * series hands them to waves still running and exits, 0..64, 0 = off; results never depend on it),
 * "search_express_blocks" (express CUs of each concurrent order-search fit, default 0; -1 = as "express_blocks"),
 * "donate_evals" / "donate_evals_drained" (evaluations before a series may move to an express wave, before / after
 * the batch's work counter ran out; 0 = the kernel's 256 / 32), "fuse_diff" (1, default: device fits of d <= 1 read the
 * caller's rows and difference them inside every pass where that pays -- compiled orders with p + q <= 6, every
 * runtime order; 2: at every order; 0: always through a k_difference workspace -- identical results),
 * "autofit_slice" (autoFit series per slice of its workspaces, 0 = from free HBM), "host_copy_threads" (host threads
 * that copy arima_fit_batch's rows into pinned blocks for the upload; default 0 = upload from pageable memory through
 * the HIP runtime's staging), "chain_overhead" (k_cg_fit's objective-pass width model; 0 = the kernel's). */
int         arima_set_option(arima_handle *h, const char *name, int64_t value);
/* Current value of a tuning knob (the names arima_set_option takes); ARIMA_E_INVALID_ARG for an unknown name. */
int         arima_get_option(const arima_handle *h, const char *name, int64_t *value);

/* ---- ARIMA.fitModel over a batch (ARIMA.scala:79-116) ----------------------------------------------- *
 * series    N x T host, series-major                 user_init  NULL (Hannan-Rissanen, ARIMA.scala:216) or N x k
 * coef_out  N x k                                    css_ll_out N: logLikelihoodCSS at coef_out (ARIMA.scala:417)
 * status_out N (ARIMA_ST_*)                          n_eval_out / n_grad_out: N, nullable (reference counters)
 * flags_out N, nullable (ARIMA_FLAG_*)                                                                     */
int arima_fit_batch(arima_handle *h, const double *series, int64_t n_series, int32_t T,
                    int32_t p, int32_t d, int32_t q, int32_t include_intercept, int32_t method,
                    const double *user_init, double *coef_out, double *css_ll_out, int32_t *status_out,
                    int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out);

/* Same, device-resident: every pointer is device memory; `ld` is the row stride (elements) of d_series. */
int arima_fit_batch_device(arima_handle *h, const double *d_series, int64_t n_series, int32_t T, int64_t ld,
                           int32_t p, int32_t d, int32_t q, int32_t include_intercept, int32_t method,
                           const double *d_user_init, double *d_coef_out, double *d_css_ll_out,
                           int32_t *d_status_out, int32_t *d_n_eval_out, int32_t *d_n_grad_out,
                           uint8_t *d_flags_out, void *stream);

/* ---- building blocks of the path (each mirrors one reference function; host buffers) --------------- */
/* UnivariateTimeSeries.differencesOfOrderD (UnivariateTimeSeries.scala:468-480): size-preserving, N x T out */
int arima_difference_batch(arima_handle *h, const double *series, int64_t n_series, int32_t T, int32_t d,
                           double *out);
/* UnivariateTimeSeries.inverseDifferencesOfOrderD (UnivariateTimeSeries.scala:489-495), N x T out */
int arima_inverse_difference_batch(arima_handle *h, const double *series, int64_t n_series, int32_t T,
                                   int32_t d, double *out);
/* ARIMAModel.logLikelihoodCSS (ARIMA.scala:417-420): differences to order d, drops d, CSS log-likelihood */
int arima_css_loglik_batch(arima_handle *h, const double *series, int64_t n_series, int32_t T,
                           int32_t p, int32_t d, int32_t q, int32_t include_intercept, const double *coef,
                           double *ll_out);
/* ARIMAModel.gradientlogLikelihoodCSSARMA (ARIMA.scala:465-534) on already-differenced series (length n) */
int arima_css_gradient_batch(arima_handle *h, const double *diffed, int64_t n_series, int32_t n,
                             int32_t p, int32_t q, int32_t include_intercept, const double *coef,
                             double *grad_out);
/* ARIMA.hannanRissanenInit (ARIMA.scala:216-242) on already-differenced series (length n), N x k out */
int arima_hannan_rissanen_batch(arima_handle *h, const double *diffed, int64_t n_series, int32_t n,
                                int32_t p, int32_t q, int32_t include_intercept, double *init_out,
                                int32_t *status_out);
/* ARIMAModel.forecast (ARIMA.scala:696-764): N x (T + n_future) out */
int arima_forecast_batch(arima_handle *h, const double *series, int64_t n_series, int32_t T,
                         int32_t p, int32_t d, int32_t q, int32_t include_intercept, const double *coef,
                         int32_t n_future, double *out);
/* Same, device-resident: d_series N x T (row stride ld), d_coef N x k, d_out N x (T + n_future) (row stride ld_out) */
int arima_forecast_batch_device(arima_handle *h, const double *d_series, int64_t n_series, int32_t T, int64_t ld,
                                int32_t p, int32_t d, int32_t q, int32_t include_intercept, const double *d_coef,
                                int32_t n_future, double *d_out, int64_t ld_out, void *stream);
/* ARIMAModel.isStationary / isInvertible (ARIMA.scala:777-815) for N coefficient rows, flags_out N */
int arima_model_flags_batch(arima_handle *h, const double *coef, int64_t n_series, int32_t p, int32_t q,
                            int32_t include_intercept, uint8_t *flags_out);

/* ---- order search (BASELINE config C5; ARIMA.autoFit's selection rule, ARIMA.scala:280-375)
 * Fits every (d, p, q, intercept) with d in [0,max_d], p in [0,max_p], q in [0,max_q] and intercept per
 * intercept_mode (0: without, 1: with, 2: both), in that lexicographic order, and keeps per series the fit
 * with the smallest approxAIC (ARIMA.scala:826-830) among those that returned normally and are stationary and
 * invertible (the isStationary && isInvertible filter, ARIMA.scala:342); ties keep the first.
 * order_out N x 4 = (p, d, q, intercept), -1s when no candidate qualified; coef_out N x 11 (zero-padded, NaN
 * when none); aic_out N (+inf when none). Host buffers; the _device variant takes device pointers.          */
int arima_order_search_batch(arima_handle *h, const double *series, int64_t n_series, int32_t T,
                             int32_t max_p, int32_t max_d, int32_t max_q, int32_t intercept_mode, int32_t method,
                             int32_t *order_out, double *coef_out, double *aic_out);
int arima_order_search_batch_device(arima_handle *h, const double *d_series, int64_t n_series, int32_t T,
                                    int64_t ld, int32_t max_p, int32_t max_d, int32_t max_q,
                                    int32_t intercept_mode, int32_t method, int32_t *d_order_out,
                                    double *d_coef_out, double *d_aic_out, void *stream);

/* ---- ARIMA.autoFit over a batch (ARIMA.scala:280-375; python/sparkts/models/ARIMA.py:25-60 `autofit`) --------- *
 * Per series: d = the first of 0..max_d whose differencesOfOrderD(ts, d) (NOT dropped) passes kpsstest(_, "c") at 5 %
 * (TimeSeriesStatisticalTests.scala:369-395); then findBestARMAModel's stepwise walk over (p, q, intercept) on that
 * differenced series with css-cgd fits, a css-bobyqa retry where css-cgd throws in the optimizer (fitTryBothStrategies,
 * ARIMA.scala:315-319) (intercept only for d <= 1; the neighbourhood never changes q -- the
 * reference's quirks, ARIMA.scala:298-300, :356-366), keeping the first minimum approxAIC among stationary and
 * invertible fits. max_p <= 8 (any max_q: the walk only meets q <= 2), any series length (KPSS lags above 32 take
 * one pass per lag). order_out N x 4 = (p, d, q, intercept) (-1s when the series has no model),
 * coef_out N x 11 (zero-padded; NaN when none), aic_out N (+inf when none), status_out N: ARIMA_ST_OK,
 * ARIMA_ST_NOT_STATIONARY, ARIMA_ST_NO_MODEL, or the KPSS regression's shape status (T <= 1). n_fits_out (nullable): candidate fits the walk ran for the series.        */
int arima_autofit_batch(arima_handle *h, const double *series, int64_t n_series, int32_t T, int32_t max_p,
                        int32_t max_d, int32_t max_q, int32_t *order_out, double *coef_out, double *aic_out,
                        int32_t *status_out, int32_t *n_fits_out);
int arima_autofit_batch_device(arima_handle *h, const double *d_series, int64_t n_series, int32_t T, int64_t ld,
                               int32_t max_p, int32_t max_d, int32_t max_q, int32_t *d_order_out,
                               double *d_coef_out, double *d_aic_out, int32_t *d_status_out, int32_t *d_n_fits_out,
                               void *stream);
/* TimeSeriesStatisticalTests.kpsstest(ts, "c") (TimeSeriesStatisticalTests.scala:369-393) per series: stat_out N,
 * status_out N (ARIMA_ST_OK, or the OLS shape status for T <= 1). Host buffers.                                  */
int arima_kpss_batch(arima_handle *h, const double *series, int64_t n_series, int32_t T, double *stat_out,
                     int32_t *status_out);

/* ---- synthetic workload generator (ARIMAModel.sample semantics, ARIMA.scala:655-678) ---------------- *
 * Writes N x T series (row stride ld) into device memory: per-series coefficients = base +/- U(0, jitter)
 * (redrawn until stationary and invertible), Philox4x32-10 + Box-Muller N(0,1) noise keyed by (seed,
 * first_series + i, t). Deterministic for a given (seed, global series id) whatever the sharding.           */
int arima_sample_batch_device(arima_handle *h, double *d_series, int64_t n_series, int32_t T, int64_t ld,
                              int32_t p, int32_t d, int32_t q, int32_t include_intercept,
                              const double *base_coef, double jitter, uint64_t seed, int64_t first_series,
                              void *stream);

#ifdef __cplusplus
}
#endif

#endif /* SPARKTS_ARIMA_H */
