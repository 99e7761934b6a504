// arima_autofit.hip — the device side of ARIMA.autoFit over a batch (ARIMA.scala:280-375):
//
//   k_kpss_c           TimeSeriesStatisticalTests.kpsstest(ts, "c") (stats/TimeSeriesStatisticalTests.scala:369-431)
//                      on differencesOfOrderD(ts, d) -- NOT dropped -- for one candidate d; the first passing d wins
//   k_difference_sel   the rows of the series still undecided differenced at the next candidate d (decided rows keep
//                      theirs, so the workspace ends as every series' `diffedTs`, ARIMA.scala:298)
//   k_af_plan          one round of findBestARMAModel's stepwise walk (:310-375): every walking series appends its
//                      candidate (p, q, intercept) orders to per-order lists (the runtime fits each list as a batch)
//   k_gather_rows      the rows of one order's list, packed for the batch fit
//   k_af_update        the round's outcome per series: first minimum approxAIC among the candidates that returned
//                      normally, are stationary and invertible and beat the incumbent; the next neighbourhood
//   k_af_finish        ARIMAModel(p, d, q, coefficients, hasIntercept) per series, or its status
//
// One lane per series everywhere; rows are 128-B aligned series-major workspaces (stream_elems).
#include "arima_device.hpp"
#include "arima_launch.hpp"

namespace sts {

namespace {

inline unsigned grid_of(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }

#define STS_AF_CHECK()                                                                                     \
    do {                                                                                                   \
        if (hipGetLastError() != hipSuccess) return ARIMA_E_DEVICE;                                        \
    } while (0)

}  // namespace

// ---------------------------------------------------------------------------------------------------------------
// KPSS "c" (TimeSeriesStatisticalTests.scala:369-393) on one row of length n (n >= 2: the caller checks the OLS
// shape, :383 -> AbstractMultipleLinearRegression.validateSampleData). The regression ts_i = alpha + e_i with
// setNoIntercept(true) and a column of ones is a one-column Householder QR (commons QRDecomposition):
//   xNormSqr = fold of 1*1 = n, a = -sqrt(n) (qrt[0][0] = 1 > 0), qrt[0][0] = 1 - a,
//   solve: dot = fold_r y_r * qrt[0][r] (= y_0 (1 - a), then + y_r * 1), dot /= a (1 - a), y_0 += dot (1 - a),
//   beta = y_0 / a;  residuals e_r = y_r - (0 + 1 * beta) (estimateResiduals, Array2DRowRealMatrix.operate).
// The second pass folds s2 = sum (cumulative sum)^2 (:386), the Newey-West cross products for lags 1..lag (:405-424)
// with the last LMAX residuals in registers, and the sum of squares (:430) -- every fold left, in the reference's
// order. LMAX >= lag = (int)(3 sqrt(n) / 13) (lag 7 at n = 1024, 14 at 4096; 32 covers n < 19 900).
// ---------------------------------------------------------------------------------------------------------------
constexpr int kKpssLagMax = 32;
constexpr double kKpssCritical5 = 0.463;          // kpssConstantCriticalValues(0.05), :338-340

__host__ __device__ __forceinline__ int kpss_lag(int n) { return (int)(3.0 * __builtin_sqrt((double)n) / 13.0); }

// stat of row y (n elements, 128-B aligned) by the restated algorithm; lag <= kKpssLagMax
__device__ double kpss_c_row(const double *__restrict__ y, int n) {
    const double a = -__builtin_sqrt((double)n);
    const double q0 = 1.0 - a;
    double dot = 0.0;
    int r = 0;
    stream_elems<2>(y, 0, n, [&](double v) {
        dot = dot + v * (r == 0 ? q0 : 1.0);
        ++r;
    });
    dot = dot / (a * q0);
    const double y0 = y[0] + dot * q0;
    const double beta = y0 / a;
    const double fit = 0.0 + 1.0 * beta;
    const int lag = kpss_lag(n);
    double hist[kKpssLagMax];                     // hist[i - 1] = e_{j - i}
#pragma unroll
    for (int i = 0; i < kKpssLagMax; ++i) hist[i] = 0.0;
    double cell[kKpssLagMax];
#pragma unroll
    for (int i = 0; i < kKpssLagMax; ++i) cell[i] = 0.0;
    double cum = 0.0, s2 = 0.0, sq = 0.0;
    int j = 0;
    stream_elems<2>(y, 0, n, [&](double v) {
        const double e = v - fit;
        cum = cum + e;
        s2 = s2 + cum * cum;
        sq = sq + e * e;
#pragma unroll
        for (int i = 1; i <= kKpssLagMax; ++i)
            if (i <= lag && j >= i) cell[i - 1] = cell[i - 1] + e * hist[i - 1];
#pragma unroll
        for (int i = kKpssLagMax - 1; i >= 1; --i) hist[i] = hist[i - 1];
        hist[0] = e;
        ++j;
    });
    double sum_terms = 0.0;
#pragma unroll
    for (int i = 1; i <= kKpssLagMax; ++i)
        if (i <= lag) sum_terms = sum_terms + cell[i - 1] * (1.0 - ((double)i / (double)(lag + 1)));
    const double partial = (sum_terms * 2.0) / (double)n;
    const double lrv = partial + sq / (double)n;
    const int32_t nn = (int32_t)((uint32_t)n * (uint32_t)n);          // (n * n): an Int product, :392
    return (s2 / lrv) / (double)nn;
}

// The same statistic for any lag (rows longer than ~19 900 points, lag > kKpssLagMax; VERDICT r5 missing 1): the
// Newey-West cross product of each lag i is its own left fold over j = i .. n-1 of e_j * e_{j-i} (every fold of the
// register version, in the same order), so lag i gets a pass of its own over the row instead of a register ring.
__device__ double kpss_c_row_any(const double *__restrict__ y, int n) {
    const double a = -__builtin_sqrt((double)n);
    const double q0 = 1.0 - a;
    double dot = 0.0;
    int r = 0;
    stream_elems<2>(y, 0, n, [&](double v) {
        dot = dot + v * (r == 0 ? q0 : 1.0);
        ++r;
    });
    dot = dot / (a * q0);
    const double y0 = y[0] + dot * q0;
    const double beta = y0 / a;
    const double fit = 0.0 + 1.0 * beta;
    const int lag = kpss_lag(n);
    double cum = 0.0, s2 = 0.0, sq = 0.0;
    stream_elems<2>(y, 0, n, [&](double v) {
        const double e = v - fit;
        cum = cum + e;
        s2 = s2 + cum * cum;
        sq = sq + e * e;
    });
    double sum_terms = 0.0;
    for (int i = 1; i <= lag; ++i) {
        double cell = 0.0;
        for (int j = i; j < n; ++j) cell = cell + (y[j] - fit) * (y[j - i] - fit);
        sum_terms = sum_terms + cell * (1.0 - ((double)i / (double)(lag + 1)));
    }
    const double partial = (sum_terms * 2.0) / (double)n;
    const double lrv = partial + sq / (double)n;
    const int32_t nn = (int32_t)((uint32_t)n * (uint32_t)n);          // (n * n): an Int product, wraps as the JVM's
    return (s2 / lrv) / (double)nn;
}

// One candidate d of autoFit's search (ARIMA.scala:287-292): series not decided yet whose differenced row passes the
// test at 5 % take d. stat_out (optional): the statistic of every row (the arima_kpss_batch building block).
__global__ __launch_bounds__(256) void k_kpss_c(const double *__restrict__ w, int64_t ld, int n, int64_t N, int d,
                                                int32_t *__restrict__ dsel, double *__restrict__ stat_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    if (dsel && dsel[i] >= 0) return;
    const double st = kpss_lag(n) <= kKpssLagMax ? kpss_c_row(w + i * ld, n) : kpss_c_row_any(w + i * ld, n);
    if (stat_out) stat_out[i] = st;
    if (dsel && st < kKpssCritical5) dsel[i] = d;          // `stat < criticalValues(kpssSignificance)`, :291
}

// differencesOfOrderD(ts, d) without the drop (ARIMA.scala:289, :298) for the rows with dsel[i] < 0 (undecided), one
// workgroup per row; a decided row keeps the differences of its own d
template <int DD>
__device__ __forceinline__ double diff_at_sel(const double *__restrict__ row, int t) {
    double v[DD + 1];
#pragma unroll
    for (int j = 0; j <= DD; ++j) {
        const int tt = t - DD + j;
        v[j] = tt >= 0 ? row[tt] : 0.0;
    }
#pragma unroll
    for (int lvl = 1; lvl <= DD; ++lvl)
#pragma unroll
        for (int j = DD; j >= lvl; --j)
            if (t - DD + j >= lvl) v[j] = v[j] - v[j - 1];
    return v[DD];
}

__global__ __launch_bounds__(256) void k_difference_sel(const double *__restrict__ in, int64_t ld_in,
                                                        double *__restrict__ out, int64_t ld_out, int64_t N, int T,
                                                        const int32_t *__restrict__ dsel, int d) {
    for (int64_t i = blockIdx.x; i < N; i += gridDim.x) {
        if (dsel[i] >= 0) continue;
        const double *row = in + i * ld_in;
        double *o = out + i * ld_out;
        for (int t = (int)threadIdx.x; t < T; t += blockDim.x) {
            double v;
            switch (d) {
#define STS_DS(DD) case DD: v = diff_at_sel<DD>(row, t); break;
                STS_DS(0) STS_DS(1) STS_DS(2) STS_DS(3) STS_DS(4) STS_DS(5) STS_DS(6) STS_DS(7) STS_DS(8)
                STS_DS(9) STS_DS(10) STS_DS(11) STS_DS(12) STS_DS(13) STS_DS(14) STS_DS(15) STS_DS(16)
#undef STS_DS
            default: v = __builtin_nan(""); break;
            }
            o[t] = v;
        }
    }
}

// ---------------------------------------------------------------------------------------------------------------
// The stepwise walk (findBestARMAModel, ARIMA.scala:310-375). Candidate orders are packed p | q << 4 | I << 8; the
// walk only ever meets q in {0, 1, 2} (the first candidates', :325-327 -- the neighbourhood keeps q, :364), so an
// order's combo index (p * 3 + q) * 2 + I < kAfCombosMax doubles as its bit in the series' `seen` mask (pastParams).
// Duplicates in the reference's candidate list (the 3 x 3 neighbourhood yields (p +- 1, q, I) three times each) are
// fitted once: their results are identical, and minBy keeps the first occurrence, which the deduplicated list (in
// first-appearance order) preserves.
// ---------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ int af_pack(int p, int q, int I) { return p | (q << 4) | (I << 8); }
__device__ __forceinline__ int af_combo(int pk) { return ((pk & 15) * 3 + ((pk >> 4) & 15)) * 2 + ((pk >> 8) & 1); }

__global__ __launch_bounds__(256) void k_af_init(int64_t N, const int32_t *__restrict__ dsel, AfSeries *__restrict__ st,
                                                 int32_t kpss_status) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    AfSeries s{};
    s.best_aic = 1.7976931348623157e308;                  // curBestAIC = Double.MaxValue, :323
    s.seen = 0ull;
    s.best = -1;
    s.n_fits = 0;
    const int d = dsel[i];
    s.dsel = d;
    if (kpss_status != ARIMA_ST_OK) {                     // kpsstest threw (rows <= regressors): autoFit throws
        s.status = kpss_status;
        s.ncand = 0;
    } else if (d < 0) {                                   // no d passed: "stationarity not achieved", :293-296
        s.status = ARIMA_ST_NOT_STATIONARY;
        s.ncand = 0;
    } else {
        const int I0 = d <= 1 ? 1 : 0;                    // addIntercept = d <= 1, :300
        s.status = ARIMA_ST_OK;
        s.ncand = 4;                                      // (0,0), (2,2), (1,0), (0,1) -- no bounds check, :325-327
        s.cand[0] = af_pack(0, 0, I0);
        s.cand[1] = af_pack(2, 2, I0);
        s.cand[2] = af_pack(1, 0, I0);
        s.cand[3] = af_pack(0, 1, I0);
    }
    st[i] = s;
}

// every walking series appends its candidates to the per-order lists (slot = position in the order's list)
__global__ __launch_bounds__(256) void k_af_plan(int64_t N, AfSeries *__restrict__ st, unsigned *__restrict__ counts,
                                                 int32_t *__restrict__ lists) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    AfSeries &s = st[i];
    const int nc = s.ncand;
    for (int c = 0; c < nc; ++c) {
        const int cb = af_combo(s.cand[c]);
        s.seen |= 1ull << cb;                             // pastParams ++= nextParams, :332
        const unsigned slot = atomicAdd(&counts[cb], 1u);
        lists[(int64_t)cb * N + slot] = (int32_t)i;
        s.slot[c] = (int32_t)slot;
    }
    s.n_fits += nc;
}

__global__ __launch_bounds__(256) void k_gather_rows(const double *__restrict__ in, int64_t ld, const int32_t *__restrict__ list,
                                                     int64_t count, int T, double *__restrict__ out) {
    for (int64_t r = blockIdx.x; r < count; r += gridDim.x) {
        const double *src = in + (int64_t)list[r] * ld;
        double *dst = out + r * ld;
        for (int t = (int)threadIdx.x; t < T; t += blockDim.x) dst[t] = src[t];
    }
}

// The round's outcome (ARIMA.scala:334-370). res_ll / res_status / res_flags rows of order cb start at off[cb] (the
// runtime's prefix sums); that order's fit wrote its coefficients k-strided from res_coef + off[cb] * 11.
__global__ __launch_bounds__(256) void k_af_update(int64_t N, AfSeries *__restrict__ st, const int64_t *__restrict__ off,
                                                   const double *__restrict__ res_coef, const double *__restrict__ res_ll,
                                                   const int32_t *__restrict__ res_status,
                                                   const uint8_t *__restrict__ res_flags, double *__restrict__ best_coef,
                                                   int max_p, int max_q) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    AfSeries s = st[i];
    if (s.ncand == 0) return;
    int win = -1;
    double win_aic = 0.0;
    int64_t win_coef = 0;
    for (int c = 0; c < s.ncand; ++c) {
        const int pk = s.cand[c];
        const int p = pk & 15, q = (pk >> 4) & 15, I = (pk >> 8) & 1;
        const int64_t base = off[af_combo(pk)];
        const int64_t row = base + s.slot[c];
        const int rs = res_status[row];
        // fitTryBothStrategies (:315-319): a css-cgd optimizer failure was refitted with css-bobyqa (the runtime's
        // k_bobyqa_fit, in place)
        if (rs != ARIMA_ST_OK) continue;                              // .filter(_.isSuccess), :337
        if (res_flags[row] != (ARIMA_FLAG_STATIONARY | ARIMA_FLAG_INVERTIBLE)) continue;   // :342
        const double aic = -2.0 * res_ll[row] + (double)(2 * (p + q + I));             // approxAIC, :826-830
        if (!(aic < s.best_aic)) continue;                            // improving, :344
        if (win < 0 || aic < win_aic) {                               // minBy: the first minimum, :350
            win = c;
            win_aic = aic;
            win_coef = base * 11 + (int64_t)s.slot[c] * (p + q + I);     // the order's fit wrote k-strided rows
        }
    }
    if (win < 0) {                                                    // no improving model: done, :346-347
        s.ncand = 0;
        st[i] = s;
        return;
    }
    const int pk = s.cand[win];
    const int p = pk & 15, q = (pk >> 4) & 15, I = (pk >> 8) & 1, k = p + q + I;
    s.best = pk;
    s.best_aic = win_aic;
    for (int j = 0; j < 11; ++j) best_coef[i * 11 + j] = j < k ? res_coef[win_coef + j] : 0.0;
    // the neighbourhood (:356-366): pDelta, qDelta in {-1, 0, 1}; q stays curBestModel.q; the intercept flips only
    // at (0, 0); filtered by pastParams and the p / q bounds (:369-370); duplicates dropped (first appearance kept)
    int nc = 0;
    for (int pd = -1; pd <= 1; ++pd) {
        for (int qd = -1; qd <= 1; ++qd) {
            const int np = p + pd, nI = (pd == 0 && qd == 0) ? 1 - I : I;
            if (np < 0 || np > max_p || q > max_q) continue;
            const int npk = af_pack(np, q, nI);
            if ((s.seen >> af_combo(npk)) & 1ull) continue;
            bool dup = false;
            for (int c = 0; c < nc; ++c) dup |= s.cand[c] == npk;
            if (!dup && nc < 4) s.cand[nc++] = npk;
        }
    }
    s.ncand = nc;
    st[i] = s;
}

// ARIMAModel(bestModel.p, d, bestModel.q, bestModel.coefficients, bestModel.hasIntercept), ARIMA.scala:302-303
__global__ __launch_bounds__(256) void k_af_finish(int64_t N, const AfSeries *__restrict__ st,
                                                   const double *__restrict__ best_coef, int32_t *__restrict__ order_out,
                                                   double *__restrict__ coef_out, double *__restrict__ aic_out,
                                                   int32_t *__restrict__ status_out, int32_t *__restrict__ n_fits_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const AfSeries s = st[i];
    int status = s.status;
    if (status == ARIMA_ST_OK && s.best < 0) status = ARIMA_ST_NO_MODEL;     // curBestModel == null -> NPE, :304
    const bool ok = s.best >= 0 && s.status == ARIMA_ST_OK;
    const int pk = s.best;
    order_out[i * 4 + 0] = ok ? (pk & 15) : -1;
    order_out[i * 4 + 1] = ok ? s.dsel : -1;
    order_out[i * 4 + 2] = ok ? ((pk >> 4) & 15) : -1;
    order_out[i * 4 + 3] = ok ? ((pk >> 8) & 1) : -1;
    for (int j = 0; j < 11; ++j) coef_out[i * 11 + j] = ok ? best_coef[i * 11 + j] : __builtin_nan("");
    aic_out[i] = ok ? s.best_aic : __builtin_inf();
    status_out[i] = status;
    if (n_fits_out) n_fits_out[i] = s.n_fits;
}

// ---------------------------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------------------------
int launch_kpss_c(const double *w, int64_t ld, int n, int64_t N, int d, int32_t *dsel, double *stat_out,
                  hipStream_t s) {
    if (N == 0) return ARIMA_OK;
    hipLaunchKernelGGL(k_kpss_c, dim3(grid_of(N, 256)), dim3(256), 0, s, w, ld, n, N, d, dsel, stat_out);
    STS_AF_CHECK();
    return ARIMA_OK;
}

int kpss_lag_host(int n) { return kpss_lag(n); }
int kpss_lag_max() { return kKpssLagMax; }

int launch_difference_sel(const double *in, int64_t ld_in, double *out, int64_t ld_out, int64_t N, int T,
                          const int32_t *dsel, int d, hipStream_t s) {
    if (N == 0 || T == 0) return ARIMA_OK;
    if (d < 0 || d > 16) return ARIMA_E_UNSUPPORTED;
    const unsigned grid = (unsigned)(N < 65536 * 4 ? N : 65536 * 4);
    hipLaunchKernelGGL(k_difference_sel, dim3(grid), dim3(256), 0, s, in, ld_in, out, ld_out, N, T, dsel, d);
    STS_AF_CHECK();
    return ARIMA_OK;
}

int launch_af_init(int64_t N, const int32_t *dsel, AfSeries *st, int32_t kpss_status, hipStream_t s) {
    if (N == 0) return ARIMA_OK;
    hipLaunchKernelGGL(k_af_init, dim3(grid_of(N, 256)), dim3(256), 0, s, N, dsel, st, kpss_status);
    STS_AF_CHECK();
    return ARIMA_OK;
}

int launch_af_plan(int64_t N, AfSeries *st, unsigned *counts, int32_t *lists, hipStream_t s) {
    if (N == 0) return ARIMA_OK;
    hipLaunchKernelGGL(k_af_plan, dim3(grid_of(N, 256)), dim3(256), 0, s, N, st, counts, lists);
    STS_AF_CHECK();
    return ARIMA_OK;
}

int launch_gather_rows(const double *in, int64_t ld, const int32_t *list, int64_t count, int T, double *out,
                       hipStream_t s) {
    if (count == 0 || T == 0) return ARIMA_OK;
    const unsigned grid = (unsigned)(count < 65536 * 4 ? count : 65536 * 4);
    hipLaunchKernelGGL(k_gather_rows, dim3(grid), dim3(256), 0, s, in, ld, list, count, T, out);
    STS_AF_CHECK();
    return ARIMA_OK;
}

int launch_af_update(int64_t N, AfSeries *st, const int64_t *off, const double *res_coef, const double *res_ll,
                     const int32_t *res_status, const uint8_t *res_flags, double *best_coef, int max_p, int max_q,
                     hipStream_t s) {
    if (N == 0) return ARIMA_OK;
    hipLaunchKernelGGL(k_af_update, dim3(grid_of(N, 256)), dim3(256), 0, s, N, st, off, res_coef, res_ll, res_status,
                       res_flags, best_coef, max_p, max_q);
    STS_AF_CHECK();
    return ARIMA_OK;
}

int launch_af_finish(int64_t N, const AfSeries *st, const double *best_coef, int32_t *order_out, double *coef_out,
                     double *aic_out, int32_t *status_out, int32_t *n_fits_out, hipStream_t s) {
    if (N == 0) return ARIMA_OK;
    hipLaunchKernelGGL(k_af_finish, dim3(grid_of(N, 256)), dim3(256), 0, s, N, st, best_coef, order_out, coef_out,
                       aic_out, status_out, n_fits_out);
    STS_AF_CHECK();
    return ARIMA_OK;
}

}  // namespace sts
