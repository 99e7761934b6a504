// arima_generic.hip — the runtime-order path: every building block of ARIMA.fitModel (ARIMA.scala:79-116) for the
// orders the compile-time kernels do not cover (p or q > 5, up to kGenMaxOrder), so a caller's ARIMA(7,1,2) or
// ARIMA(9,0,0) gets a fit instead of ARIMA_E_UNSUPPORTED (VERDICT r5 missing 1).
//
//   k_gen_hr_init     hannanRissanenInit (ARIMA.scala:216-242): two Householder least squares, commons QRDecomposition
//                     restated with runtime column counts (rows regenerated from the series, as arima_device.hpp's
//                     streamed QR does for compile-time orders -- same operations, same order)
//   k_gen_ar_fit      the AR-only shortcut (ARIMA.scala:90-96, Autoregression.scala:38-53)
//   k_gen_fit         fitWithCSSCGD (ARIMA.scala:174-200): one CGLane state machine per lane (cg_lane.hpp, with the
//                     restart period `iter % n` at the runtime parameter count), objective and gradient passes at
//                     runtime orders; no speculation (a pure shortcut: counts and results do not depend on it)
//   k_gen_css_loglik / k_gen_css_grad / k_gen_model_flags   the building blocks
//   k_gen_forecast    ARIMAModel.forecast (ARIMA.scala:696-764) for any order, the oracle's arrays in a global
//                     workspace (one slice of series at a time)
//
// One lane per series; the per-lane arrays (coefficients, the QR state, dEdTheta) are indexed at run time and live in
// private memory. This path is for correctness at orders the reference accepts and the fast kernels do not compile:
// it is not tuned.
#include <algorithm>

#include "arima_device.hpp"
#include "arima_launch.hpp"

namespace sts {

namespace {
inline unsigned gen_grid(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }
}  // namespace

#define STS_GEN_CHECK()                                                                                    \
    do {                                                                                                   \
        if (hipGetLastError() != hipSuccess) return ARIMA_E_DEVICE;                                        \
    } while (0)

// ---- gradientlogLikelihoodCSSARMA (ARIMA.scala:465-534) at runtime orders; returns the css at the same point ----
// dE: (rows x k) scratch, rows = 2 under the Breeze smear (every lag row holds the previous row 0) and
// q + 1 under the row-shift reading. g[0..k): the gradient, already divided by -sigma2 (:532).
__device__ double gen_grad(const GRow &r, int n, int p, int q, int I, const double *c, int smear, double *g,
                           double *dE) {
    const int k = I + p + q, M = p > q ? p : q;
    const int rows = smear ? (q > 0 ? 2 : 1) : q + 1;
    for (int j = 0; j < rows * k; ++j) dE[j] = 0.0;
    for (int j = 0; j < k; ++j) g[j] = 0.0;
    double e1 = 0.0, e2 = 0.0, sigma2 = 0.0, css = 0.0;
    const double nd = (double)n;
    const double yh0 = 0.0 + (double)I * c[0];
    for (int t = M; t < n; ++t) {
        for (int j = 0; j < k; ++j)                                                     // :492-499
            for (int kk = 0; kk < q; ++kk) dE[j] = dE[j] - c[I + p + kk] * dE[(smear ? 1 : kk + 1) * k + j];
        double yh = yh0;                                                                // :502
        if (k > 0) dE[0] = dE[0] - (double)I;                                           // :503
        for (int j = 0; j < p; ++j) {                                                   // :506-510
            const double v = r.at(t - 1 - j);
            yh = yh + v * c[I + j];
            dE[I + j] = dE[I + j] - v;
        }
        for (int j = 0; j < q; ++j) {                                                   // :514-518
            const double mj = (j == 0 ? e1 : e2);
            yh = yh + mj * c[I + p + j];
            dE[I + p + j] = dE[I + p + j] - mj;
        }
        const double e = r.at(t) - yh;                                                  // :520
        const double e_sq = e * e;
        sigma2 = sigma2 + e_sq / nd;                                                    // :521
        css = css + e_sq;
        e2 = e1;                                                                        // :522
        e1 = e;
        for (int j = 0; j < k; ++j) g[j] = g[j] + dE[j] * e;                            // :524
        if (smear) {                                                                    // :526, ascending element copy
            if (q > 0)
                for (int j = 0; j < k; ++j) dE[k + j] = dE[j];
        } else {                                                                        // :526, row shift
            for (int rr = q; rr >= 1; --rr)
                for (int j = 0; j < k; ++j) dE[rr * k + j] = dE[(rr - 1) * k + j];
        }
        for (int j = 0; j < k; ++j) dE[j] = 0.0;                                        // :528
    }
    for (int j = 0; j < k; ++j) g[j] = g[j] / -sigma2;                                  // :532
    return css;
}

// ---- commons-math3 OLSMultipleLinearRegression + QRDecomposition(threshold 0) at runtime column counts ----------
// The operations of arima_device.hpp's ols_stage / stream_ols in the same order, with every row regenerated by
// random access: stage s needs column s after reflections 0..s-1, so each row is rebuilt from the series and
// re-transformed (hh_apply). Row r: x[0..C), response y (RowGen::row).
struct GenQR {
    double a[kGenMaxK], vtop[kGenMaxK], dot[kGenMaxK];
    double alpha[kGenMaxK * kGenMaxK];            // alpha[s * C + c], c > s
};

__device__ __forceinline__ void gen_hh_apply(const GenQR &H, int C, int s, double *x, double &y) {
    for (int j = 0; j < s; ++j) {
        const double v = x[j];
        for (int c = j + 1; c < C; ++c) x[c] = x[c] - H.alpha[j * C + c] * v;
        y = y + H.dot[j] * v;
    }
}

template <class RowGen>
__device__ int gen_ols(const RowGen &gen, int R, int C, bool ones_first, GenQR &H, double *beta) {
    double x[kGenMaxK], xs[kGenMaxK], al[kGenMaxK];
    for (int S = 0; S < C; ++S) {
        double ys;
        gen.row(S, xs);
        ys = gen.resp(S);
        gen_hh_apply(H, C, S, xs, ys);
        const double xss = xs[S];
        double xnorm = 0.0 + xss * xss;
        if (S == 0 && ones_first) {
            xnorm = (double)R;                           // the intercept's ones: the sequential sum of R ones
        } else {
            for (int r = S + 1; r < R; ++r) {
                double y = gen.resp(r);
                gen.row(r, x);
                gen_hh_apply(H, C, S, x, y);
                xnorm = xnorm + x[S] * x[S];
            }
        }
        const double a = (xss > 0) ? -sqrt(xnorm) : sqrt(xnorm);
        H.a[S] = a;
        if (a == 0.0) return ARIMA_ST_SINGULAR;
        const double vt = xss - a;
        H.vtop[S] = vt;
        for (int c = 0; c < C; ++c) al[c] = (c > S) ? 0.0 - xs[c] * vt : 0.0;
        double dt = 0.0 + ys * vt;
        for (int r = S + 1; r < R; ++r) {
            double y = gen.resp(r);
            gen.row(r, x);
            gen_hh_apply(H, C, S, x, y);
            const double vs = x[S];
            for (int c = S + 1; c < C; ++c) al[c] = al[c] - x[c] * vs;
            dt = dt + y * vs;
        }
        const double den = a * vt;
        for (int c = 0; c < C; ++c) H.alpha[S * C + c] = (c > S) ? al[c] / den : 0.0;
        H.dot[S] = dt / den;
    }
    // rows 0..C-1 after their own reflection (the upper triangle of R, the top of Q^T y), then Solver.solve. Row i
    // reads reflections 0..i, so going from the last row down, row i of R can replace row i of alpha (no later
    // row reads it); every row's values are those of stream_ols's ascending loop.
    double ytop[kGenMaxK];
    for (int i = C - 1; i >= 0; --i) {
        double y = gen.resp(i);
        gen.row(i, x);
        gen_hh_apply(H, C, i, x, y);
        for (int c = i + 1; c < C; ++c) x[c] = x[c] - H.alpha[i * C + c] * H.vtop[i];
        y = y + H.dot[i] * H.vtop[i];
        for (int c = 0; c < C; ++c) H.alpha[i * C + c] = x[c];
        ytop[i] = y;
    }
    for (int r = C - 1; r >= 0; --r) {
        ytop[r] = ytop[r] / H.a[r];
        const double yRow = ytop[r];
        beta[r] = yRow;
        for (int i = 0; i < r; ++i) ytop[i] = ytop[i] - yRow * H.alpha[i * C + r];
    }
    return ARIMA_ST_OK;
}

// AR(m) rows (Autoregression.fitModel / Lag.lagMatTrimBoth): row r = [1?, y(r+m-1), ..., y(r)], response y(r+m)
struct GenARRows {
    GRow y;
    int m, I;
    __device__ __forceinline__ void row(int r, double *x) const {
        if (I) x[0] = 1.0;
        for (int l = 1; l <= m; ++l) x[I + l - 1] = y.at(r + m - l);
    }
    __device__ __forceinline__ double resp(int r) const { return y.at(r + m); }
};

// Hannan-Rissanen's second regression (ARIMA.scala:226-239): errors(s) = y(s+m) - ((sum_j y(s+m-1-j) a_j) + c),
// row r = [1?, y(m+r+M-1..m+r+M-p), errors(r+M-1..r+M-q)], response y(m+r+M)
struct GenHRRows {
    GRow y;
    int p, q, I, M, m;
    const double *a;                                     // [c, a_0 .. a_{m-1}] of the AR(m) stage
    __device__ __forceinline__ double err_at(int s) const {
        double acc = 0.0;
        for (int j = 0; j < m; ++j) acc = acc + y.at(s + m - 1 - j) * a[1 + j];
        return y.at(s + m) - (acc + a[0]);
    }
    __device__ __forceinline__ void row(int r, double *x) const {
        if (I) x[0] = 1.0;
        for (int l = 1; l <= p; ++l) x[I + l - 1] = y.at(m + r + M - l);
        for (int l = 1; l <= q; ++l) x[I + p + l - 1] = err_at(r + M - l);
    }
    __device__ __forceinline__ double resp(int r) const { return y.at(m + r + M); }
};

__device__ int gen_hannan_rissanen(const GRow &y, int n, int p, int q, int I, GenQR &H, double *beta) {
    int st = hr_shape_status(n, p, q, I);
    if (st != ARIMA_ST_OK) return st;
    const int M = p > q ? p : q, m = M + 1, K = I + p + q;
    double ab[kGenMaxK + 1];
    GenARRows ga{y, m, 1};
    st = gen_ols(ga, n - m, 1 + m, true, H, ab);                                        // :225
    if (st != ARIMA_ST_OK) return st;
    if (K == 0) return ARIMA_ST_OK;
    GenHRRows gb{y, p, q, I, M, m, ab};
    return gen_ols(gb, n - m - M, K, I != 0, H, beta);                                  // :237-240
}

// =======================================================================================================
// kernels
// =======================================================================================================
__global__ __launch_bounds__(64) void k_gen_hr_init(const double *__restrict__ y, int64_t ld, int n, int64_t N,
                                                    int p, int q, int I, double *__restrict__ init_out,
                                                    int32_t *__restrict__ status_out, int dd, FitPrep prep) {
    fit_prep(prep);
    const int K = I + p + q;
    for (int64_t sid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; sid < N;
         sid += (int64_t)gridDim.x * blockDim.x) {
        GenQR H;
        double beta[kGenMaxK];
        const GRow row{y + sid * ld, dd};
        const int st = gen_hannan_rissanen(row, n, p, q, I, H, beta);
        for (int j = 0; j < K; ++j) init_out[sid * K + j] = st == ARIMA_ST_OK ? beta[j] : __builtin_nan("");
        status_out[sid] = st;
    }
}

__global__ __launch_bounds__(64) void k_gen_ar_fit(const double *__restrict__ y, int64_t ld, int n, int64_t N, int p,
                                                   int I, double *__restrict__ coef_out, double *__restrict__ ll_out,
                                                   int32_t *__restrict__ status_out, int32_t *__restrict__ n_eval_out,
                                                   int32_t *__restrict__ n_grad_out, uint8_t *__restrict__ flags_out,
                                                   int dd) {
    const int K = I + p;
    for (int64_t sid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; sid < N;
         sid += (int64_t)gridDim.x * blockDim.x) {
        const GRow row{y + sid * ld, dd};
        int st = ar_shape_status(n, p, I);
        double beta[kGenMaxK];
        double ll = __builtin_nan("");
        uint8_t fl = 0;
        if (st == ARIMA_ST_OK) {
            GenQR H;
            GenARRows ga{row, p, I};
            st = gen_ols(ga, n - p, K, I != 0, H, beta);
            if (st == ARIMA_ST_OK) {
                double c[kGenMaxK];
                for (int j = 0; j < kGenMaxK; ++j) c[j] = j < K ? beta[j] : 0.0;
                ll = css_to_loglik(gen_css(row, n, p, 0, I, c), n);
                fl = gen_model_flags(c, p, 0, I);
            }
        }
        for (int j = 0; j < K; ++j) coef_out[sid * K + j] = st == ARIMA_ST_OK ? beta[j] : __builtin_nan("");
        ll_out[sid] = st == ARIMA_ST_OK ? ll : __builtin_nan("");
        status_out[sid] = st;
        if (n_eval_out) n_eval_out[sid] = 0;
        if (n_grad_out) n_grad_out[sid] = 0;
        if (flags_out) flags_out[sid] = st == ARIMA_ST_OK ? fl : 0;
    }
}

// fitWithCSSCGD per lane: the state machine posts objective (F) or gradient (G) requests; the lane serves each with
// one pass over its own row. Counters for arima_get_last_stats go to the fit-kernel words the runtime reads (ctl[1]
// F passes, ctl[2] G passes, ctl[5] evaluations, ctl[6] gradients, ctl[32] series written).
__global__ __launch_bounds__(64) void k_gen_fit(const double *__restrict__ y, int64_t ld, int n, int64_t N, int p,
                                                int q, int I, int smear, const double *__restrict__ init,
                                                const int32_t *__restrict__ init_status, double *__restrict__ coef_out,
                                                double *__restrict__ ll_out, int32_t *__restrict__ status_out,
                                                int32_t *__restrict__ n_eval_out, int32_t *__restrict__ n_grad_out,
                                                uint8_t *__restrict__ flags_out, unsigned long long *__restrict__ ctl,
                                                int dd) {
    const int K = I + p + q;
    unsigned long long nf = 0, ng = 0, ne = 0, ngr = 0, done = 0;
    for (int64_t sid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; sid < N;
         sid += (int64_t)gridDim.x * blockDim.x) {
        const int st0 = init_status ? init_status[sid] : ARIMA_ST_OK;
        if (st0 != ARIMA_ST_OK) {
            for (int j = 0; j < K; ++j) coef_out[sid * K + j] = __builtin_nan("");
            ll_out[sid] = __builtin_nan("");
            status_out[sid] = st0;
            if (n_eval_out) n_eval_out[sid] = 0;
            if (n_grad_out) n_grad_out[sid] = 0;
            if (flags_out) flags_out[sid] = 0;
            ++done;
            continue;
        }
        const GRow row{y + sid * ld, dd};
        GenLane L;
        L.kdim = K;
        double x0[kGenMaxK];
        for (int j = 0; j < kGenMaxK; ++j) x0[j] = j < K ? init[sid * K + j] : 0.0;
        L.start_posted(x0);
        double g[kGenMaxK], c[kGenMaxK], dE[(kGenMaxOrder + 1) * kGenMaxK];
        for (int j = 0; j < kGenMaxK; ++j) g[j] = 0.0;
        while (!L.done()) {
            const int req = L.req;
            if (req == REQ_NONE) {                      // the machine always posts a request or finishes
                L.fail(ARIMA_ST_MAX_EVAL);
                break;
            }
            L.request_point(c);
            double css;
            if (req == REQ_G) {
                css = gen_grad(row, n, p, q, I, c, smear, g, dE);
                ++ng;
            } else {
                css = gen_css(row, n, p, q, I, c);
                ++nf;
            }
            L.req = REQ_NONE;
            L.advance(css_to_loglik(css, n), g);
        }
        const bool ok = L.status == ARIMA_ST_OK;
        for (int j = 0; j < K; ++j) coef_out[sid * K + j] = ok ? L.point[j] : __builtin_nan("");
        ll_out[sid] = ok ? L.prev_obj : __builtin_nan("");
        status_out[sid] = L.status;
        if (n_eval_out) n_eval_out[sid] = L.n_eval;
        if (n_grad_out) n_grad_out[sid] = L.n_grad;
        if (flags_out) flags_out[sid] = ok ? gen_model_flags(L.point, p, q, I) : 0;
        ne += L.n_eval;
        ngr += L.n_grad;
        ++done;
    }
    if (ctl) {
        atomicAdd(&ctl[1], nf);
        atomicAdd(&ctl[2], ng);
        atomicAdd(&ctl[5], ne);
        atomicAdd(&ctl[6], ngr);
        atomicAdd(&ctl[32], done);
    }
}

__global__ __launch_bounds__(64) void k_gen_css_loglik(const double *__restrict__ y, int64_t ld, int n, int64_t N,
                                                       int p, int q, int I, const double *__restrict__ coef,
                                                       double *__restrict__ ll_out) {
    const int K = I + p + q;
    const int64_t sid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sid >= N) return;
    double c[kGenMaxK];
    for (int j = 0; j < kGenMaxK; ++j) c[j] = j < K ? coef[sid * K + j] : 0.0;
    ll_out[sid] = css_to_loglik(gen_css(GRow{y + sid * ld, 0}, n, p, q, I, c), n);
}

__global__ __launch_bounds__(64) void k_gen_css_grad(const double *__restrict__ y, int64_t ld, int n, int64_t N,
                                                     int p, int q, int I, int smear, const double *__restrict__ coef,
                                                     double *__restrict__ g_out) {
    const int K = I + p + q;
    const int64_t sid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sid >= N) return;
    double c[kGenMaxK], g[kGenMaxK], dE[(kGenMaxOrder + 1) * kGenMaxK];
    for (int j = 0; j < kGenMaxK; ++j) c[j] = j < K ? coef[sid * K + j] : 0.0;
    gen_grad(GRow{y + sid * ld, 0}, n, p, q, I, c, smear, g, dE);
    for (int j = 0; j < K; ++j) g_out[sid * K + j] = g[j];
}

__global__ __launch_bounds__(64) void k_gen_model_flags(const double *__restrict__ coef, int64_t N, int p, int q,
                                                        int I, uint8_t *__restrict__ flags_out) {
    const int K = I + p + q;
    const int64_t sid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sid >= N) return;
    double c[kGenMaxK];
    for (int j = 0; j < kGenMaxK; ++j) c[j] = j < K ? coef[sid * K + j] : 0.0;
    flags_out[sid] = gen_model_flags(c, p, q, I);
}

// ---- ARIMAModel.forecast (ARIMA.scala:696-764) at any order, restated array by array as the oracle does ----------
// differencesOfOrderD (UnivariateTimeSeries.scala:468-480): d passes of differencesAtLag(lag 1, start i), ping-pong
__device__ void gen_diff_d(const double *ts, int T, int d, double *out, double *tmp) {
    for (int t = 0; t < T; ++t) out[t] = ts[t];
    for (int i = 1; i <= d; ++i) {
        for (int t = 0; t < T; ++t) tmp[t] = out[t];
        for (int t = 0; t < T; ++t) out[t] = (t < i) ? tmp[t] : tmp[t] - tmp[t - 1];
    }
}

__device__ __forceinline__ void gen_update_ma(double *errs, int len, double e) {
    for (int i = 0; i < len - 1; ++i) errs[i + 1] = errs[i];
    if (len > 0) errs[0] = e;
}

// workspace per series (doubles): gen_forecast_ws(T, d, M, nF)
__host__ __device__ __forceinline__ int64_t gen_forecast_ws(int T, int d, int M, int nF) {
    const int64_t n = T - d, histLen = M + n, fl = nF + M;
    return 2 * (int64_t)(T + 1) + 2 * (histLen + 1) + (fl + 1) + (int64_t)(d + 1) * T + 2 * (int64_t)(d + nF + 1);
}

__global__ __launch_bounds__(64) void k_gen_forecast(const double *__restrict__ ts_all, int64_t ld_in,
                                                     const double *__restrict__ coef_all, int k,
                                                     double *__restrict__ out_all, int64_t ld_out, int64_t N, int T,
                                                     int p, int d, int q, int I, int nF, double *__restrict__ ws_all,
                                                     int64_t ws_stride) {
    const int64_t sid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sid >= N) return;
    const double *ts = ts_all + sid * ld_in;
    const double *coef = coef_all + sid * k;
    double *out = out_all + sid * ld_out;
    double *w = ws_all + sid * ws_stride;
    const int M = p > q ? p : q;
    const int n = T - d, histLen = M + n, fl = nF + M, L = T + nF;
    double *dts = w;                  w += T + 1;
    double *tmp = w;                  w += T + 1;
    double *ext = w;                  w += histLen + 1;
    double *hist = w;                 w += histLen + 1;
    double *fwd = w;                  w += fl + 1;
    double *dm = w;                   w += (int64_t)(d + 1) * T;
    double *fi = w;                   w += d + nF + 1;
    double *fo = w;
    double c[kGenMaxK];
    for (int j = 0; j < kGenMaxK; ++j) c[j] = j < k ? coef[j] : 0.0;
    gen_diff_d(ts, T, d, dts, tmp);                                                     // :700
    const double intercept_amt = I ? c[0] : 0.0;
    for (int i = 0; i < M; ++i) ext[i] = intercept_amt;                                 // :703-707
    for (int i = 0; i < n; ++i) ext[M + i] = dts[d + i];
    for (int i = 0; i < histLen; ++i) hist[i] = 0.0;
    {                                                                                   // iterateARMA(ext, hist, +, gold = ext) :708
        double ma[kGenMaxOrder];
        for (int j = 0; j < q; ++j) ma[j] = 0.0;
        for (int i = M; i < histLen; ++i) {
            double t = (double)I * c[0];
            hist[i] = hist[i] + t;
            for (int j = 0; j < p && i - j - 1 >= 0; ++j) hist[i] = hist[i] + ext[i - j - 1] * c[I + j];
            for (int j = 0; j < q; ++j) hist[i] = hist[i] + ma[j] * c[I + p + j];
            gen_update_ma(ma, q, ext[i] - hist[i]);
        }
    }
    double maTerms[kGenMaxOrder];
    for (int i = histLen - M, j = 0; i < histLen; ++i, ++j) maTerms[j] = ext[i] - hist[i];   // :711-713
    for (int i = 0; i < fl; ++i) fwd[i] = 0.0;
    for (int i = 0; i < M; ++i) fwd[i] = hist[histLen - M + i];                        // :717
    for (int i = M; i < fl; ++i) {                                                      // :720, maTerms of length M
        const double t = (double)I * c[0];
        fwd[i] = fwd[i] + t;
        for (int j = 0; j < p && i - j - 1 >= 0; ++j) fwd[i] = fwd[i] + fwd[i - j - 1] * c[I + j];
        for (int j = 0; j < q; ++j) fwd[i] = fwd[i] + maTerms[j] * c[I + p + j];
        gen_update_ma(maTerms, M, fwd[i] - fwd[i]);
    }
    for (int i = 0; i < L; ++i) out[i] = 0.0;
    for (int i = 0; i < d && i < T; ++i) out[i] = ts[i];                                // :724
    for (int i = 0; i < histLen - M; ++i) out[d + i] = hist[M + i];                     // :726
    for (int i = 0; i < nF; ++i) out[T + i] = fwd[M + i];                               // :728
    if (d != 0) {                                                                       // :730-762
        for (int t = 0; t < (d + 1) * T; ++t) dm[t] = 0.0;
        for (int t = 0; t < T; ++t) dm[t] = ts[t];
        for (int i = 1; i <= d; ++i) {
            const int len = T - i;
            if (len > 0) {                  // differencesOfOrderD(row i-1 from i, 1): first kept, then differences
                const double *src = dm + (int64_t)(i - 1) * T + i;
                double *dst = dm + (int64_t)i * T + i;
                for (int t = 0; t < len; ++t) tmp[t] = src[t];
                for (int t = 0; t < len; ++t) dst[t] = (t < 1) ? tmp[t] : tmp[t] - tmp[t - 1];
            }
        }
        for (int i = d; i < histLen - M; ++i) {                                         // :745-751
            double s = 0.0;
            for (int r = 0; r < d; ++r) s = s + dm[(int64_t)r * T + (i - 1)];
            out[i] = s + hist[M + i];
        }
        for (int r = 0; r < d; ++r) fi[r] = dm[(int64_t)r * T + (T - d + r)];
        for (int i = 0; i < nF; ++i) fi[d + i] = fwd[M + i];
        for (int j = 0; j < d + nF; ++j) fo[j] = fi[j];                                 // inverseDifferencesOfOrderD
        for (int lv = d; lv >= 1; --lv)
            for (int j = 0; j < d + nF; ++j) fo[j] = (j < lv) ? fo[j] : fo[j] + fo[j - 1];
        for (int i = 0; i < d + nF; ++i) out[L - (d + nF) + i] = fo[i];                 // :761
    }
}

// =======================================================================================================
// launchers (orders up to kGenMaxOrder; arima_launch.hpp)
// =======================================================================================================
bool gen_orders_ok(int p, int q) { return p >= 0 && q >= 0 && p <= kGenMaxOrder && q <= kGenMaxOrder; }

// fixed grids: one lane per series in single-wave workgroups, grid-stride (bounds the private memory in flight)
constexpr unsigned kGenGridMax = 4096;

int launch_gen_hr_init(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, double *init_out,
                       int32_t *status_out, int dd, const FitPrep &prep, hipStream_t s) {
    if (!gen_orders_ok(p, q)) return ARIMA_E_UNSUPPORTED;
    const unsigned grid = std::max(1u, std::min(gen_grid(N, 64), kGenGridMax));
    hipLaunchKernelGGL(k_gen_hr_init, dim3(grid), dim3(64), 0, s, y, ld, n, N, p, q, I, init_out, status_out, dd, prep);
    STS_GEN_CHECK();
    return ARIMA_OK;
}

int launch_gen_ar_fit(const double *y, int64_t ld, int n, int64_t N, int p, int I, double *coef_out, double *ll_out,
                      int32_t *status_out, int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out, int dd,
                      hipStream_t s) {
    if (!gen_orders_ok(p, 0)) return ARIMA_E_UNSUPPORTED;
    if (N == 0) return ARIMA_OK;
    const unsigned grid = std::min(gen_grid(N, 64), kGenGridMax);
    hipLaunchKernelGGL(k_gen_ar_fit, dim3(grid), dim3(64), 0, s, y, ld, n, N, p, I, coef_out, ll_out, status_out,
                       n_eval_out, n_grad_out, flags_out, dd);
    STS_GEN_CHECK();
    return ARIMA_OK;
}

int launch_gen_fit(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, int smear, const double *init,
                   const int32_t *init_status, double *coef_out, double *ll_out, int32_t *status_out,
                   int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out, unsigned long long *ctl, int dd,
                   hipStream_t s) {
    if (!gen_orders_ok(p, q)) return ARIMA_E_UNSUPPORTED;
    if (N == 0) return ARIMA_OK;
    const unsigned grid = std::min(gen_grid(N, 64), kGenGridMax);
    hipLaunchKernelGGL(k_gen_fit, dim3(grid), dim3(64), 0, s, y, ld, n, N, p, q, I, smear, init, init_status, coef_out,
                       ll_out, status_out, n_eval_out, n_grad_out, flags_out, ctl, dd);
    STS_GEN_CHECK();
    return ARIMA_OK;
}

int launch_gen_css_loglik(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, const double *coef,
                          double *ll_out, hipStream_t s) {
    if (!gen_orders_ok(p, q)) return ARIMA_E_UNSUPPORTED;
    if (N == 0) return ARIMA_OK;
    hipLaunchKernelGGL(k_gen_css_loglik, dim3(gen_grid(N, 64)), dim3(64), 0, s, y, ld, n, N, p, q, I, coef, ll_out);
    STS_GEN_CHECK();
    return ARIMA_OK;
}

int launch_gen_css_grad(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, int smear,
                        const double *coef, double *g_out, hipStream_t s) {
    if (!gen_orders_ok(p, q)) return ARIMA_E_UNSUPPORTED;
    if (N == 0) return ARIMA_OK;
    hipLaunchKernelGGL(k_gen_css_grad, dim3(gen_grid(N, 64)), dim3(64), 0, s, y, ld, n, N, p, q, I, smear, coef,
                       g_out);
    STS_GEN_CHECK();
    return ARIMA_OK;
}

int launch_gen_model_flags(const double *coef, int64_t N, int p, int q, int I, uint8_t *flags_out, hipStream_t s) {
    if (!gen_orders_ok(p, q)) return ARIMA_E_UNSUPPORTED;
    if (N == 0) return ARIMA_OK;
    hipLaunchKernelGGL(k_gen_model_flags, dim3(gen_grid(N, 64)), dim3(64), 0, s, coef, N, p, q, I, flags_out);
    STS_GEN_CHECK();
    return ARIMA_OK;
}

int64_t gen_forecast_ws_doubles(int T, int p, int d, int q, int n_future) {
    return gen_forecast_ws(T, d, p > q ? p : q, n_future);
}

int launch_gen_forecast(const double *ts, int64_t ld_in, const double *coef, int k, double *out, int64_t ld_out,
                        int64_t N, int T, int p, int d, int q, int I, int n_future, double *ws, int64_t ws_stride,
                        hipStream_t s) {
    if (!gen_orders_ok(p, q)) return ARIMA_E_UNSUPPORTED;
    if (N == 0) return ARIMA_OK;
    hipLaunchKernelGGL(k_gen_forecast, dim3(gen_grid(N, 64)), dim3(64), 0, s, ts, ld_in, coef, k, out, ld_out, N, T, p,
                       d, q, I, n_future, ws, ws_stride);
    STS_GEN_CHECK();
    return ARIMA_OK;
}

}  // namespace sts
