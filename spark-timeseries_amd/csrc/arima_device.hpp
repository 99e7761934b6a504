// arima_device.hpp — device-side algorithms of the MI355X batched ARIMA (CSS-CGD) engine.
//
// Everything here runs one series per lane (wave64 = 64 independent series). The arithmetic follows the
// reference operation by operation so that results are bit-identical to the CPU restatement in oracle/:
//   * every fp64 operation is a separate IEEE op: the library is compiled with -ffp-contract=off (Java never
//     fuses a*b+c), fp64 denormals are kept, division and sqrt are the correctly rounded AMDGPU expansions;
//   * `math.log` is fdlibm's __ieee754_log (the algorithm of java.lang.StrictMath.log), restated below;
//   * sums are folded left in the reference's order.
// Reference citations are relative to the spark-ts root (src/main/scala/com/cloudera/sparkts/...).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sparkts_arima.h"

namespace sts {

constexpr int kMaxEval = 10000;      // new MaxEval(10000)  ARIMA.scala:196
constexpr int kMaxIter = 10000;      // new MaxIter(10000)  ARIMA.scala:195
constexpr int kBracketMax = 500;     // commons BracketFinder() = BracketFinder(growLimit 100, maxEval 500)
constexpr int kChunk = 16;           // doubles per lane per streamed chunk (one 128-B line)


// ------------------------------------------------------------------------------------------------------
// fdlibm __ieee754_log (used by logLikelihoodCSSARMA, ARIMA.scala:444)
// ------------------------------------------------------------------------------------------------------
__device__ __forceinline__ double dlog(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                 two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
                 Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                 Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
                 Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
    int64_t bits = __double_as_longlong(x);
    int32_t hx = (int32_t)(bits >> 32);
    uint32_t lx = (uint32_t)bits;
    int32_t k = 0;
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | lx) == 0) return -two54 / 0.0;
        if (hx < 0) return (x - x) / 0.0;
        k -= 54;
        x *= two54;
        hx = (int32_t)(__double_as_longlong(x) >> 32);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    int32_t i = (hx + 0x95f64) & 0x100000;
    {
        uint64_t u = (uint64_t)__double_as_longlong(x);
        u = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (u & 0xffffffffull);
        x = __longlong_as_double((long long)u);
    }
    k += (i >> 20);
    double f = x - 1.0;
    double dk;
    if ((0x000fffff & (2 + hx)) < 3) {
        if (f == 0.0) {
            if (k == 0) return 0.0;
            dk = (double)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        double R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        dk = (double)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    double s = f / (2.0 + f);
    dk = (double)k;
    double z = s * s;
    i = hx - 0x6147a;
    double w = z * z;
    int32_t j = 0x6b851 - hx;
    double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    double R = t2 + t1;
    if (i > 0) {
        double hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// logLikelihoodCSSARMA tail: sigma2 = css / n; (-n/2 as Int) * log(2*pi*sigma2) - css / (2*sigma2)  (:443-444)
__device__ __forceinline__ double css_to_loglik(double css, int n) {
    double sigma2 = css / (double)n;
    return (double)(-n / 2) * dlog(2.0 * 3.141592653589793 * sigma2) - css / (2.0 * sigma2);
}

__device__ __forceinline__ bool finite(double v) { return __builtin_isfinite(v); }

// ------------------------------------------------------------------------------------------------------
// Per-lane streaming of one series row. Every lane walks its own row front to back, so a wave touches 64
// different 128-B lines per load instruction; each lane therefore fetches whole lines (8 x 16-B loads = one
// 128-B chunk) and keeps D chunks in flight in registers (chunk c+D is requested while chunk c is consumed).
// The unaligned head (up to the first 16-element boundary) and the tail use single loads, so the unrolled body
// has no guards.
// ------------------------------------------------------------------------------------------------------
struct Chunk {
    double v[kChunk];
};

__device__ __forceinline__ void load_chunk(const double *__restrict__ p, Chunk &out) {
    const double2 *q = reinterpret_cast<const double2 *>(p);
#pragma unroll
    for (int u = 0; u < kChunk / 2; ++u) {
        const double2 t = q[u];
        out.v[2 * u] = t.x;
        out.v[2 * u + 1] = t.y;
    }
}

// fn(row[i]) for i = first .. last-1, in order. `row` must be 128-B aligned and readable over the 128-B
// chunks that contain first .. last-1. Every chunk of the range is fetched whole; loads are UNCONDITIONAL
// (refills past the end re-read the last chunk, an L2 hit) so no control-flow join ever merges a load result
// (a join would force s_waitcnt vmcnt(0) and kill the prefetch). Only the first and the last chunk test the
// element range.
template <int D, class Fn>
__device__ __forceinline__ void stream_elems(const double *__restrict__ row, int first, int last, Fn &&fn) {
    if (first >= last) return;
    const int c_first = first / kChunk;
    const int c_last = (last - 1) / kChunk;
    const int nch = c_last - c_first + 1;
    const double *base = row + c_first * kChunk;
    Chunk ring[D];
#pragma unroll
    for (int j = 0; j < D; ++j) load_chunk(base + (j < nch ? j : nch - 1) * kChunk, ring[j]);
    const int head = first - c_first * kChunk;          // elements of chunk 0 before `first`
    const int tail = last - c_last * kChunk;            // elements of the last chunk that are in range
    for (int c0 = 0; c0 < nch; c0 += D) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const int ch = c0 + j;
            if (ch < nch) {
                const bool full = (ch > 0 || head == 0) && (ch < nch - 1 || tail == kChunk);
                if (full) {
#pragma unroll
                    for (int u = 0; u < kChunk; ++u) fn(ring[j].v[u]);
                } else {
                    const int lo = (ch == 0) ? head : 0;
                    const int hi = (ch == nch - 1) ? tail : kChunk;
#pragma unroll
                    for (int u = 0; u < kChunk; ++u)
                        if (u >= lo && u < hi) fn(ring[j].v[u]);
                }
            }
            const int nx = ch + D;
            load_chunk(base + (nx < nch ? nx : nch - 1) * kChunk, ring[j]);
        }
    }
}

// ------------------------------------------------------------------------------------------------------
// CSS pass (objective, and optionally gradient) over one series — ARIMA.scala:430-534
//
// Lanes hold the maTerms buffer as two registers: updateMAErrors (:544-554) copies errs(i) -> errs(i+1) in
// ASCENDING i, so after every update positions 1..q-1 all equal the previous errs(0): maTerms is
// [e_{t-1}, e_{t-2}, e_{t-2}, ...] (a smear for q >= 3, exactly what the reference computes).
// ------------------------------------------------------------------------------------------------------
#ifndef STS_PREFETCH_F
#define STS_PREFETCH_F 4
#endif
#ifndef STS_PREFETCH_G
#define STS_PREFETCH_G 2
#endif
constexpr int kPrefetchF = STS_PREFETCH_F;   // chunks in flight per lane in objective passes
constexpr int kPrefetchG = STS_PREFETCH_G;   // ... in gradient passes (5x the VALU work per byte)

// Full pass. G = false: objective only -> css. G = true: also gradientlogLikelihoodCSSARMA -> g[] (already
// divided by -sigma2, :532). SMEAR selects the Breeze overlap semantics of :526 (false = row shift).
template <int P, int Q, int I, bool G, bool SMEAR>
__device__ __forceinline__ void css_pass(const double *__restrict__ row, int n,
                                         const double (&c)[I + P + Q > 0 ? I + P + Q : 1], double &css_out,
                                         double (&g)[I + P + Q > 0 ? I + P + Q : 1]) {
    constexpr int K = I + P + Q;
    constexpr int KA = K > 0 ? K : 1;
    constexpr int M = (P > Q ? P : Q);
    constexpr int PA = P > 0 ? P : 1;
    double yl[PA];                        // yl[j] = y_{i-1-j}; the row is padded to >= 16 elements
#pragma unroll
    for (int j = 0; j < PA; ++j) yl[j] = (j < P) ? row[M - 1 - j] : 0.0;
    double e1 = 0.0, e2 = 0.0, css = 0.0, sigma2 = 0.0;
    const double yh0 = 0.0 + (double)I * c[0];
    const double nd = (double)n;
    double dE[G ? Q + 1 : 1][KA];         // dEdTheta (:476), row r = d e_{t-r} / d theta
    if constexpr (G) {
#pragma unroll
        for (int r = 0; r <= Q; ++r)
#pragma unroll
            for (int j = 0; j < KA; ++j) dE[r][j] = 0.0;
    }
#pragma unroll
    for (int j = 0; j < KA; ++j) g[j] = 0.0;

    auto step = [&](double yi) {
        if constexpr (!G) {
            double yh = yh0;                                          // 0.0 + intercept * coef(0)   (:600)
#pragma unroll
            for (int j = 0; j < P; ++j) yh = yh + yl[j] * c[I + j];   // AR terms, lag 1..p          (:602-605)
#pragma unroll
            for (int j = 0; j < Q; ++j) yh = yh + (j == 0 ? e1 : e2) * c[I + P + j];   // MA terms  (:608-611)
            const double e = yi - yh;                                 // goldStandard(i) - dest(i)  (:613)
            css = css + e * e;                                        // pow(obs - pred, 2), folded (:440-442)
            e2 = e1;
            e1 = e;
        } else {
#pragma unroll
            for (int j = 0; j < K; ++j)                               // :492-499
#pragma unroll
                for (int kk = 0; kk < Q; ++kk) dE[0][j] = dE[0][j] - c[I + P + kk] * dE[kk + 1][j];
            double yh = yh0;                                          // :502
            if constexpr (K > 0) dE[0][0] = dE[0][0] - (double)I;     // :503
#pragma unroll
            for (int j = 0; j < P; ++j) {                             // :506-510
                yh = yh + yl[j] * c[I + j];
                dE[0][I + j] = dE[0][I + j] - yl[j];
            }
#pragma unroll
            for (int j = 0; j < Q; ++j) {                             // :514-518
                const double mj = (j == 0 ? e1 : e2);
                yh = yh + mj * c[I + P + j];
                dE[0][I + P + j] = dE[0][I + P + j] - mj;
            }
            const double e = yi - yh;                                 // :520
            const double e_sq = e * e;
            sigma2 = sigma2 + e_sq / nd;                              // :521
            css = css + e_sq;                                         // objective at the same point (fused)
            e2 = e1;                                                  // :522
            e1 = e;
#pragma unroll
            for (int j = 0; j < K; ++j) g[j] = g[j] + dE[0][j] * e;   // :524
            if constexpr (SMEAR) {                                    // :526, ascending element copy
#pragma unroll
                for (int r = 1; r <= Q; ++r)
#pragma unroll
                    for (int j = 0; j < KA; ++j) dE[r][j] = dE[r - 1][j];
            } else {                                                  // :526, memmove-like row shift
#pragma unroll
                for (int r = Q; r >= 1; --r)
#pragma unroll
                    for (int j = 0; j < KA; ++j) dE[r][j] = dE[r - 1][j];
            }
#pragma unroll
            for (int j = 0; j < KA; ++j) dE[0][j] = 0.0;              // :528
        }
        if constexpr (P > 0) {
#pragma unroll
            for (int j = PA - 1; j >= 1; --j) yl[j] = yl[j - 1];
            yl[0] = yi;
        }
    };
    stream_elems<G ? kPrefetchG : kPrefetchF>(row, M, n, step);
    css_out = css;
    if constexpr (G) {
#pragma unroll
        for (int j = 0; j < KA; ++j) g[j] = g[j] / -sigma2;         // :532
    }
}

// Objective pass for NCH points at once (speculative line-search points): NCH independent recursions over the
// same streamed series. Each chain is exactly the single-point objective (same ops, same order).
template <int P, int Q, int I, int NCH>
__device__ __forceinline__ void css_pass_multi(const double *__restrict__ row, int n,
                                               const double (&c)[NCH][I + P + Q > 0 ? I + P + Q : 1],
                                               double (&css_out)[NCH]) {
    constexpr int M = (P > Q ? P : Q);
    constexpr int PA = P > 0 ? P : 1;
    double yl[PA];
#pragma unroll
    for (int j = 0; j < PA; ++j) yl[j] = (j < P) ? row[M - 1 - j] : 0.0;
    double e1[NCH], e2[NCH], css[NCH], yh0[NCH];
#pragma unroll
    for (int h = 0; h < NCH; ++h) {
        e1[h] = e2[h] = css[h] = 0.0;
        yh0[h] = 0.0 + (double)I * c[h][0];
    }
    auto step = [&](double yi) {
#pragma unroll
        for (int h = 0; h < NCH; ++h) {
            double yh = yh0[h];
#pragma unroll
            for (int j = 0; j < P; ++j) yh = yh + yl[j] * c[h][I + j];
#pragma unroll
            for (int j = 0; j < Q; ++j) yh = yh + (j == 0 ? e1[h] : e2[h]) * c[h][I + P + j];
            const double e = yi - yh;
            css[h] = css[h] + e * e;
            e2[h] = e1[h];
            e1[h] = e;
        }
        if constexpr (P > 0) {
#pragma unroll
            for (int j = PA - 1; j >= 1; --j) yl[j] = yl[j - 1];
            yl[0] = yi;
        }
    };
    stream_elems<kPrefetchF>(row, M, n, step);
#pragma unroll
    for (int h = 0; h < NCH; ++h) css_out[h] = css[h];
}

// ------------------------------------------------------------------------------------------------------
// Streaming Householder least squares, bit-identical to commons-math3 3.4.1
// OLSMultipleLinearRegression + QRDecomposition(threshold 0) without materialising the design matrix.
//
// Reflection s (QRDecomposition.performHouseholderReflection) needs column s after reflections 0..s-1, and
// each reflection updates a row independently of the other rows, so every row can be regenerated from the
// series and re-transformed by the already-known reflections (same ops, same order per element). Two passes
// per column: (1) xNormSqr -> rDiag[s] = a_s, v_s[s] = x_s[s] - a_s; (2) alpha_{s,c} for c > s and the
// Q^T y dot product of Solver.solve (which only needs reflection s). Row s itself (the only row whose v
// differs) is generated by random access; rows s+1.. are streamed. The upper triangle of R and the top of
// Q^T y come from re-transforming rows 0..C-1 once more. Back-substitution as Solver.solve.
//
// Gen provides: row_at(r, x, y) (random access), begin(r) (prime the sliding window for streaming from row r),
// first_elem(r) (series index of the element that completes row r), push(v, x, y) (next row from the next
// series element).
// ------------------------------------------------------------------------------------------------------
template <int C>
struct HouseholderState {
    double a[C];          // rDiag
    double vtop[C];       // qrt[s][s] after its own reflection
    double alpha[C][C];   // alpha[s][c], c > s (already divided by a_s * vtop_s)
    double dot[C];        // Q^T y coefficients (already divided by rDiag[s] * vtop_s)
};

// apply reflections 0..s-1 (in order) to a row x[] and response y
template <int C>
__device__ __forceinline__ void hh_apply(const HouseholderState<C> &H, int s, double (&x)[C], double &y) {
#pragma unroll
    for (int j = 0; j < C; ++j) {
        if (j < s) {
            const double v = x[j];
#pragma unroll
            for (int c = j + 1; c < C; ++c) x[c] = x[c] - H.alpha[j][c] * v;
            y = y + H.dot[j] * v;
        }
    }
}

// One Householder stage S (compile-time, so every reflection index below is a constant).
template <int C, int S, class Gen>
__device__ __forceinline__ int ols_stage(Gen &gen, const double *__restrict__ row, int n, int R,
                                         HouseholderState<C> &H) {
    if constexpr (S == C) {
        return ARIMA_ST_OK;
    } else {
        // pass 1: xNormSqr over rows S..R-1 of column S after reflections 0..S-1
        double xs[C], ys;
        gen.row_at(S, xs, ys);
        hh_apply<C>(H, S, xs, ys);
        const double xss = xs[S];
        double xnorm = 0.0 + xss * xss;
        if (S + 1 < R) {
            gen.begin(S + 1);
            stream_elems<2>(row, gen.first_elem(S + 1), n, [&](double v) {
                double x[C], y;
                gen.push(v, x, y);
                hh_apply<C>(H, S, x, y);
                xnorm = xnorm + x[S] * x[S];
            });
        }
        const double a = (xss > 0) ? -sqrt(xnorm) : sqrt(xnorm);
        H.a[S] = a;
        if (a == 0.0) return ARIMA_ST_SINGULAR;   // decompose skips it; Solver.solve then throws Singular
        const double vt = xss - a;
        H.vtop[S] = vt;
        // pass 2: alpha_{S,c} (c > S) and the Q^T y dot product, both sequential over rows S..R-1
        double al[C], dt;
#pragma unroll
        for (int c = 0; c < C; ++c) al[c] = (c > S) ? 0.0 - xs[c] * vt : 0.0;
        dt = 0.0 + ys * vt;
        if (S + 1 < R) {
            gen.begin(S + 1);
            stream_elems<2>(row, gen.first_elem(S + 1), n, [&](double v) {
                double x[C], y;
                gen.push(v, x, y);
                hh_apply<C>(H, S, x, y);
                const double vs = x[S];
#pragma unroll
                for (int c = S + 1; c < C; ++c) al[c] = al[c] - x[c] * vs;
                dt = dt + y * vs;
            });
        }
        const double den = a * vt;
#pragma unroll
        for (int c = 0; c < C; ++c) H.alpha[S][c] = (c > S) ? al[c] / den : 0.0;
        H.dot[S] = dt / den;
        return ols_stage<C, S + 1>(gen, row, n, R, H);
    }
}

template <int C, class Gen>
__device__ __forceinline__ int stream_ols(Gen &gen, const double *__restrict__ row, int n, int R, double (&beta)[C]) {
    HouseholderState<C> H;
    const int st = ols_stage<C, 0>(gen, row, n, R, H);
    if (st != ARIMA_ST_OK) return st;
    // rows 0..C-1 after their own reflection: upper triangle of R (rrow) and the top of Q^T y
    double rrow[C][C];
    double ytop[C];
#pragma unroll
    for (int i = 0; i < C; ++i) {
        double x[C], y;
        gen.row_at(i, x, y);
        hh_apply<C>(H, i, x, y);
        // reflection i on row i: qrt[c][i] -= alpha * qrt[i][i] (= vtop_i); y[i] += dot * vtop_i
#pragma unroll
        for (int c = i + 1; c < C; ++c) x[c] = x[c] - H.alpha[i][c] * H.vtop[i];
        y = y + H.dot[i] * H.vtop[i];
#pragma unroll
        for (int c = 0; c < C; ++c) rrow[i][c] = x[c];
        ytop[i] = y;
    }
    // Solver.solve back-substitution
#pragma unroll
    for (int r = C - 1; r >= 0; --r) {
        ytop[r] = ytop[r] / H.a[r];
        const double yRow = ytop[r];
        beta[r] = yRow;
#pragma unroll
        for (int i = 0; i < C; ++i)
            if (i < r) ytop[i] = ytop[i] - yRow * rrow[i][r];
    }
    return ARIMA_ST_OK;
}

// ------------------------------------------------------------------------------------------------------
// Row generators over one series (ARIMA.scala:216-242, Autoregression.scala:38-53, Lag.scala:33-99).
// ------------------------------------------------------------------------------------------------------

// AR(m) regression: row r = [1?, y(r+m-1), ..., y(r)], response y(r+m).  C = INTERCEPT + m.
// Streaming: row r is completed by element r + m; window w[l] = y(r + m - l), l = 0..m.
template <int m, int INTERCEPT>
struct ARGen {
    static constexpr int C = INTERCEPT + m;
    const double *__restrict__ y;
    double w[m + 1];
    __device__ __forceinline__ void row_at(int r, double (&x)[C], double &yv) const {
        if constexpr (INTERCEPT) x[0] = 1.0;
#pragma unroll
        for (int l = 1; l <= m; ++l) x[INTERCEPT + l - 1] = y[r + m - l];
        yv = y[r + m];
    }
    __device__ __forceinline__ int first_elem(int r) const { return r + m; }
    __device__ __forceinline__ void begin(int r) {
#pragma unroll
        for (int l = 1; l <= m; ++l) w[l] = y[r + m - l];
    }
    __device__ __forceinline__ void push(double v, double (&x)[C], double &yv) {
        w[0] = v;
        if constexpr (INTERCEPT) x[0] = 1.0;
#pragma unroll
        for (int l = 1; l <= m; ++l) x[INTERCEPT + l - 1] = w[l];
        yv = w[0];
#pragma unroll
        for (int l = m; l >= 1; --l) w[l] = w[l - 1];
    }
};

// Hannan-Rissanen second-stage regression (ARIMA.scala:226-239):
//   errors(s) = yTrunc(s) - ((sum_j y(s+m-1-j) * a_j) + c)    with yTrunc = y.drop(m)     (:228-232)
//   row r = [1?, yTrunc(r+M-1..r+M-p), errors(r+M-1..r+M-q)],  response yTrunc(r + M)   (:234-239)
// Streaming: row r is completed by element e(r) = m + M + r; y window w[l] = y(e(r) - l), l = 0..m+1;
// errors window ew[l] = errors(r + M - l), l = 1..q; the newest error of row r is errors(r+M-1), which uses
// y(e(r)-1-m .. e(r)-1) = w[1..m+1].
template <int P, int Q, int I>
struct HRGen {
    static constexpr int M = (P > Q ? P : Q);
    static constexpr int m = M + 1;
    static constexpr int C = I + P + Q;
    static constexpr int QA = Q > 0 ? Q : 1;
    const double *__restrict__ y;
    double a[m];
    double c;
    double w[m + 2];
    double ew[QA + 1];
    __device__ __forceinline__ double err_at(int s) const {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < m; ++j) acc = acc + y[s + m - 1 - j] * a[j];
        return y[s + m] - (acc + c);
    }
    __device__ __forceinline__ void row_at(int r, double (&x)[C > 0 ? C : 1], double &yv) const {
        if constexpr (I) x[0] = 1.0;
#pragma unroll
        for (int l = 1; l <= P; ++l) x[I + l - 1] = y[m + r + M - l];
#pragma unroll
        for (int l = 1; l <= Q; ++l) x[I + P + l - 1] = err_at(r + M - l);
        yv = y[m + r + M];
    }
    __device__ __forceinline__ int first_elem(int r) const { return m + M + r; }
    __device__ __forceinline__ void begin(int r) {
        const int e = m + M + r;
#pragma unroll
        for (int l = 1; l <= m + 1; ++l) w[l] = y[e - l];
#pragma unroll
        for (int l = 2; l <= Q; ++l) ew[l] = err_at(r + M - l);
    }
    __device__ __forceinline__ void push(double v, double (&x)[C > 0 ? C : 1], double &yv) {
        w[0] = v;
        if constexpr (Q > 0) {
            double acc = 0.0;
#pragma unroll
            for (int j = 0; j < m; ++j) acc = acc + w[2 + j] * a[j];
            ew[1] = w[1] - (acc + c);
        }
        if constexpr (I) x[0] = 1.0;
#pragma unroll
        for (int l = 1; l <= P; ++l) x[I + l - 1] = w[l];
#pragma unroll
        for (int l = 1; l <= Q; ++l) x[I + P + l - 1] = ew[l];
        yv = w[0];
#pragma unroll
        for (int l = m + 1; l >= 1; --l) w[l] = w[l - 1];
#pragma unroll
        for (int l = QA; l >= 2; --l) ew[l] = ew[l - 1];
    }
};

// ------------------------------------------------------------------------------------------------------
// ARIMAModel.isStationary / isInvertible (ARIMA.scala:777-815): "no root of 1 + c_1 x + ... + c_k x^k with
// |root| <= 1". The reference takes companion-matrix eigenvalues (commons EigenDecomposition); the lane uses
// the equivalent Schur-Cohn step-down: all roots of the reversed polynomial strictly inside the unit circle
// <=> every reflection coefficient |k_m| < 1. Same boolean except for roots within rounding of |z| = 1.
// ------------------------------------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ bool roots_outside_unit_circle(const double (&poly)[N + 1]) {
    double a[N + 1];
#pragma unroll
    for (int i = 0; i <= N; ++i) {
        a[i] = poly[i];
        if (!finite(a[i])) return false;
    }
#pragma unroll
    for (int mm = N; mm >= 1; --mm) {
        const double kk = a[mm];
        if (!(fabs(kk) < 1.0)) return false;
        const double den = 1.0 - kk * kk;
        double b[N + 1];
#pragma unroll
        for (int i = 0; i <= N; ++i) b[i] = (i < mm) ? (a[i] - kk * a[mm - i]) / den : 0.0;
#pragma unroll
        for (int i = 0; i <= N; ++i) a[i] = b[i];
    }
    return true;
}

template <int P, int Q, int I>
__device__ __forceinline__ uint8_t model_flags(const double (&c)[I + P + Q > 0 ? I + P + Q : 1]) {
    uint8_t f = 0;
    bool st = true, inv = true;
    if constexpr (P > 0) {
        double poly[P + 1];
        poly[0] = 1.0;
#pragma unroll
        for (int j = 0; j < P; ++j) poly[1 + j] = -1.0 * c[I + j];
        st = roots_outside_unit_circle<P>(poly);
    }
    if constexpr (Q > 0) {
        double poly[Q + 1];
        poly[0] = 1.0;
#pragma unroll
        for (int j = 0; j < Q; ++j) poly[1 + j] = c[I + P + j];
        inv = roots_outside_unit_circle<Q>(poly);
    }
    if (st) f |= ARIMA_FLAG_STATIONARY;
    if (inv) f |= ARIMA_FLAG_INVERTIBLE;
    return f;
}

// ------------------------------------------------------------------------------------------------------
// commons-math3 3.4.1 NonLinearConjugateGradientOptimizer(FLETCHER_REEVES, SimpleValueChecker(1e-7, 1e-7))
// with LineSearch (BracketFinder + BrentOptimizer(1e-15, MIN_VALUE, SimpleUnivariateValueChecker(1e-8,1e-8)))
// as a per-lane resumable state machine (ARIMA.scala:174-200). The lane posts one request at a time
// (objective F or gradient G at `x`); the wave serves all posted requests in one pass over the series.
//
// Requests that need no pass (every one of them still counted exactly as the reference counts it):
//   - F(point) at the top of each CG iteration: equals the line search's best value (same point, same ops)
//     or, on the first iteration, the objective fused into the G(x0) pass;
//   - the bracket's f(0) = F(point) when the direction is finite; Brent's f(mid) = the bracket's f at mid;
//   - any non-finite point: the CSS objective and gradient are NaN (every step multiplies every coefficient).
// ------------------------------------------------------------------------------------------------------
enum : int { REQ_NONE = 0, REQ_F = 1, REQ_G = 2 };

// Speculative line-search points. In most line searches the bracket's next points do not depend on function
// values (BracketFinder's golden extension xC = xB + GOLD(xB - xA), then the grow-limit extrapolation
// wLim = xB + 100 (xC - xB) while the objective keeps rising), so an objective request in the bracket phase
// carries up to kSpec predicted alphas. The pass evaluates them as extra chains over the same streamed series
// (same bytes); their values go into a per-lane cache keyed by the exact alpha bits, consulted before any
// later evaluation of the same line search. A hit is a point the reference evaluates with the same operations,
// so results (and evaluation counts) are unchanged; a miss only costs the extra chain's arithmetic.
#ifndef STS_SPEC
#define STS_SPEC 1
#endif
template <int K>
constexpr int spec_slots() { return K <= 8 ? STS_SPEC : 0; }   // LDS budget: no speculation at K > 8

enum : int {
    PC_START = 0, PC_G0, PC_TOP, PC_BR_FA, PC_BR_FB, PC_BR_FC, PC_BR_LOOP, PC_BR_A1, PC_BR_C1,
    PC_BR_SHIFT_EV, PC_BR_SHIFT, PC_BR_END, PC_BRENT_FX, PC_BRENT_LOOP, PC_BRENT_FU, PC_LS_DONE, PC_G,
    PC_EVAL, PC_DONE
};

// Precision.equals(x, y, 1)
__device__ __forceinline__ bool prec_equals(double x, double y) {
    const long long xi = __double_as_longlong(x), yi = __double_as_longlong(y);
    bool eq;
    if (((xi ^ yi) & (long long)0x8000000000000000ull) == 0) {
        long long dd = xi - yi;
        eq = (dd < 0 ? -dd : dd) <= 1;
    } else {
        const long long NEG0 = (long long)0x8000000000000000ull;
        long long dplus, dminus;
        if (xi < yi) { dplus = yi; dminus = xi - NEG0; } else { dplus = xi; dminus = yi - NEG0; }
        eq = (dplus > 1) ? false : (dminus <= (1 - dplus));
    }
    return eq && !__builtin_isnan(x) && !__builtin_isnan(y);
}

// SimpleValueChecker.converged: |p-c| <= max(|p|,|c|)*rel || |p-c| <= abs, FastMath.max propagates NaN
__device__ __forceinline__ bool value_converged(double p, double c, double rel, double abs_) {
    const double diff = fabs(p - c);
    const double ap = fabs(p), ac = fabs(c);
    double size;
    if (ap > ac) size = ap;
    else if (ap < ac) size = ac;
    else if (ap != ac) size = __builtin_nan("");
    else size = ap;
    return (diff <= size * rel) || (diff <= abs_);
}

// One lane's optimizer state, kept compact because it lives in LDS for every lane of the persistent fit kernel
// and its size sets how many waves share a CU: bracket and Brent fields share storage (they are
// never live together), the request point is recomputed by the pass from (point, dir, ev_alpha) with the same
// operations, responses arrive as advance() arguments (registers), counters are 16-bit (all bounded by 10001).
template <int K, int NS_>
struct CGLane {
    static constexpr int NS = NS_;
    static constexpr int NS1 = NS > 0 ? NS : 1;
    // optimizer (NonLinearConjugateGradientOptimizer.doOptimize)
    double point[K], dir[K];
    double delta, memo_obj, prev_obj;
    // line search: BracketFinder and BrentOptimizer state (disjoint lifetimes)
    union {
        struct { double xA, xB, xC, fA, fB, fC, w, fW; };
        struct { double a, b, bx, bv, bw, bd, be, fx, fv, fw, u, prev_x, prev_f, cur_x, cur_f, best_x, best_f; };
    };
    double ev_alpha;                       // pending objective request: point + ev_alpha * dir
    // speculation: cache of the current line search, and the predicted alphas of the posted request
    double sp_alpha[NS1], sp_f[NS1], rq_spec[NS1];
    uint16_t n_eval, n_grad, iter, bcount, spec_hits;
    uint8_t pc, status, req, have_prev_obj, have_prev, sp_n, rq_nspec;

    __device__ __forceinline__ void start(const double (&init)[K]) {
#pragma unroll
        for (int i = 0; i < K; ++i) point[i] = init[i];
        pc = PC_START;
        status = ARIMA_ST_OK;
        n_eval = n_grad = iter = 0;
        have_prev_obj = 0;
        req = REQ_NONE;
        sp_n = rq_nspec = 0;
        spec_hits = 0;
    }

    __device__ __forceinline__ void fail(int st) {
        status = (uint8_t)st;
        pc = PC_DONE;
    }

    __device__ __forceinline__ bool done() const { return pc == PC_DONE; }

    // coefficients of the posted request (the same expression PC_EVAL checks for finiteness)
    __device__ __forceinline__ void request_point(double (&c)[K]) const {
        if (req == REQ_G) {
#pragma unroll
            for (int i = 0; i < K; ++i) c[i] = point[i];
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i) c[i] = point[i] + ev_alpha * dir[i];
        }
    }

    // Run the state machine until a request is posted (req != REQ_NONE) or the fit is finished. fr / gr are
    // the response to the request served last (objective; and the gradient for a G request).
    __device__ void advance(double fr, const double (&gr)[K]) {
        const double GOLD = 1.618034, EPS_MIN = 1e-21, GROW = 100.0;
        const double GS = 0.5 * (3 - __builtin_sqrt(5.0));   // BrentOptimizer.GOLDEN_SECTION
        double ev_val = fr;                                   // objective value delivered to the resume point
        double grad[K];                                       // gradient delivered to PC_G0 / PC_G
#pragma unroll
        for (int i = 0; i < K; ++i) grad[i] = gr[i];
        // eval subroutine (LineSearch's objective): locals of this call, never live across a pass
        double ev_memo = 0.0;
        int ev_memo_ok = 0, ev_bracket = 0, ev_ret = PC_DONE;
        auto eval = [&](double alpha, int bracket, int memo_ok, double memo, int ret) {
            ev_alpha = alpha;
            ev_bracket = bracket;
            ev_memo_ok = memo_ok;
            ev_memo = memo;
            ev_ret = ret;
            pc = PC_EVAL;
        };
        for (;;) {
            switch (pc) {
            case PC_START:
                // r = computeObjectiveGradient(point)
                req = REQ_G;
                pc = PC_G0;
                return;
            case PC_G0: {
                n_grad++;
                double dl = 0.0;
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    dir[i] = grad[i];                     // steepestDescent = precondition(r) = r.clone()
                    dl = dl + grad[i] * dir[i];
                }
                delta = dl;
                memo_obj = ev_val;                        // F(point) fused into the gradient pass
                pc = PC_TOP;
                break;
            }
            case PC_TOP: {
                if (iter + 1 > kMaxIter) { fail(ARIMA_ST_MAX_ITER); return; }
                iter++;
                if (n_eval + 1 > kMaxEval) { fail(ARIMA_ST_MAX_EVAL); return; }
                n_eval++;
                const double objective = memo_obj;
                const bool conv = have_prev_obj && value_converged(prev_obj, objective, 1e-7, 1e-7);
                prev_obj = objective;
                have_prev_obj = 1;
                if (conv) { pc = PC_DONE; return; }   // status OK; point / prev_obj are the result
                // line.search(point, searchDirection)
                sp_n = 0;
                bcount = 0;
                xA = 0.0;
                xB = 1e-8;
                bool dfin = true;
#pragma unroll
                for (int i = 0; i < K; ++i) dfin = dfin && finite(dir[i]);
                eval(xA, 1, dfin ? 1 : 0, objective, PC_BR_FA);
                break;
            }
            case PC_BR_FA:
                fA = ev_val;
                eval(xB, 1, 0, 0.0, PC_BR_FB);
                break;
            case PC_BR_FB: {
                fB = ev_val;
                if (fA > fB) {
                    double t = xA; xA = xB; xB = t;
                    t = fA; fA = fB; fB = t;
                }
                xC = xB + GOLD * (xB - xA);
                eval(xC, 1, 0, 0.0, PC_BR_FC);
                break;
            }
            case PC_BR_FC:
                fC = ev_val;
                pc = PC_BR_LOOP;
                break;
            case PC_BR_LOOP: {
                if (!(fC > fB)) { pc = PC_BR_END; break; }
                const double tmp1 = (xB - xA) * (fB - fC);
                const double tmp2 = (xB - xC) * (fB - fA);
                const double val = tmp2 - tmp1;
                const double denom = fabs(val) < EPS_MIN ? 2 * EPS_MIN : val;
                w = xB - ((xB - xC) * tmp2 - (xB - xA) * tmp1) / (2 * denom);
                const double wLim = xB + GROW * (xC - xB);
                if ((w - xC) * (xB - w) > 0) {
                    eval(w, 1, 0, 0.0, PC_BR_A1);
                } else if ((w - wLim) * (wLim - xC) >= 0) {
                    w = wLim;
                    eval(w, 1, 0, 0.0, PC_BR_SHIFT_EV);
                } else if ((w - wLim) * (xC - w) > 0) {
                    eval(w, 1, 0, 0.0, PC_BR_C1);
                } else {
                    w = xC + GOLD * (xC - xB);
                    eval(w, 1, 0, 0.0, PC_BR_SHIFT_EV);
                }
                break;
            }
            case PC_BR_A1:
                fW = ev_val;
                if (fW > fC) {
                    xA = xB; xB = w; fA = fB; fB = fW;
                    pc = PC_BR_END;
                } else if (fW < fB) {
                    xC = w; fC = fW;
                    pc = PC_BR_END;
                } else {
                    w = xC + GOLD * (xC - xB);
                    eval(w, 1, 0, 0.0, PC_BR_SHIFT_EV);
                }
                break;
            case PC_BR_C1:
                fW = ev_val;
                if (fW > fC) {
                    xB = xC; xC = w; w = xC + GOLD * (xC - xB); fB = fC; fC = fW;
                    eval(w, 1, 0, 0.0, PC_BR_SHIFT_EV);
                } else {
                    pc = PC_BR_SHIFT;
                }
                break;
            case PC_BR_SHIFT_EV:
                fW = ev_val;
                pc = PC_BR_SHIFT;
                break;
            case PC_BR_SHIFT:
                xA = xB; fA = fB; xB = xC; fB = fC; xC = w; fC = fW;
                pc = PC_BR_LOOP;
                break;
            case PC_BR_END: {
                // bracket -> Brent (shared storage: read everything needed before writing)
                double lo = xA, hi = xC;
                const double mid = xB, fmid = fB;
                if (lo > hi) { double t = lo; lo = hi; hi = t; }
                if (lo >= hi || mid < lo || mid > hi) { fail(ARIMA_ST_BAD_INTERVAL); return; }  // SearchInterval
                if (lo < hi) { a = lo; b = hi; } else { a = hi; b = lo; }
                bx = bv = bw = mid;
                bd = be = 0.0;
                eval(mid, 0, 1, fmid, PC_BRENT_FX);                      // fx = f(mid) (memo: bracket fMid)
                break;
            }
            case PC_BRENT_FX:
                fx = -ev_val;
                fv = fw = fx;
                have_prev = 0;
                cur_x = bx; cur_f = -fx;
                best_x = cur_x; best_f = cur_f;
                pc = PC_BRENT_LOOP;
                break;
            case PC_BRENT_LOOP: {
                const double m = 0.5 * (a + b);
                const double tol1 = 1e-15 * fabs(bx) + 4.9e-324;
                const double tol2 = 2 * tol1;
                if (fabs(bx - m) <= tol2 - 0.5 * (b - a)) {
                    // return best(best, best(previous, current))
                    double ix = cur_x, iv = cur_f;
                    if (have_prev && prev_f >= cur_f) { ix = prev_x; iv = prev_f; }
                    if (!(best_f >= iv)) { best_x = ix; best_f = iv; }
                    pc = PC_LS_DONE;
                    break;
                }
                double p = 0, q = 0, r = 0;
                if (fabs(be) > tol1) {
                    r = (bx - bw) * (fx - fv);
                    q = (bx - bv) * (fx - fw);
                    p = (bx - bv) * q - (bx - bw) * r;
                    q = 2 * (q - r);
                    if (q > 0) p = -p; else q = -q;
                    r = be;
                    be = bd;
                    if (p > q * (a - bx) && p < q * (b - bx) && fabs(p) < fabs(0.5 * q * r)) {
                        bd = p / q;
                        u = bx + bd;
                        if (u - a < tol2 || b - u < tol2) bd = (bx <= m) ? tol1 : -tol1;
                    } else {
                        be = (bx < m) ? b - bx : a - bx;
                        bd = GS * be;
                    }
                } else {
                    be = (bx < m) ? b - bx : a - bx;
                    bd = GS * be;
                }
                if (fabs(bd) < tol1) u = (bd >= 0) ? bx + tol1 : bx - tol1;
                else u = bx + bd;
                eval(u, 0, 0, 0.0, PC_BRENT_FU);
                break;
            }
            case PC_BRENT_FU: {
                const double fu = -ev_val;
                prev_x = cur_x; prev_f = cur_f; have_prev = 1;
                cur_x = u; cur_f = ev_val;
                {
                    double ix = cur_x, iv = cur_f;
                    if (prev_f >= cur_f) { ix = prev_x; iv = prev_f; }
                    if (!(best_f >= iv)) { best_x = ix; best_f = iv; }
                }
                if (value_converged(prev_f, cur_f, 1e-8, 1e-8)) { pc = PC_LS_DONE; break; }
                if (fu <= fx) {
                    if (u < bx) b = bx; else a = bx;
                    bv = bw; fv = fw; bw = bx; fw = fx; bx = u; fx = fu;
                } else {
                    if (u < bx) a = u; else b = u;
                    if (fu <= fw || prec_equals(bw, bx)) { bv = bw; fv = fw; bw = u; fw = fu; }
                    else if (fu <= fv || prec_equals(bv, bx) || prec_equals(bv, bw)) { bv = u; fv = fu; }
                }
                pc = PC_BRENT_LOOP;
                break;
            }
            case PC_LS_DONE: {
                // point[i] += step * searchDirection[i]; r = computeObjectiveGradient(point)
                const double step = best_x;
                memo_obj = best_f;                    // F(point) == Brent's value at `step`
                bool pfin = true;
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    point[i] = point[i] + step * dir[i];
                    pfin = pfin && finite(point[i]);
                }
                if (!pfin) {                          // the gradient at a non-finite point is NaN: no pass
#pragma unroll
                    for (int i = 0; i < K; ++i) grad[i] = __builtin_nan("");
                    pc = PC_G;
                    break;
                }
                req = REQ_G;
                pc = PC_G;
                return;
            }
            case PC_G: {
                n_grad++;
                const double deltaOld = delta;
                double dl = 0.0;
#pragma unroll
                for (int i = 0; i < K; ++i) dl = dl + grad[i] * grad[i];
                delta = dl;
                const double beta = delta / deltaOld;       // FLETCHER_REEVES
                if (iter % K == 0 || beta < 0) {
#pragma unroll
                    for (int i = 0; i < K; ++i) dir[i] = grad[i];
                } else {
#pragma unroll
                    for (int i = 0; i < K; ++i) dir[i] = grad[i] + beta * dir[i];
                }
                pc = PC_TOP;
                break;
            }
            case PC_EVAL: {
                if (ev_bracket) {
                    if (bcount + 1 > kBracketMax) { fail(ARIMA_ST_BRACKET_MAX_EVAL); return; }
                    bcount++;
                }
                if (n_eval + 1 > kMaxEval) { fail(ARIMA_ST_MAX_EVAL); return; }
                n_eval++;
                if (ev_memo_ok) { ev_val = ev_memo; pc = ev_ret; break; }
                bool fin = true;
#pragma unroll
                for (int i = 0; i < K; ++i) fin = fin && finite(point[i] + ev_alpha * dir[i]);
                if (!fin) { ev_val = __builtin_nan(""); pc = ev_ret; break; }
                rq_nspec = 0;
                if constexpr (NS > 0) {
                    // (static indexing only: the state never needs scratch)
                    const long long ab = __double_as_longlong(ev_alpha);
                    bool hit = false;
#pragma unroll
                    for (int s = 0; s < NS; ++s)
                        if (s < sp_n && __double_as_longlong(sp_alpha[s]) == ab) { ev_val = sp_f[s]; hit = true; }
                    if (hit) { spec_hits++; pc = ev_ret; break; }
                    // predict the bracket's next value-independent points (same expressions as above)
                    double bb = 0.0, cc = 0.0, first = 0.0;
                    bool chain = true, has_first = false;
                    switch (ev_ret) {
                    case PC_BR_FB:                                      // xC if fA <= fB, then the wLim chain
                        cc = xB + GOLD * (xB - xA);
                        first = cc;
                        has_first = true;
                        bb = xB;
                        break;
                    case PC_BR_FC: bb = xB; cc = xC; break;            // wLim chain from (xB, xC)
                    case PC_BR_SHIFT_EV: bb = xC; cc = w; break;       // the shift makes (xB, xC) = (xC, w)
                    case PC_BR_A1:                                      // no break: golden extension
                        first = xC + GOLD * (xC - xB);
                        has_first = true;
                        chain = false;
                        break;
                    case PC_BR_C1:                                      // fW > fC: golden extension from w
                        first = w + GOLD * (w - xC);
                        has_first = true;
                        chain = false;
                        break;
                    default: chain = false; break;
                    }
                    int cnt = 0;
#pragma unroll
                    for (int h = 0; h < NS; ++h) {
                        if (h == 0 && has_first) {
                            rq_spec[h] = first;
                            cnt++;
                        } else if (chain) {
                            const double nx = bb + GROW * (cc - bb);
                            rq_spec[h] = nx;
                            bb = cc;
                            cc = nx;
                            cnt++;
                        }
                    }
                    rq_nspec = (uint8_t)cnt;
                }
                req = REQ_F;
                pc = (uint8_t)ev_ret;                  // resume point once the response arrives
                return;
            }
            case PC_DONE:
            default:
                return;
            }
        }
    }
};

// LDS slot of one lane's optimizer state: padded to an odd number of 8-byte words so that 64 lanes reading the
// same field with ds_read_b64 hit distinct bank pairs (stride = 8 * odd bytes; MI355X_MICROARCH.md LDS table).
template <int K, int NS>
struct alignas(8) LaneSlot {
    static constexpr int kWords = (int)((sizeof(CGLane<K, NS>) + 7) / 8);
    static constexpr int kPadWords = (kWords % 2 == 0) ? 1 : 2;   // total word count odd
    CGLane<K, NS> s;
    double pad[kPadWords];
};

// Waves per workgroup of the fit kernel (one workgroup per CU, 64 lanes per wave): as many as the LDS slots of
// 64 lanes fit in 160 KiB, at most STS_CG_MAX_WAVES (4 = one per SIMD: measured faster than two per SIMD,
// which halves the pass's register budget and doubles the in-flight streams per CU).
#ifndef STS_CG_MAX_WAVES
#define STS_CG_MAX_WAVES 4
#endif
template <int K, int NS>
constexpr int cg_waves() {
    constexpr int per_wave = 64 * (int)sizeof(LaneSlot<K, NS>);
    constexpr int w = 163840 / per_wave;
    return w > STS_CG_MAX_WAVES ? STS_CG_MAX_WAVES : (w < 1 ? 1 : w);
}

// ------------------------------------------------------------------------------------------------------
// Philox4x32-10 (counter-based) + Box-Muller for the synthetic generator
// ------------------------------------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t ctr[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ ctr[1] ^ k0;
        const uint32_t n2 = hi0 ^ ctr[3] ^ k1;
        ctr[0] = n0; ctr[1] = lo1; ctr[2] = n2; ctr[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

__device__ __forceinline__ double u01_53(uint32_t a, uint32_t b) {    // [0, 1)
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

}  // namespace sts
