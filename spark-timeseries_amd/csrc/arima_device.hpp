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

#include <type_traits>

#include "../../include/sparkts_arima.h"
#include "arima_launch.hpp"
#include "cg_lane.hpp"

namespace sts {

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
// The differenced series read straight from the caller's row (round 6, fused differencing). The fit path works on
// differencesOfOrderD(ts, d).drop(d) (ARIMA.scala:88): element i of it is raw[i + 1] - raw[i] for d = 1 (the
// subtraction differencesAtLag performs, UnivariateTimeSeries.scala:384-405) and raw[i] for d = 0. Passes form it on
// the fly from the raw row instead of reading a differenced copy that a separate kernel wrote (17 GB of HBM traffic
// per 1M x 1024 fit, and its own pipeline stage); d >= 2 still goes through the k_difference workspace (dd = 0).
// `raw` needs only the 8-B alignment of a double: stream_row streams whole 128-B lines from the line that holds its
// first element (a line that holds a valid element never crosses a page, so the head and tail reads stay mapped).
// ------------------------------------------------------------------------------------------------------
__device__ __forceinline__ double drow_at(const double *__restrict__ raw, int dd, int i) {
    return dd ? raw[i + 1] - raw[i] : raw[i];
}

// fn(x_i) for i = first .. last-1 of the differenced row (dd = 0 or 1) over the raw row, in order
template <int D, class Fn>
__device__ __forceinline__ void stream_row(const double *__restrict__ raw, int dd, int first, int last, Fn &&fn) {
    if (first >= last) return;
    const int off = (int)((reinterpret_cast<uintptr_t>(raw) >> 3) & (kChunk - 1));   // elements before raw in its line
    double prev = raw[first];                          // raw[first + dd - 1] for dd = 1 (unused for dd = 0)
    stream_elems<D>(raw - off, first + dd + off, last + dd + off, [&](double x) {
        const double v = dd ? x - prev : x;            // wave-uniform select: no branch in the unrolled stream
        prev = x;
        fn(v);
    });
}

// ------------------------------------------------------------------------------------------------------
// CSS pass (objective, and optionally gradient) over one series — ARIMA.scala:430-534
//
// Lanes hold the maTerms buffer as two registers: updateMAErrors (:544-554) copies errs(i) -> errs(i+1) in
// ASCENDING i, so after every update positions 1..q-1 all equal the previous errs(0): maTerms is
// [e_{t-1}, e_{t-2}, e_{t-2}, ...] (a smear for q >= 3, exactly what the reference computes).
// ------------------------------------------------------------------------------------------------------
// (round 4: 4 / 2 -> 3 / 1 on one box: pipelined C2 9.47-9.59 -> 10.47-10.58 M series/s, isolated launch 138.5 ->
// 128.6 ms, profiles/r04/p_pf; registers and scratch of k_cg_fit unchanged -- the F pass's inner loop schedules better)
constexpr int kPrefetchF = 3;   // chunks in flight per lane in objective passes
constexpr int kPrefetchG = 1;   // ... in gradient passes (5x the VALU work per byte)

// Full pass. G = false: objective only -> css. G = true: also gradientlogLikelihoodCSSARMA -> g[] (already
// divided by -sigma2, :532). SMEAR selects the Breeze overlap semantics of :526 (false = row shift).
// RAW (the fit kernel): `row` is the caller's row at any 8-B alignment, differenced on the fly when dd = 1
// (stream_row); otherwise a 128-B aligned differenced workspace row, padded to >= 16 elements (stream_elems).
template <int P, int Q, int I, bool G, bool SMEAR, bool RAW = false, int DPF = (G ? kPrefetchG : kPrefetchF)>
__device__ __forceinline__ void css_pass(const double *__restrict__ row, int n,
                                         const double (&c)[I + P + Q > 0 ? I + P + Q : 1], double &css_out,
                                         double (&g)[I + P + Q > 0 ? I + P + Q : 1], int dd = 0) {
    constexpr int K = I + P + Q;
    constexpr int KA = K > 0 ? K : 1;
    constexpr int M = (P > Q ? P : Q);
    constexpr int PA = P > 0 ? P : 1;
    double yl[PA];                        // yl[j] = y_{i-1-j}
#pragma unroll
    for (int j = 0; j < PA; ++j) {
        if constexpr (RAW) yl[j] = (j < P && M - 1 - j < n) ? drow_at(row, dd, M - 1 - j) : 0.0;
        else yl[j] = (j < P) ? row[M - 1 - j] : 0.0;
    }
    double e1 = 0.0, e2 = 0.0, css = 0.0, sigma2 = 0.0;
    const double yh0 = 0.0 + (double)I * c[0];
    const double nd = (double)n;
    // dEdTheta (:476), row r = d e_{t-r} / d theta. Under SMEAR (Breeze's element-wise copy at :526, DESIGN.md
    // 5.1) rows 1..q always hold the same values (the previous row 0), so two rows carry the whole matrix.
    constexpr int DER = G ? (SMEAR ? (Q > 0 ? 2 : 1) : Q + 1) : 1;
    double dE[DER][KA];
    if constexpr (G) {
#pragma unroll
        for (int r = 0; r < DER; ++r)
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
                for (int kk = 0; kk < Q; ++kk) dE[0][j] = dE[0][j] - c[I + P + kk] * dE[SMEAR ? DER - 1 : kk + 1][j];
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
                if constexpr (Q > 0) {
#pragma unroll
                    for (int j = 0; j < KA; ++j) dE[1][j] = dE[0][j];
                }
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
    if constexpr (RAW) stream_row<DPF>(row, dd, M, n, step);
    else stream_elems<DPF>(row, M, n, step);
    css_out = css;
    if constexpr (G) {
#pragma unroll
        for (int j = 0; j < KA; ++j) g[j] = g[j] / -sigma2;         // :532
    }
}

// Objective pass for NCH points at once (speculative line-search points): NCH independent recursions over the
// same streamed series. Each chain is exactly the single-point objective (same ops, same order).
template <int P, int Q, int I, int NCH, int DPF = kPrefetchF>
__device__ __forceinline__ void css_pass_multi(const double *__restrict__ row, int n,
                                               const double (&c)[NCH][I + P + Q > 0 ? I + P + Q : 1],
                                               double (&css_out)[NCH], int dd = 0) {
    constexpr int M = (P > Q ? P : Q);
    constexpr int PA = P > 0 ? P : 1;
    double yl[PA];
#pragma unroll
    for (int j = 0; j < PA; ++j) yl[j] = (j < P && M - 1 - j < n) ? drow_at(row, dd, M - 1 - j) : 0.0;
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
    stream_row<DPF>(row, dd, M, n, step);
#pragma unroll
    for (int h = 0; h < NCH; ++h) css_out[h] = css[h];
}

// ------------------------------------------------------------------------------------------------------
// Passes over a series held in LDS by a whole wave (the express path of k_cg_fit: one long-running series per
// wave). Every lane reads the same element at the same step (LDS broadcast).
//   css_row_lds       one objective chain per lane (the lanes evaluate the request's point and its predictions)
//   grad_column_lds   gradientlogLikelihoodCSSARMA split by column: lane `col` carries column `col` of dEdTheta;
//                     every lane also carries the shared residual recursion, so css and sigma2 come out the same
//                     in every lane. Same operations in the same order as css_pass<..., true, SMEAR>.
// ------------------------------------------------------------------------------------------------------
template <int P, int Q, int I>
__device__ __forceinline__ double css_row_lds(const double *row, int n,
                                              const double (&c)[I + P + Q > 0 ? I + P + Q : 1]) {
    constexpr int M = (P > Q ? P : Q);
    constexpr int PA = P > 0 ? P : 1;
    double yl[PA];
#pragma unroll
    for (int j = 0; j < PA; ++j) yl[j] = (j < P && M - 1 - j >= 0 && M - 1 - j < n) ? row[M - 1 - j] : 0.0;
    double e1 = 0.0, e2 = 0.0, css = 0.0;
    const double yh0 = 0.0 + (double)I * c[0];
#pragma unroll 8
    for (int t = M; t < n; ++t) {
        const double yi = row[t];
        double yh = yh0;
#pragma unroll
        for (int j = 0; j < P; ++j) yh = yh + yl[j] * c[I + j];
#pragma unroll
        for (int j = 0; j < Q; ++j) yh = yh + (j == 0 ? e1 : e2) * c[I + P + j];
        const double e = yi - yh;
        css = css + e * e;
        e2 = e1;
        e1 = e;
        if constexpr (P > 0) {
#pragma unroll
            for (int j = PA - 1; j >= 1; --j) yl[j] = yl[j - 1];
            yl[0] = yi;
        }
    }
    return css;
}

// ------------------------------------------------------------------------------------------------------
// Objective passes of NCH points over one series in LDS with all 64 lanes of the wave (the express path's
// objective requests, parallel in time). The CSS recursion e_t = y_t - yh_t(e_{t-1}, e_{t-2}) is serial in t,
// but a step only needs the two previous residuals (updateMAErrors leaves e_{t-1}, e_{t-2}, e_{t-2}, ... in
// maTerms, ARIMA.scala:544-554). Lane L owns the time block [M + L*B, M + (L+1)*B): a SWEEP recomputes every
// block from the two residuals its left neighbour ended the previous sweep with (lane 0 from the reference's
// zero maTerms), with the reference's operations in the reference's order. When every lane's inputs equal its
// neighbour's outputs of the same sweep, each block was computed from the exact serial residuals (by induction
// from lane 0), so the block values ARE the serial recursion's, bit for bit; block 0 is exact after one sweep,
// block L after at most L + 1, so the loop ends by sweep 64 whatever the coefficients (for a stable MA part an
// input error shrinks by ~|root|^B per block and rounds away in 2-4 sweeps). The sum of squares is then folded
// left over t across the lanes in order, exactly as `css = css + e * e`. Every lane returns every chain's css.
// Chains: row h of c (all lanes pass the same coefficients); nch <= NCH of them are live (the rest are skipped).
// ------------------------------------------------------------------------------------------------------
template <int P, int Q, int I, int NCH, int BMAX>
__device__ __forceinline__ void css_pit_lds(const double *row, int n, const double (&c)[NCH][I + P + Q > 0 ? I + P + Q : 1],
                                            double (&css_out)[NCH], int lane, int *sweeps_out = nullptr) {
    constexpr int M = (P > Q ? P : Q);
    constexpr int PA = P > 0 ? P : 1;
    const int S = n - M;
    const int B = S > 0 ? (S + 63) / 64 : 0;                  // <= BMAX (the caller checks)
    const int t0 = M + lane * B;
    int len = n - t0;
    len = len < 0 ? 0 : (len > B ? B : len);
    double E[NCH][BMAX];
    double b1[NCH], b2[NCH], yh0[NCH];
#pragma unroll
    for (int h = 0; h < NCH; ++h) {
        b1[h] = b2[h] = 0.0;
        yh0[h] = 0.0 + (double)I * c[h][0];
    }
    int sweeps = 0;
    for (;;) {
        ++sweeps;
        double yl[PA];
#pragma unroll
        for (int j = 0; j < PA; ++j) yl[j] = (j < P && len > 0) ? row[t0 - 1 - j] : 0.0;
        double e1[NCH], e2[NCH];
#pragma unroll
        for (int h = 0; h < NCH; ++h) {
            e1[h] = b1[h];
            e2[h] = b2[h];
        }
#pragma unroll
        for (int b = 0; b < BMAX; ++b) {
            if (b < len) {
                const double yi = row[t0 + b];
#pragma unroll
                for (int h = 0; h < NCH; ++h) {
                    double yh = yh0[h];                                                 // ARIMA.scala:600
#pragma unroll
                    for (int j = 0; j < P; ++j) yh = yh + yl[j] * c[h][I + j];          // :602-605
#pragma unroll
                    for (int j = 0; j < Q; ++j) yh = yh + (j == 0 ? e1[h] : e2[h]) * c[h][I + P + j];   // :608-611
                    const double e = yi - yh;                                           // :613
                    E[h][b] = e;
                    e2[h] = e1[h];
                    e1[h] = e;
                }
                if constexpr (P > 0) {
#pragma unroll
                    for (int j = PA - 1; j >= 1; --j) yl[j] = yl[j - 1];
                    yl[0] = yi;
                }
            }
        }
        // the next sweep's inputs: the left neighbour's outputs (lane 0 keeps the zero maTerms)
        bool moved = false;
#pragma unroll
        for (int h = 0; h < NCH; ++h) {
            double n1 = __shfl_up(e1[h], 1), n2 = __shfl_up(e2[h], 1);
            if (lane == 0) n1 = n2 = 0.0;
            moved = moved || __double_as_longlong(n1) != __double_as_longlong(b1[h]) ||
                    __double_as_longlong(n2) != __double_as_longlong(b2[h]);
            b1[h] = n1;
            b2[h] = n2;
        }
        if (!__any(moved)) break;                                // every block computed from exact inputs
    }
    // css = css + e * e over t = M .. n-1 in order (ARIMA.scala:440-442): block by block, lane by lane
    double css[NCH];
#pragma unroll
    for (int h = 0; h < NCH; ++h) css[h] = 0.0;
    for (int L = 0; L < 64; ++L) {
        if (lane == L) {
#pragma unroll
            for (int b = 0; b < BMAX; ++b)
                if (b < len) {
#pragma unroll
                    for (int h = 0; h < NCH; ++h) css[h] = css[h] + E[h][b] * E[h][b];
                }
        }
#pragma unroll
        for (int h = 0; h < NCH; ++h) css[h] = __shfl(css[h], L);
    }
#pragma unroll
    for (int h = 0; h < NCH; ++h) css_out[h] = css[h];
    if (sweeps_out) *sweeps_out = sweeps;
}

// Gradient pass (gradientlogLikelihoodCSSARMA, ARIMA.scala:465-534) over one series in LDS with all 64 lanes,
// parallel in time like css_pit_lds: (1) the residual recursion by block sweeps; (2) every column of dEdTheta by
// block sweeps -- row 0 of step t is (((0 - theta_1 dE_1) - theta_2 dE_2) ...) - direct_j(t) (:492-518), where under
// SMEAR every lag row holds the previous row 0 (one lag value per column) and under the row shift the q previous
// row-0 values; direct_j(t) is 1 (intercept), y_{t-1-j} (AR) or e_{t-1} / e_{t-2} (MA, the exact residuals of (1));
// (3) the left folds of sigma2 (+ e^2 / n), css and every g_j (+ dE_0j * e) over t in order, lane by lane.
// Every lane returns css and the whole gradient (already divided by -sigma2, :532). Storage per lane: the block's
// residuals and up to 6 columns of dEdTheta at a time (K > 6: two column chunks, each swept and folded in turn).
template <int P, int Q, int I, bool SMEAR, int BMAX>
__device__ __forceinline__ void grad_pit_lds(const double *row, int n, const double (&c)[I + P + Q > 0 ? I + P + Q : 1],
                                             double &css_out, double (&g_out)[I + P + Q > 0 ? I + P + Q : 1], int lane,
                                             int *sweeps_out = nullptr) {
    constexpr int K = I + P + Q;
    constexpr int KA = K > 0 ? K : 1;
    constexpr int M = (P > Q ? P : Q);
    constexpr int PA = P > 0 ? P : 1;
    constexpr int DR = SMEAR ? 1 : (Q > 0 ? Q : 1);       // lag values of one column that a step reads
    const int S = n - M;
    const int B = S > 0 ? (S + 63) / 64 : 0;
    const int t0 = M + lane * B;
    int len = n - t0;
    len = len < 0 ? 0 : (len > B ? B : len);
    const double yh0 = 0.0 + (double)I * c[0];
    // ---- (1) residuals ----
    double E[BMAX];
    double b1 = 0.0, b2 = 0.0;                            // after convergence: the exact e_{t0-1}, e_{t0-2}
    int sweeps = 0;
    for (;;) {
        ++sweeps;
        double yl[PA];
#pragma unroll
        for (int j = 0; j < PA; ++j) yl[j] = (j < P && len > 0) ? row[t0 - 1 - j] : 0.0;
        double e1 = b1, e2 = b2;
#pragma unroll
        for (int b = 0; b < BMAX; ++b) {
            if (b < len) {
                const double yi = row[t0 + b];
                double yh = yh0;
#pragma unroll
                for (int j = 0; j < P; ++j) yh = yh + yl[j] * c[I + j];
#pragma unroll
                for (int j = 0; j < Q; ++j) yh = yh + (j == 0 ? e1 : e2) * c[I + P + j];
                const double e = yi - yh;                  // :520
                E[b] = e;
                e2 = e1;
                e1 = e;
                if constexpr (P > 0) {
#pragma unroll
                    for (int j = PA - 1; j >= 1; --j) yl[j] = yl[j - 1];
                    yl[0] = yi;
                }
            }
        }
        double n1 = __shfl_up(e1, 1), n2 = __shfl_up(e2, 1);
        if (lane == 0) n1 = n2 = 0.0;
        const bool moved = __double_as_longlong(n1) != __double_as_longlong(b1) ||
                           __double_as_longlong(n2) != __double_as_longlong(b2);
        b1 = n1;
        b2 = n2;
        if (!__any(moved)) break;
    }
    // ---- (2) + (3) per chunk of at most 6 columns of dEdTheta (K * BMAX doubles would not fit the registers) ----
    constexpr int KC = K <= 6 ? KA : 6;
    const double nd = (double)n;
    double sigma2 = 0.0, css = 0.0, g[KA];
#pragma unroll
    for (int j = 0; j < KA; ++j) g[j] = 0.0;
    auto chunk = [&](auto J0c) {
        constexpr int J0 = decltype(J0c)::value;
        constexpr int JN = (J0 + KC < K ? J0 + KC : K) - J0;      // columns J0 .. J0 + JN - 1
        double D[KC][BMAX];
        double bd[KC][DR];                                       // a column's lag values entering the block
#pragma unroll
        for (int jj = 0; jj < KC; ++jj)
#pragma unroll
            for (int r = 0; r < DR; ++r) bd[jj][r] = 0.0;
        for (;;) {
            ++sweeps;
            double yl[PA];
#pragma unroll
            for (int j = 0; j < PA; ++j) yl[j] = (j < P && len > 0) ? row[t0 - 1 - j] : 0.0;
            double e1 = b1, e2 = b2;
            double dl[KC][DR];
#pragma unroll
            for (int jj = 0; jj < KC; ++jj)
#pragma unroll
                for (int r = 0; r < DR; ++r) dl[jj][r] = bd[jj][r];
#pragma unroll
            for (int b = 0; b < BMAX; ++b) {
                if (b < len) {
#pragma unroll
                    for (int jj = 0; jj < JN; ++jj) {
                        const int j = J0 + jj;
                        double d = 0.0;
#pragma unroll
                        for (int kk = 0; kk < Q; ++kk) d = d - c[I + P + kk] * dl[jj][SMEAR ? 0 : kk];   // :492-499
                        // the column's direct term (:503, :506-510, :514-518); "- I" on column 0 for I = 0 is
                        // "- 0.0", an identity, so one subtraction per column is exact
                        double dv;
                        if (I && j == 0) dv = 1.0;
                        else if (j < I + P) dv = yl[(j - I >= 0 && j - I < PA) ? j - I : 0];
                        else dv = (j == I + P) ? e1 : e2;
                        d = d - dv;
                        D[jj][b] = d;
                        if constexpr (Q > 0) {                                             // :526 (this column)
                            if constexpr (!SMEAR) {
#pragma unroll
                                for (int r = DR - 1; r >= 1; --r) dl[jj][r] = dl[jj][r - 1];
                            }
                            dl[jj][0] = d;
                        }
                    }
                    const double e = E[b];
                    e2 = e1;
                    e1 = e;
                    if constexpr (P > 0) {
#pragma unroll
                        for (int j = PA - 1; j >= 1; --j) yl[j] = yl[j - 1];
                        yl[0] = row[t0 + b];
                    }
                }
            }
            bool moved = false;
#pragma unroll
            for (int jj = 0; jj < JN; ++jj)
#pragma unroll
                for (int r = 0; r < DR; ++r) {
                    double v = __shfl_up(dl[jj][r], 1);
                    if (lane == 0) v = 0.0;
                    moved = moved || __double_as_longlong(v) != __double_as_longlong(bd[jj][r]);
                    bd[jj][r] = v;
                }
            if (Q == 0 || !__any(moved)) break;                 // no MA part: the columns do not recur
        }
        // (3) left folds over t in order, lane by lane: sigma2 and css with the first chunk, this chunk's g_j
        for (int L = 0; L < 64; ++L) {
            if (lane == L) {
#pragma unroll
                for (int b = 0; b < BMAX; ++b)
                    if (b < len) {
                        const double e = E[b];
                        if constexpr (J0 == 0) {
                            const double e_sq = e * e;
                            sigma2 = sigma2 + e_sq / nd;                                   // :521
                            css = css + e_sq;
                        }
#pragma unroll
                        for (int jj = 0; jj < JN; ++jj) g[J0 + jj] = g[J0 + jj] + D[jj][b] * e;   // :524
                    }
            }
            if constexpr (J0 == 0) {
                sigma2 = __shfl(sigma2, L);
                css = __shfl(css, L);
            }
#pragma unroll
            for (int jj = 0; jj < JN; ++jj) g[J0 + jj] = __shfl(g[J0 + jj], L);
        }
    };
    if constexpr (K > 0) chunk(std::integral_constant<int, 0>{});
    if constexpr (K > KC) chunk(std::integral_constant<int, KC>{});
    css_out = css;
#pragma unroll
    for (int j = 0; j < KA; ++j) g_out[j] = g[j] / -sigma2;                                // :532
    if (sweeps_out) *sweeps_out = sweeps;
}

template <int P, int Q, int I, bool SMEAR>
__device__ __forceinline__ void grad_column_lds(const double *row, int n,
                                                const double (&c)[I + P + Q > 0 ? I + P + Q : 1], int col,
                                                double &css_out, double &g_out) {
    constexpr int M = (P > Q ? P : Q);
    constexpr int PA = P > 0 ? P : 1;
    constexpr int DR = SMEAR ? 1 : (Q > 0 ? Q : 1);     // lag rows 1.. of this column
    double yl[PA];
#pragma unroll
    for (int j = 0; j < PA; ++j) yl[j] = (j < P && M - 1 - j >= 0 && M - 1 - j < n) ? row[M - 1 - j] : 0.0;
    double e1 = 0.0, e2 = 0.0, css = 0.0, sigma2 = 0.0, g = 0.0;
    double dl[DR];                                      // dl[r] = dEdTheta(r + 1, col)
#pragma unroll
    for (int r = 0; r < DR; ++r) dl[r] = 0.0;
    const double yh0 = 0.0 + (double)I * c[0];
    const double nd = (double)n;
#pragma unroll 4
    for (int t = M; t < n; ++t) {
        const double yi = row[t];
        double d0 = 0.0;                                                // dEdTheta(0, col), reset at :528
#pragma unroll
        for (int kk = 0; kk < Q; ++kk) d0 = d0 - c[I + P + kk] * dl[SMEAR ? 0 : kk];   // :492-499
        // the column's own direct term (:503, :506-510, :514-518). Column 0 also gets `- I` in the reference, which
        // for I = 0 subtracts 0.0 (an identity) before its AR term, so one subtraction per column is exact.
        double dv = 0.0;
        if constexpr (I) dv = (col == 0) ? 1.0 : dv;
        double yh = yh0;
#pragma unroll
        for (int j = 0; j < P; ++j) {
            yh = yh + yl[j] * c[I + j];
            dv = (col == I + j) ? yl[j] : dv;
        }
#pragma unroll
        for (int j = 0; j < Q; ++j) {
            const double mj = (j == 0 ? e1 : e2);
            yh = yh + mj * c[I + P + j];
            dv = (col == I + P + j) ? mj : dv;
        }
        d0 = d0 - dv;
        const double e = yi - yh;                                       // :520
        const double e_sq = e * e;
        sigma2 = sigma2 + e_sq / nd;                                    // :521
        css = css + e_sq;
        e2 = e1;                                                        // :522
        e1 = e;
        g = g + d0 * e;                                                 // :524
        if constexpr (Q > 0) {                                          // :526
            if constexpr (SMEAR) {
                dl[0] = d0;
            } else {
#pragma unroll
                for (int r = DR - 1; r >= 1; --r) dl[r] = dl[r - 1];
                dl[0] = d0;
            }
        }
        if constexpr (P > 0) {
#pragma unroll
            for (int j = PA - 1; j >= 1; --j) yl[j] = yl[j - 1];
            yl[0] = yi;
        }
    }
    css_out = css;
    g_out = g / -sigma2;                                                // :532
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
// differs) is generated by random access; rows s+1.. are streamed. An intercept column of ones needs no norm pass
// (its sum of squares is the row count, exactly). The upper triangle of R and the top of
// Q^T y come from re-transforming rows 0..C-1 once more. Back-substitution as Solver.solve.
//
// Gen provides: row_at(r, x, y) (random access), begin(r) (prime the sliding window for streaming from row r),
// first_elem(r) (series index of the element that completes row r), push(v, x, y) (next row from the next
// series element).
// ------------------------------------------------------------------------------------------------------
constexpr int kPrefetchHR = 2;   // 128-B chunks in flight per lane in the Householder passes

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

// the generator's row elements first .. last-1 in order, differenced on the fly when the generator fuses (F) and
// dd = 1; F = false streams rows that are already differenced (dd a compile-time 0)
template <class Gen, class Fn>
__device__ __forceinline__ void gen_stream(const Gen &gen, const double *__restrict__ row, int first, int last,
                                           Fn &&fn) {
    if constexpr (Gen::kFuse) stream_row<kPrefetchHR>(row, gen.dd, first, last, fn);
    else stream_row<kPrefetchHR>(row, 0, first, last, fn);
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
        if constexpr (S == 0 && Gen::kOnesFirst) {
            // column 0 is the intercept's 1.0 in every row: the sequential sum of R ones is R exactly (R < 2^53),
            // so this pass needs no stream
            xnorm = (double)R;
        } else if (S + 1 < R) {
            gen.begin(S + 1);
            gen_stream(gen, row, gen.first_elem(S + 1), n, [&](double v) {
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
            gen_stream(gen, row, gen.first_elem(S + 1), n, [&](double v) {
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
// F (fused differencing): y may be the caller's raw row, differenced on the fly when dd = 1 (stream_row); F = false
// reads rows that are already differenced (dd a compile-time 0, no differencing logic) -- k_hr_init's variant for
// dd = 0, and for the orders whose fused Householder would outgrow the register file (gen_stream, fuse_hr_pays)
template <int m, int INTERCEPT, bool F = true>
struct ARGen {
    static constexpr int C = INTERCEPT + m;
    static constexpr bool kOnesFirst = INTERCEPT != 0;       // column 0 = the intercept's ones
    static constexpr bool kFuse = F;
    const double *__restrict__ y;             // raw row (dd = 1: differenced on the fly) or differenced row (dd = 0)
    int dd = 0;
    double w[m + 1];
    __device__ __forceinline__ double at(int i) const {
        if constexpr (F) return drow_at(y, dd, i);
        else return y[i];
    }
    __device__ __forceinline__ void row_at(int r, double (&x)[C], double &yv) const {
        if constexpr (INTERCEPT) x[0] = 1.0;
#pragma unroll
        for (int l = 1; l <= m; ++l) x[INTERCEPT + l - 1] = at(r + m - l);
        yv = at(r + m);
    }
    __device__ __forceinline__ int first_elem(int r) const { return r + m; }
    __device__ __forceinline__ void begin(int r) {
#pragma unroll
        for (int l = 1; l <= m; ++l) w[l] = at(r + m - l);
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
template <int P, int Q, int I, bool F = true>
struct HRGen {
    static constexpr int M = (P > Q ? P : Q);
    static constexpr int m = M + 1;
    static constexpr int C = I + P + Q;
    static constexpr int QA = Q > 0 ? Q : 1;
    static constexpr bool kOnesFirst = I != 0;
    static constexpr bool kFuse = F;          // as ARGen's F
    const double *__restrict__ y;             // raw row (dd = 1: differenced on the fly) or differenced row (dd = 0)
    int dd = 0;
    double a[m];
    double c;
    double w[m + 2];
    double ew[QA + 1];
    __device__ __forceinline__ double at(int i) const {
        if constexpr (F) return drow_at(y, dd, i);
        else return y[i];
    }
    __device__ __forceinline__ double err_at(int s) const {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < m; ++j) acc = acc + at(s + m - 1 - j) * a[j];
        return at(s + m) - (acc + c);
    }
    __device__ __forceinline__ void row_at(int r, double (&x)[C > 0 ? C : 1], double &yv) const {
        if constexpr (I) x[0] = 1.0;
#pragma unroll
        for (int l = 1; l <= P; ++l) x[I + l - 1] = at(m + r + M - l);
#pragma unroll
        for (int l = 1; l <= Q; ++l) x[I + P + l - 1] = err_at(r + M - l);
        yv = at(m + r + M);
    }
    __device__ __forceinline__ int first_elem(int r) const { return m + M + r; }
    __device__ __forceinline__ void begin(int r) {
        const int e = m + M + r;
#pragma unroll
        for (int l = 1; l <= m + 1; ++l) w[l] = at(e - l);
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

// =======================================================================================================
// least-squares shape checks (commons validateSampleData / Array2DRowRealMatrix), uniform per batch
// =======================================================================================================
__host__ __device__ inline int ols_check(int rows, int ncx, int intercept) {
    if (rows <= 0) return ARIMA_ST_NO_DATA;
    if (ncx + 1 > rows) return ARIMA_ST_NOT_ENOUGH_DATA;
    if (!intercept && ncx == 0) return ARIMA_ST_NO_DATA;
    return ARIMA_ST_OK;
}

// Static outcome of hannanRissanenInit's shapes (ARIMA.scala:216-242) for series of length n.
__host__ __device__ inline int hr_shape_status(int n, int p, int q, int I) {
    const int M = p > q ? p : q, m = M + 1;
    if (n - m < 0) return ARIMA_ST_SERIES_TOO_SHORT;              // Y = ts(m until n)
    int st = ols_check(n - m, m, 1);                               // AR(m) with intercept
    if (st != ARIMA_ST_OK) return st;
    const int nt = n - m;
    if (nt - p < 0 || nt - q < 0) return ARIMA_ST_SERIES_TOO_SHORT;
    int rows = nt - M;
    if (rows < 0) rows = 0;
    return ols_check(rows, p + q, I);
}

__host__ __device__ inline int ar_shape_status(int n, int p, int I) {
    if (n - p < 0) return ARIMA_ST_SERIES_TOO_SHORT;
    return ols_check(n - p, p, I);
}

// =======================================================================================================
// Initial words of the fit kernel's counters and express ring (FitPrep, arima_launch.hpp), written by the kernel
// that runs before k_cg_fit on the same stream (k_hr_init, or k_fit_prep): one dispatch instead of up to six fills
// that queued behind other contexts' persistent fit waves (round 5: 113.6 ms of fill dispatches in a 1 949-ms
// pipelined C2 span, 65 % of it with no fit running; profiles/r05/zc_pipe)
// =======================================================================================================
__device__ __forceinline__ void fit_prep(const FitPrep &fp) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    if (fp.ctl && g < kFitCtlWords) {
        unsigned long long v = 0;
        if (g == 15) v = ~0ull;                  // atomicMin of the kernel's start stamp (timing builds)
        else if (g == 19) v = fp.v19;            // express ring entries of the launch (option "express_ring")
        else if (g == 44) v = fp.v44;            // drain merge threshold ("merge_live")
        else if (g == 45) v = fp.v45;            // donation thresholds ("donate_evals", "donate_evals_drained")
        else if (g == 46) v = fp.v46;
        else if (g == 47) v = fp.v47;            // objective-pass width model ("chain_overhead")
        fp.ctl[g] = v;
    }
    for (int64_t i = g; i < fp.xready_words; i += stride) fp.xready[i] = 0u;
}

// the runtime-order path's optimizer lane (arima_generic.hip): kGenMaxK padded coordinates, the first kdim real
using GenLane = CGLane<kGenMaxK, 0, 0, true, RuntimeDim>;

// ---- runtime-order helpers (arima_generic.hip; css-bobyqa at orders above the compiled ones) -------------------
// a differenced row: element i = raw[i + 1] - raw[i] (dd = 1, fused differencing) or y[i] (dd = 0)
struct GRow {
    const double *y;
    int dd;
    __device__ __forceinline__ double at(int i) const { return drow_at(y, dd, i); }
};

// ---- logLikelihoodCSSARMA's sum of squares (ARIMA.scala:430-445, iterateARMA :581-618, updateMAErrors :544-554) ----
// c has at least one entry (the intercept term multiplies c[0] even when I = 0, as css_pass does with its padded c)
__device__ double gen_css(const GRow &r, int n, int p, int q, int I, const double *c) {
    const int M = p > q ? p : q;
    double e1 = 0.0, e2 = 0.0, css = 0.0;
    const double yh0 = 0.0 + (double)I * c[0];                       // :600
    for (int t = M; t < n; ++t) {
        double yh = yh0;
        for (int j = 0; j < p; ++j) yh = yh + r.at(t - 1 - j) * c[I + j];               // :602-605
        for (int j = 0; j < q; ++j) yh = yh + (j == 0 ? e1 : e2) * c[I + p + j];        // :608-611 (ascending copy)
        const double e = r.at(t) - yh;                                                  // :613
        css = css + e * e;                                                              // :440-442
        e2 = e1;
        e1 = e;
    }
    return css;
}

// ---- ARIMAModel.isStationary / isInvertible (ARIMA.scala:777-815): the step-down of model_flags<P, Q, I> ----------
__device__ bool gen_roots_outside(const double *poly, int N) {
    double a[kGenMaxOrder + 1], b[kGenMaxOrder + 1];
    for (int i = 0; i <= N; ++i) {
        a[i] = poly[i];
        if (!finite(a[i])) return false;
    }
    for (int mm = N; mm >= 1; --mm) {
        const double kk = a[mm];
        if (!(fabs(kk) < 1.0)) return false;
        const double den = 1.0 - kk * kk;
        for (int i = 0; i <= N; ++i) b[i] = (i < mm) ? (a[i] - kk * a[mm - i]) / den : 0.0;
        for (int i = 0; i <= N; ++i) a[i] = b[i];
    }
    return true;
}

__device__ uint8_t gen_model_flags(const double *c, int p, int q, int I) {
    double poly[kGenMaxOrder + 1];
    bool st = true, inv = true;
    if (p > 0) {
        poly[0] = 1.0;
        for (int j = 0; j < p; ++j) poly[1 + j] = -1.0 * c[I + j];
        st = gen_roots_outside(poly, p);
    }
    if (q > 0) {
        poly[0] = 1.0;
        for (int j = 0; j < q; ++j) poly[1 + j] = c[I + p + j];
        inv = gen_roots_outside(poly, q);
    }
    return (uint8_t)((st ? ARIMA_FLAG_STATIONARY : 0) | (inv ? ARIMA_FLAG_INVERTIBLE : 0));
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
