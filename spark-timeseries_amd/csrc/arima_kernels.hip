// arima_kernels.hip — non-template kernels (differencing, generator) and the p-dispatch of the launchers.
// The order-specialised kernels live in arima_kernels_impl.hpp and are instantiated one AR order p per
// translation unit (arima_inst_p0..5.hip) so the build compiles in parallel.
#include "arima_kernels_impl.hpp"

namespace sts {

// =======================================================================================================
// differencing
// =======================================================================================================
constexpr int kMaxD = 16;

// D(i, t) = t < i ? D(i-1, t) : D(i-1, t) - D(i-1, t-1), D(0, t) = ts(t)   (UnivariateTimeSeries.scala:384-480)
// Evaluated per element from the window ts(t-DD..t) with the same subtractions in the same order.
template <int DD>
__device__ __forceinline__ double diff_at(const double *__restrict__ row, int t) {
    double v[DD + 1];
#pragma unroll
    for (int j = 0; j <= DD; ++j) {
        const int tt = t - DD + j;
        v[j] = tt >= 0 ? row[tt] : 0.0;
    }
#pragma unroll
    for (int lvl = 1; lvl <= DD; ++lvl)
#pragma unroll
        for (int j = DD; j >= lvl; --j)           // position t' = t - DD + j; only j >= lvl is ever needed
            if (t - DD + j >= lvl) v[j] = v[j] - v[j - 1];
    return v[DD];
}

template <int DD>
__device__ __forceinline__ void diff_rows(const double *__restrict__ in, int64_t ld_in, double *__restrict__ out,
                                          int64_t ld_out, int64_t N, int T, int drop) {
    for (int64_t i = blockIdx.x; i < N; i += gridDim.x) {
        const double *row = in + i * ld_in;
        double *o = out + i * ld_out;
        for (int t = (drop ? DD : 0) + (int)threadIdx.x; t < T; t += blockDim.x)
            o[drop ? t - DD : t] = diff_at<DD>(row, t);
    }
}

// one workgroup per row (grid-stride over rows), threads over t: coalesced reads and writes
__global__ __launch_bounds__(256) void k_difference(const double *__restrict__ in, int64_t ld_in,
                                                    double *__restrict__ out, int64_t ld_out, int64_t N, int T,
                                                    int d, int drop) {
    switch (d) {
    case 0: diff_rows<0>(in, ld_in, out, ld_out, N, T, drop); break;
    case 1: diff_rows<1>(in, ld_in, out, ld_out, N, T, drop); break;
    case 2: diff_rows<2>(in, ld_in, out, ld_out, N, T, drop); break;
    case 3: diff_rows<3>(in, ld_in, out, ld_out, N, T, drop); break;
    case 4: diff_rows<4>(in, ld_in, out, ld_out, N, T, drop); break;
    case 5: diff_rows<5>(in, ld_in, out, ld_out, N, T, drop); break;
    case 6: diff_rows<6>(in, ld_in, out, ld_out, N, T, drop); break;
    case 7: diff_rows<7>(in, ld_in, out, ld_out, N, T, drop); break;
    case 8: diff_rows<8>(in, ld_in, out, ld_out, N, T, drop); break;
    case 9: diff_rows<9>(in, ld_in, out, ld_out, N, T, drop); break;
    case 10: diff_rows<10>(in, ld_in, out, ld_out, N, T, drop); break;
    case 11: diff_rows<11>(in, ld_in, out, ld_out, N, T, drop); break;
    case 12: diff_rows<12>(in, ld_in, out, ld_out, N, T, drop); break;
    case 13: diff_rows<13>(in, ld_in, out, ld_out, N, T, drop); break;
    case 14: diff_rows<14>(in, ld_in, out, ld_out, N, T, drop); break;
    case 15: diff_rows<15>(in, ld_in, out, ld_out, N, T, drop); break;
    default: diff_rows<16>(in, ld_in, out, ld_out, N, T, drop); break;
    }
}

// inverseDifferencesOfOrderD (UnivariateTimeSeries.scala:489-495): in-place prefix sums, one lane per series
__global__ __launch_bounds__(256) void k_inverse_difference(const double *__restrict__ in, int64_t ld_in,
                                                            double *__restrict__ out, int64_t ld_out,
                                                            int64_t N, int T, int d) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const double *src = in + i * ld_in;
    double *dst = out + i * ld_out;
    for (int t = 0; t < T; ++t) dst[t] = src[t];
    for (int lvl = d; lvl >= 1; --lvl)
        for (int t = lvl; t < T; ++t) dst[t] = dst[t] + dst[t - 1];
}

// =======================================================================================================
// ARIMAModel.forecast (ARIMA.scala:696-764), one lane per series, one streaming pass over the row.
// Every quantity the reference materialises as an array is carried in registers instead:
//   Dc[r]  = D(r, t), the ping-pong differencing column (differencesOfOrderD, :700)
//   Mc[r]  = diffMatrix(r, t) (:731-743): like D except diffMatrix(r, r) copies diffMatrix(r-1, r)
//   xr[j]  = ext(cur-1-j)  (ext = [c]*M ++ diffed, :703-707), hr[j] = hist(cur-1-j) (iterateARMA result :708)
//   sr[j]  = column sums of diffMatrix(0 until d, t-j) (:745-751), delayed d+1 steps to meet hist(M+idx)
// Same operations in the same order as the oracle's restatement (oracle/arima_oracle.c orc_forecast), so the
// result is bit-identical. The final inverseDifferencesOfOrderD over [T-d, T+nFuture) runs in place on the
// lane's own output row.
//
// Memory path (round 2): one wave per workgroup, 64 series. The wave reads its 64 rows as a [64 x kFcCh]
// tile with coalesced loads (kFcCh consecutive doubles of 64/kFcCh rows per instruction, the next tile
// prefetched into registers while this one is consumed) and transposes it through LDS, so each lane steps
// through its own series from LDS. Outputs [0, T-d) go the other way: every lane writes the same output
// index at the same step (T and d are uniform), into the same LDS ring (the consumed input's column); after each tile the
// indices no later step can touch (< tile end - d: index x is written at step x or x + d) leave as coalesced
// row segments. [T-d, T + nFuture) (the diffMatrix diagonal, the forecasts and their re-integration, ≤ 3 % of
// the bytes) is written by the lane itself, as before.
// Tiles are phase-shifted by d (round 3): tile k covers steps [d + (k-1) kFcCh, d + k kFcCh), so after it exactly the
// outputs below k kFcCh are final and every flush is a whole kFcCh-element segment at a kFcCh boundary -- with a
// 128-B aligned output row stride (ld_out % 16 == 0) each one is two full 128-B lines per row instead of a segment
// straddling three (the round-2 kernel wrote 1.18x its output bytes).
// =======================================================================================================
constexpr int kFcMaxOrder = 5;   // p, q <= 5 (check_orders)
constexpr int kFcMaxD = 8;
constexpr int kFcWave = 64;
constexpr int kFcCh = 32;                                            // time steps per tile
constexpr int kFcRing = kFcCh + kFcMaxD;                             // LDS ring columns (>= kFcCh + kFcMaxD)
constexpr int kFcRowsPerLd = kFcWave / kFcCh;                        // rows per coalesced load instruction
static_assert(kFcRing >= kFcCh + kFcMaxD, "output ring too small");
static_assert(kFcWave % kFcCh == 0, "tile width must divide the wave");

template <int DD, int MM>
__global__ __launch_bounds__(kFcWave) void k_forecast(const double *__restrict__ ts_all, int64_t ld_in,
                                                      const double *__restrict__ coef_all, int k,
                                                      double *__restrict__ out_all, int64_t ld_out, int64_t N,
                                                      int T, int p, int q, int I, int nF) {
    constexpr int d = DD;                                              // d templated: register arrays sized to it
    constexpr int kD = DD > 0 ? DD : 1;
    constexpr int kM = MM > 0 ? MM : 1;                                // max(p, q) templated as well
    // one LDS ring of kFcRing columns per row: the input tile of steps [cb, cb + kFcCh) sits in columns
    // (cb + u) mod kFcRing; output index x (written at step x or x + d, after input x was consumed) goes to
    // column x mod kFcRing until it is flushed. Pending outputs [cb - d, cb) and the tile never overlap
    // because kFcRing >= kFcCh + kFcMaxD.
    __shared__ double ring[kFcWave][kFcRing + 1];
    const int lane = (int)threadIdx.x;
    const int64_t row0 = (int64_t)blockIdx.x * kFcWave;
    const int64_t sid = row0 + lane;
    const bool live = sid < N;
    double *out = out_all + (live ? sid : N - 1) * ld_out;
    constexpr int M = MM;
    // coefficients [c?, phi_1..phi_p, theta_1..theta_q] (ARIMA.scala:74-77); k == 0 reads nothing
    const double *cf = coef_all + (live ? sid : N - 1) * k;
    const double c0 = k > 0 ? cf[0] : 0.0;
    double phi[kM], th[kM];
#pragma unroll
    for (int j = 0; j < MM; ++j) {
        phi[j] = j < p ? cf[I + j] : 0.0;
        th[j] = j < q ? cf[I + p + j] : 0.0;
    }
    const double ia = I ? c0 : 0.0;
    double xr[kM], hr[kM], ma[kM];
#pragma unroll
    for (int j = 0; j < MM; ++j) { xr[j] = ia; hr[j] = 0.0; ma[j] = 0.0; }
    double Dc[DD + 1], Dp[DD + 1], Mc[kD], Mp[kD], sr[DD + 2];
#pragma unroll
    for (int r = 0; r <= DD; ++r) { Dc[r] = 0.0; Dp[r] = 0.0; }
#pragma unroll
    for (int r = 0; r < kD; ++r) { Mc[r] = 0.0; Mp[r] = 0.0; }
#pragma unroll
    for (int j = 0; j < DD + 2; ++j) sr[j] = 0.0;

    const int lim = T - d;                                             // LDS-staged output indices [0, lim)
    auto put = [&](int idx, double val) {
        if (idx < lim) ring[lane][idx % kFcRing] = val;   // idx is wave-uniform
        else if (live) out[idx] = val;
    };
    // tile loads: lane reads element tu of row j * kFcRowsPerLd + tr; clamped addresses, so the loads are
    // unconditional (values outside [0, N) x [0, T) are never consumed)
    const int tu = lane % kFcCh, tr = lane / kFcCh;
    double pf[kFcCh];
    auto load_tile = [&](int cb) {
        const int tt = cb + tu < T ? cb + tu : T - 1;
        const int t = tt < 0 ? 0 : tt;                                 // the first tile starts before t = 0
#pragma unroll
        for (int j = 0; j < kFcCh; ++j) {
            const int64_t gi = row0 + j * kFcRowsPerLd + tr;
            pf[j] = ts_all[(gi < N ? gi : N - 1) * ld_in + t];
        }
    };
    int flushed = 0;                                                   // [0, flushed) is in HBM
    const int cb0 = d - kFcCh;                                         // first tile: steps [0, d)
    if (T > 0) load_tile(cb0);
    for (int cb = cb0; cb < T; cb += kFcCh) {
        __syncthreads();                                               // last tile's reads and flush done
        if (cb + tu >= 0) {
#pragma unroll
            for (int j = 0; j < kFcCh; ++j) ring[j * kFcRowsPerLd + tr][(cb + tu) % kFcRing] = pf[j];
        }
        __syncthreads();
        if (cb + kFcCh < T) load_tile(cb + kFcCh);
        const int ce = cb + kFcCh < T ? cb + kFcCh : T;
#pragma unroll 1
        for (int t = cb < 0 ? 0 : cb; t < ce; ++t) {
            const double v = ring[lane][t % kFcRing];
            // differencing column t (UnivariateTimeSeries.scala:384-405 pass r: out(t) = in(t) - in(t-1) for t >= r)
            Dc[0] = v;
#pragma unroll
            for (int r = 1; r <= DD; ++r)
                if (r <= d) Dc[r] = t < r ? Dc[r - 1] : Dc[r - 1] - Dp[r - 1];
            // diffMatrix column t and its column sum (d > 0 only)
            double s = 0.0;
            if (d > 0) {
                Mc[0] = v;
#pragma unroll
                for (int r = 1; r < DD; ++r)
                    if (r < d) Mc[r] = t < r ? 0.0 : (t == r ? Mc[r - 1] : Mc[r - 1] - Mp[r - 1]);
#pragma unroll
                for (int r = 0; r < kD; ++r)
                    if (r < d) s = s + Mc[r];
#pragma unroll
                for (int j = DD + 1; j >= 1; --j) sr[j] = sr[j - 1];
                sr[0] = s;
#pragma unroll
                for (int r = 0; r < kD; ++r) Mp[r] = Mc[r];
            }
#pragma unroll
            for (int r = 0; r <= DD; ++r) Dp[r] = Dc[r];
            if (t < d) put(t, v);                                      // :724
            if (t >= d) {
                // iterateARMA(ext, hist, +, goldStandard = ext) step at ext index M + i, i = t - d (:708, :581-618)
                const int i = t - d;
                const double y = Dc[d];
                double f = 0.0;
                f = f + (double)I * c0;
#pragma unroll
                for (int j = 0; j < MM; ++j)
                    if (j < p) f = f + xr[j] * phi[j];
#pragma unroll
                for (int j = 0; j < MM; ++j)
                    if (j < q) f = f + ma[j] * th[j];
                const double err = y - f;
#pragma unroll
                for (int j = MM - 1; j >= 1; --j)             // updateMAErrors (:544-554): smear
                    if (j < q) ma[j] = ma[0];
                if (q > 0) ma[0] = err;
#pragma unroll
                for (int j = MM - 1; j >= 1; --j) { xr[j] = xr[j - 1]; hr[j] = hr[j - 1]; }
                xr[0] = y;
                hr[0] = f;
                if (d == 0) {
                    put(i, f);                                         // :726
                } else if (i >= d && i < T - d) {
                    double sd = 0.0;                                   // column sum at i - 1 = t - d - 1
#pragma unroll
                    for (int j = 0; j < DD + 2; ++j)
                        if (j == d + 1) sd = sr[j];
                    put(i, sd + f);                                    // :745-751
                }
            }
            if (d > 0 && t >= T - d) {                                 // diag(diffMatrix(0 until d, -d to -1))
                const int r = t - (T - d);
                double dg = 0.0;
#pragma unroll
                for (int j = 0; j < DD; ++j)
                    if (j == r) dg = Mc[j];
                put(t, dg);
            }
        }
        __syncthreads();                                               // ring entries of every lane written
        const int fe = ce - d < lim ? ce - d : lim;                    // indices < fe are final
        if (fe > flushed) {
            const int idx = flushed + tu;
            if (idx < fe) {
#pragma unroll
                for (int j = 0; j < kFcCh; ++j) {
                    const int r = j * kFcRowsPerLd + tr;
                    if (row0 + r < N) out_all[(row0 + r) * ld_out + idx] = ring[r][idx % kFcRing];
                }
            }
            flushed = fe;
        }
    }
    if (!live) return;
    // forward = hist(-M..) ++ zeros(nFuture); iterateARMA(forward, forward, +, gold = forward, maTerms) (:711-720)
    double fr[kM], mt[kM];
#pragma unroll
    for (int j = 0; j < MM; ++j) {
        fr[j] = hr[j];                                                 // fwd(i-1-j)
        mt[j] = 0.0;
    }
#pragma unroll
    for (int j = 0; j < MM; ++j)                              // maTerms(j) = ext(L-M+j) - hist(L-M+j)
        if (j < M) {
            double xv = 0.0, hv = 0.0;
#pragma unroll
            for (int jj = 0; jj < MM; ++jj)
                if (jj == M - 1 - j) { xv = xr[jj]; hv = hr[jj]; }
            mt[j] = xv - hv;
        }
    double *fo = out + T;
    for (int i = 0; i < nF; ++i) {
        double f = 0.0;
        f = f + (double)I * c0;
#pragma unroll
        for (int j = 0; j < MM; ++j)
            if (j < p) f = f + fr[j] * phi[j];
#pragma unroll
        for (int j = 0; j < MM; ++j)
            if (j < q) f = f + mt[j] * th[j];
        const double err = f - f;
#pragma unroll
        for (int j = MM - 1; j >= 1; --j)                     // updateMAErrors over maTerms' length M
            if (j < M) mt[j] = mt[0];
        if (M > 0) mt[0] = err;
#pragma unroll
        for (int j = MM - 1; j >= 1; --j) fr[j] = fr[j - 1];
        fr[0] = f;
        fo[i] = f;                                                     // :728
    }
    if (d > 0) {                                                       // inverseDifferencesOfOrderD (:756-761)
        double *w = out + (T - d);
        const int L = d + nF;
        for (int lvl = d; lvl >= 1; --lvl)
            for (int j = lvl; j < L; ++j) w[j] = w[j] + w[j - 1];
    }
}

// =======================================================================================================
// Order search: keep, per series, the min-approxAIC model among the fits
// that succeeded and are stationary and invertible (the filter of ARIMA.autoFit, ARIMA.scala:342).
// approxAIC (ARIMA.scala:826-830) = -2 * logLikelihoodCSS(ts) + 2 * (p + q + interceptTerm), the second term
// an Int. Candidates arrive in (d, p, q, intercept) lexicographic order; strict < keeps the first on ties.
// =======================================================================================================
constexpr int kSearchK = 11;   // 1 + 5 + 5

__global__ __launch_bounds__(256) void k_search_init(double *__restrict__ best_aic, int32_t *__restrict__ order,
                                                     double *__restrict__ coef, int64_t N) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    best_aic[i] = __builtin_inf();
    for (int j = 0; j < 4; ++j) order[i * 4 + j] = -1;
    for (int j = 0; j < kSearchK; ++j) coef[i * kSearchK + j] = __builtin_nan("");
}

// position of (p, d, q, I) in the grid's (d, p, q, intercept) order; an empty best (order -1) sorts last
__device__ __forceinline__ int search_key(int p, int d, int q, int I) { return ((d * 16 + p) * 16 + q) * 2 + I; }
__device__ __forceinline__ int search_key(const int32_t *o) {
    return o[0] < 0 ? 0x7fffffff : search_key(o[0], o[1], o[2], o[3]);
}

__global__ __launch_bounds__(256) void k_search_select(const double *__restrict__ cand_coef,
                                                       const double *__restrict__ cand_ll,
                                                       const int32_t *__restrict__ cand_status,
                                                       const uint8_t *__restrict__ cand_flags, int64_t N, int p,
                                                       int d, int q, int I,
                                                       const unsigned long long *__restrict__ fit_ctl,
                                                       double *__restrict__ best_aic,
                                                       int32_t *__restrict__ order, double *__restrict__ coef) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    if (fit_ctl && fit_ctl[26] != 0) return;     // the fit kernel dropped series (watchdog): no candidate is valid
    if (cand_status[i] != ARIMA_ST_OK) return;
    if ((cand_flags[i] & (ARIMA_FLAG_STATIONARY | ARIMA_FLAG_INVERTIBLE)) !=
        (ARIMA_FLAG_STATIONARY | ARIMA_FLAG_INVERTIBLE))
        return;
    const int k = I + p + q;
    const double aic = -2.0 * cand_ll[i] + (double)(2 * k);
    // autoFit keeps `_ < curBestAIC` with curBestAIC = Double.MaxValue at the start (ARIMA.scala:323, :344): a
    // +inf or NaN approxAIC never qualifies, not even against the empty best
    if (!(aic < 1.7976931348623157e308)) return;
    // the first minimum in (d, p, q, intercept) order wins (minBy), whatever order the candidates arrive in; the
    // grid-position tie-break applies only against a real candidate
    const double b = best_aic[i];
    const bool have = order[i * 4] >= 0;
    if (have && !(aic < b) && !(aic == b && search_key(p, d, q, I) < search_key(order + i * 4))) return;
    best_aic[i] = aic;
    order[i * 4 + 0] = p;
    order[i * 4 + 1] = d;
    order[i * 4 + 2] = q;
    order[i * 4 + 3] = I;
    for (int j = 0; j < kSearchK; ++j) coef[i * kSearchK + j] = j < k ? cand_coef[i * k + j] : 0.0;
}

// the lanes' bests -> the call's outputs, by the same rule (approxAIC, then grid position)
__global__ __launch_bounds__(256) void k_search_merge(const SearchBests b, int lanes, int64_t N,
                                                      double *__restrict__ best_aic, int32_t *__restrict__ order,
                                                      double *__restrict__ coef) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    int w = -1;
    double wa = __builtin_inf();
    int wk = 0x7fffffff;
    for (int l = 0; l < lanes; ++l) {
        const int32_t *o = b.order[l] + i * 4;
        if (o[0] < 0) continue;
        const double a = b.aic[l][i];
        if (!(a < 1.7976931348623157e308)) continue;    // never stored by k_search_select; kept for symmetry
        const int key = search_key(o);
        if (w < 0 || a < wa || (a == wa && key < wk)) {
            w = l;
            wa = a;
            wk = key;
        }
    }
    best_aic[i] = w < 0 ? __builtin_inf() : wa;
    for (int j = 0; j < 4; ++j) order[i * 4 + j] = w < 0 ? -1 : b.order[w][i * 4 + j];
    for (int j = 0; j < kSearchK; ++j) coef[i * kSearchK + j] = w < 0 ? __builtin_nan("") : b.coef[w][i * kSearchK + j];
}

int launch_search_merge(const SearchBests &b, int lanes, int64_t N, double *best_aic, int32_t *order, double *coef,
                        hipStream_t s) {
    if (N == 0) return ARIMA_OK;
    if (lanes < 1 || lanes > kSearchMaxLanes) return ARIMA_E_INVALID_ARG;
    hipLaunchKernelGGL(k_search_merge, dim3(grid_for(N, 256)), dim3(256), 0, s, b, lanes, N, best_aic, order, coef);
    STS_CHECK_LAUNCH();
    return ARIMA_OK;
}

int launch_search_init(double *best_aic, int32_t *order, double *coef, int64_t N, hipStream_t s) {
    if (N == 0) return ARIMA_OK;
    hipLaunchKernelGGL(k_search_init, dim3(grid_for(N, 256)), dim3(256), 0, s, best_aic, order, coef, N);
    STS_CHECK_LAUNCH();
    return ARIMA_OK;
}

int launch_search_select(const double *cand_coef, const double *cand_ll, const int32_t *cand_status,
                         const uint8_t *cand_flags, int64_t N, int p, int d, int q, int I,
                         const unsigned long long *fit_ctl, double *best_aic, int32_t *order, double *coef,
                         hipStream_t s) {
    if (N == 0) return ARIMA_OK;
    if (I + p + q > kSearchK) return ARIMA_E_UNSUPPORTED;
    hipLaunchKernelGGL(k_search_select, dim3(grid_for(N, 256)), dim3(256), 0, s, cand_coef, cand_ll, cand_status,
                       cand_flags, N, p, d, q, I, fit_ctl, best_aic, order, coef);
    STS_CHECK_LAUNCH();
    return ARIMA_OK;
}

// =======================================================================================================
// Synthetic generator: ARIMAModel.sample (ARIMA.scala:655-678) with per-series jittered coefficients
// =======================================================================================================
constexpr int kSampleMaxOrder = kGenMaxOrder;   // every order the library fits
struct SampleCoef {
    double c[1 + 2 * kSampleMaxOrder];
};

__device__ bool sample_roots_ok(const double *poly, int N) {   // runtime-order Schur-Cohn (see model_flags)
    double a[kSampleMaxOrder + 1], b[kSampleMaxOrder + 1];
    for (int i = 0; i <= N; ++i) a[i] = poly[i];
    for (int mm = N; mm >= 1; --mm) {
        const double kk = a[mm];
        if (!(fabs(kk) < 1.0)) return false;
        const double den = 1.0 - kk * kk;
        for (int i = 0; i < mm; ++i) b[i] = (a[i] - kk * a[mm - i]) / den;
        for (int i = 0; i < mm; ++i) a[i] = b[i];
    }
    return true;
}

__global__ __launch_bounds__(256) void k_sample(double *__restrict__ out, int64_t ld, int64_t N, int T, int p,
                                                int d, int q, int I, const SampleCoef base_arg,
                                                double jitter, uint64_t seed, int64_t first) {
    const double *base = base_arg.c;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const uint64_t gsid = (uint64_t)(first + i);
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const int K = I + p + q, M = p > q ? p : q;
    double c[1 + 2 * kSampleMaxOrder];
    for (int j = 0; j < K; ++j) c[j] = base[j];
    for (int attempt = 0; attempt < 16; ++attempt) {
        double trial[1 + 2 * kSampleMaxOrder];
        for (int j = 0; j < K; j += 2) {
            uint32_t ctr[4] = {(uint32_t)j, (uint32_t)gsid, (uint32_t)(gsid >> 32), 0x5A17u + (uint32_t)attempt};
            philox4x32_10(ctr, k0 ^ 0x3C6EF372u, k1 ^ 0xA54FF53Au);
            trial[j] = base[j] + jitter * (2.0 * u01_53(ctr[0], ctr[1]) - 1.0);
            if (j + 1 < K) trial[j + 1] = base[j + 1] + jitter * (2.0 * u01_53(ctr[2], ctr[3]) - 1.0);
        }
        double poly[kSampleMaxOrder + 1];
        poly[0] = 1.0;
        for (int j = 0; j < p; ++j) poly[1 + j] = -trial[I + j];
        bool ok = sample_roots_ok(poly, p);
        for (int j = 0; j < q; ++j) poly[1 + j] = trial[I + p + j];
        ok = ok && sample_roots_ok(poly, q);
        if (ok) {
            for (int j = 0; j < K; ++j) c[j] = trial[j];
            break;
        }
    }
    // addTimeDependentEffects(noise): changes = [c]*M ++ noise; iterateARMA(changes, changes, +, errors = copy)
    const double ia = (I && K > 0) ? c[0] : 0.0;
    double hist[kSampleMaxOrder];   // hist[j] = changes(i - 1 - j)
    double ma[kSampleMaxOrder];
    for (int j = 0; j < kSampleMaxOrder; ++j) { hist[j] = ia; ma[j] = 0.0; }
    double *row = out + i * ld;
    double z1 = 0.0;
    for (int t = 0; t < T; ++t) {
        double z;
        if ((t & 1) == 0) {
            uint32_t ctr[4] = {(uint32_t)(t >> 1), (uint32_t)gsid, (uint32_t)(gsid >> 32), 0xB0B0u};
            philox4x32_10(ctr, k0, k1);
            const double u1 = 1.0 - u01_53(ctr[0], ctr[1]);           // (0, 1]
            const double u2 = u01_53(ctr[2], ctr[3]);
            const double r = sqrt(-2.0 * log(u1));
            const double ang = 6.283185307179586 * u2;
            z = r * cos(ang);
            z1 = r * sin(ang);
        } else {
            z = z1;
        }
        double v = z;                                     // dest(i) starts as the noise value
        v = v + (double)I * (K > 0 ? c[0] : 0.0);     // `intercept * coefficients(0)` (K = 0: pure noise)
        for (int j = 0; j < p; ++j) v = v + hist[j] * c[I + j];
        for (int j = 0; j < q; ++j) v = v + ma[j] * c[I + p + j];
        for (int j = 0; j < q - 1; ++j) ma[j + 1] = ma[j];     // updateMAErrors (ascending copy)
        if (q > 0) ma[0] = z;                                  // error = errors(i) = the noise
        for (int j = (M > 0 ? M : 1) - 1; j >= 1; --j) hist[j] = hist[j - 1];
        hist[0] = v;
        row[t] = v;
    }
    for (int lvl = d; lvl >= 1; --lvl)                             // inverseDifferencesOfOrderD
        for (int t = lvl; t < T; ++t) row[t] = row[t] + row[t - 1];
}


// =======================================================================================================
// launchers
// =======================================================================================================
int launch_difference(const double *in, int64_t ld_in, double *out, int64_t ld_out, int64_t N, int T, int d,
                      int drop, hipStream_t s) {
    if (d > kMaxD) return ARIMA_E_UNSUPPORTED;
    if (N == 0 || T == 0) return ARIMA_OK;
    const unsigned grid = (unsigned)(N < 65536 * 4 ? N : 65536 * 4);
    hipLaunchKernelGGL(k_difference, dim3(grid), dim3(256), 0, s, in, ld_in, out, ld_out, N, T, d, drop);
    STS_CHECK_LAUNCH();
    return ARIMA_OK;
}

int launch_inverse_difference(const double *in, int64_t ld_in, double *out, int64_t ld_out, int64_t N, int T,
                              int d, hipStream_t s) {
    if (N == 0) return ARIMA_OK;
    hipLaunchKernelGGL(k_inverse_difference, dim3(grid_for(N, 256)), dim3(256), 0, s, in, ld_in, out, ld_out, N,
                       T, d);
    STS_CHECK_LAUNCH();
    return ARIMA_OK;
}

int launch_forecast(const double *ts, int64_t ld_in, const double *coef, int k, double *out, int64_t ld_out,
                    int64_t N, int T, int p, int d, int q, int I, int n_future, hipStream_t s) {
    if (N == 0) return ARIMA_OK;
    if (p > kFcMaxOrder || q > kFcMaxOrder || d > kFcMaxD) return ARIMA_E_UNSUPPORTED;
    if (T < d || n_future < 0 || k != I + p + q || ld_out < (int64_t)T + n_future) return ARIMA_E_INVALID_ARG;
    const dim3 grid(grid_for(N, kFcWave)), block(kFcWave);
    const int M = p > q ? p : q;
    switch (d * (kFcMaxOrder + 1) + M) {
#define STS_FC_CASE(D, MM)                                                                                          \
    case D * (kFcMaxOrder + 1) + MM:                                                                                \
        hipLaunchKernelGGL((k_forecast<D, MM>), grid, block, 0, s, ts, ld_in, coef, k, out, ld_out, N, T, p, q, I, \
                           n_future);                                                                               \
        break;
#define STS_FC_CASES(D) STS_FC_CASE(D, 0) STS_FC_CASE(D, 1) STS_FC_CASE(D, 2) STS_FC_CASE(D, 3) STS_FC_CASE(D, 4)    \
    STS_FC_CASE(D, 5)
    STS_FC_CASES(0) STS_FC_CASES(1) STS_FC_CASES(2) STS_FC_CASES(3) STS_FC_CASES(4) STS_FC_CASES(5) STS_FC_CASES(6)
    STS_FC_CASES(7) STS_FC_CASES(8)
#undef STS_FC_CASES
#undef STS_FC_CASE
    }
    STS_CHECK_LAUNCH();
    return ARIMA_OK;
}

int launch_sample(double *out, int64_t ld, int64_t N, int T, int p, int d, int q, int I, const double *base_host,
                  double jitter, uint64_t seed, int64_t first, hipStream_t s) {
    if (N == 0) return ARIMA_OK;
    if (p > kSampleMaxOrder || q > kSampleMaxOrder) return ARIMA_E_UNSUPPORTED;
    SampleCoef base{};                          // by value: no host buffer outlives the call
    for (int j = 0; j < I + p + q; ++j) base.c[j] = base_host[j];
    hipLaunchKernelGGL(k_sample, dim3(grid_for(N, 256)), dim3(256), 0, s, out, ld, N, T, p, d, q, I, base, jitter,
                       seed, first);
    STS_CHECK_LAUNCH();
    return ARIMA_OK;
}

#ifdef STS_DEV
STS_DECLARE_P(STS_DEV_P, extern)
#define STS_P_SWITCH(CALL)                                                                                 \
    if (p == STS_DEV_P) return CALL(STS_DEV_P);                                                            \
    return ARIMA_E_UNSUPPORTED;
#else
STS_DECLARE_P(0, extern)
STS_DECLARE_P(1, extern)
STS_DECLARE_P(2, extern)
STS_DECLARE_P(3, extern)
STS_DECLARE_P(4, extern)
STS_DECLARE_P(5, extern)

#define STS_P_SWITCH(CALL)                                                                                 \
    switch (p) {                                                                                           \
    case 0: return CALL(0);                                                                                \
    case 1: return CALL(1);                                                                                \
    case 2: return CALL(2);                                                                                \
    case 3: return CALL(3);                                                                                \
    case 4: return CALL(4);                                                                                \
    case 5: return CALL(5);                                                                                \
    default: return ARIMA_E_UNSUPPORTED;                                                                   \
    }
#endif

// one dispatch that prepares a fit kernel's counters and ring when no k_hr_init runs before it (FitPrep)
__global__ __launch_bounds__(256) void k_fit_prep(FitPrep prep) { fit_prep(prep); }

int launch_fit_prep(const FitPrep &prep, hipStream_t s) {
    const int64_t words = std::max<int64_t>(prep.xready_words, kFitCtlWords);
    const unsigned grid = (unsigned)std::min<int64_t>(grid_for(words, 256), 128);
    hipLaunchKernelGGL(k_fit_prep, dim3(grid), dim3(256), 0, s, prep);
    STS_CHECK_LAUNCH();
    return ARIMA_OK;
}

int launch_hr_init(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, double *init_out,
                   int32_t *status_out, hipStream_t s, int hr_grid, int dd, const FitPrep &prep) {
    if (N == 0) return launch_fit_prep(prep, s);
    if (gen_order(p, q)) return launch_gen_hr_init(y, ld, n, N, p, q, I, init_out, status_out, dd, prep, s);
#define C_(PP) launch_hr_init_P<PP>(y, ld, n, N, q, I, init_out, status_out, s, hr_grid, dd, prep)
    STS_P_SWITCH(C_)
#undef C_
}

int launch_ar_fit(const double *y, int64_t ld, int n, int64_t N, int p, int I, double *coef_out, double *ll_out,
                  int32_t *status_out, int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out,
                  hipStream_t s, int dd) {
    if (N == 0) return ARIMA_OK;
    if (gen_order(p, 0))
        return launch_gen_ar_fit(y, ld, n, N, p, I, coef_out, ll_out, status_out, n_eval_out, n_grad_out, flags_out, dd,
                                 s);
#define C_(PP) launch_ar_fit_P<PP>(y, ld, n, N, I, coef_out, ll_out, status_out, n_eval_out, n_grad_out, flags_out, s, dd)
    STS_P_SWITCH(C_)
#undef C_
}

int launch_cg_fit(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, int smear,
                  const double *init, const int32_t *init_status, double *coef_out, double *ll_out,
                  int32_t *status_out, int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out,
                  unsigned long long *ctl, int grid_blocks, int express_blocks, unsigned char *xq, unsigned *xready,
                  int join_express, hipStream_t s, int dd) {
    if (N == 0) return ARIMA_OK;
#define C_(PP)                                                                                             \
    launch_cg_fit_P<PP>(y, ld, n, N, q, I, smear, init, init_status, coef_out, ll_out, status_out, n_eval_out, \
                        n_grad_out, flags_out, ctl, grid_blocks, express_blocks, xq, xready, join_express, s, dd)
    STS_P_SWITCH(C_)
#undef C_
}

int cg_fit_series_per_block(int p, int q, int I) {
#define C_(PP) cg_fit_series_per_block_P<PP>(q, I)
    STS_P_SWITCH(C_)
#undef C_
}

int launch_css_loglik(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, const double *coef,
                      double *ll_out, hipStream_t s) {
    if (N == 0) return ARIMA_OK;
    if (gen_order(p, q)) return launch_gen_css_loglik(y, ld, n, N, p, q, I, coef, ll_out, s);
#define C_(PP) launch_css_loglik_P<PP>(y, ld, n, N, q, I, coef, ll_out, s)
    STS_P_SWITCH(C_)
#undef C_
}

int launch_css_grad(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, int smear,
                    const double *coef, double *g_out, hipStream_t s) {
    if (N == 0) return ARIMA_OK;
    if (gen_order(p, q)) return launch_gen_css_grad(y, ld, n, N, p, q, I, smear, coef, g_out, s);
#define C_(PP) launch_css_grad_P<PP>(y, ld, n, N, q, I, smear, coef, g_out, s)
    STS_P_SWITCH(C_)
#undef C_
}

int launch_model_flags(const double *coef, int64_t N, int p, int q, int I, uint8_t *flags_out, hipStream_t s) {
    if (N == 0) return ARIMA_OK;
    if (gen_order(p, q)) return launch_gen_model_flags(coef, N, p, q, I, flags_out, s);
#define C_(PP) launch_model_flags_P<PP>(coef, N, q, I, flags_out, s)
    STS_P_SWITCH(C_)
#undef C_
}

int hr_shape_status_host(int n, int p, int q, int I) { return hr_shape_status(n, p, q, I); }
int ar_shape_status_host(int n, int p, int I) { return ar_shape_status(n, p, I); }

}  // namespace sts
