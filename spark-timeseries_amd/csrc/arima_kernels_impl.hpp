#pragma once
// arima_kernels_impl.hpp — HIP kernel templates of the MI355X batched ARIMA (CSS-CGD) engine (gfx950).
//
// Kernels (one series per lane everywhere; DESIGN.md has the data layout and the roofline of each):
//   k_difference          differencesOfOrderD (+ .drop(d)) into a 128-B-aligned series-major workspace
//   k_inverse_difference  inverseDifferencesOfOrderD
//   k_hr_init             ARIMA.hannanRissanenInit: two streaming-Householder least squares per lane
//   k_ar_fit              ARIMA.fitModel's AR-only shortcut (p > 0, q == 0): Autoregression.fitModel + CSS
//   k_cg_fit              persistent fit kernel: per-lane FR-CG / bracket / Brent state machine, one CSS or
//                         CSS+gradient pass over every lane's own series per wave iteration, lanes refill
//                         from a device work counter when their series finishes
//   k_css_loglik / k_css_grad / k_model_flags   building blocks (parity tests, the Python mirror)
//   k_sample              ARIMAModel.sample-style synthetic generator (Philox4x32-10 + Box-Muller)
#include <hip/hip_runtime.h>

#include <utility>

#include "arima_device.hpp"
#include "arima_launch.hpp"
#include <type_traits>

namespace sts {

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
// Hannan-Rissanen init (ARIMA.scala:216-242)
// =======================================================================================================
template <int P, int Q, int I>
__global__ __launch_bounds__(256) void k_hr_init(const double *__restrict__ y, int64_t ld, int n, int64_t N,
                                                 double *__restrict__ init_out, int32_t *__restrict__ status_out) {
    constexpr int K = I + P + Q;
    constexpr int KA = K > 0 ? K : 1;
    constexpr int M = P > Q ? P : Q;
    constexpr int m = M + 1;
    const int64_t sid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sid >= N) return;
    const double *row = y + sid * ld;
    int st = hr_shape_status(n, P, Q, I);
    double beta[KA];
#pragma unroll
    for (int j = 0; j < KA; ++j) beta[j] = __builtin_nan("");
    if (st == ARIMA_ST_OK) {
        double ab[1 + m];
        ARGen<m, 1> genA;
        genA.y = row;
        st = stream_ols<1 + m>(genA, row, n, n - m, ab);           // Autoregression.fitModel(y, m)  :225
        if (st == ARIMA_ST_OK) {
            HRGen<P, Q, I> genB;
            genB.y = row;
            genB.c = ab[0];
#pragma unroll
            for (int j = 0; j < m; ++j) genB.a[j] = ab[1 + j];
            double bb[KA];
            if constexpr (K > 0) {
                st = stream_ols<K>(genB, row, n, n - m - M, bb);   // :237-240
                if (st == ARIMA_ST_OK) {
#pragma unroll
                    for (int j = 0; j < K; ++j) beta[j] = bb[j];
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < K; ++j) init_out[sid * K + j] = beta[j];
    status_out[sid] = st;
}

// =======================================================================================================
// AR-only shortcut of fitModel (ARIMA.scala:90-96): Autoregression.fitModel(diffed, p, !includeIntercept)
// =======================================================================================================
template <int P, int I>
__global__ __launch_bounds__(256) void k_ar_fit(const double *__restrict__ y, int64_t ld, int n, int64_t N,
                                                double *__restrict__ coef_out, double *__restrict__ ll_out,
                                                int32_t *__restrict__ status_out, int32_t *__restrict__ n_eval_out,
                                                int32_t *__restrict__ n_grad_out, uint8_t *__restrict__ flags_out) {
    constexpr int K = I + P;
    const int64_t sid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sid >= N) return;
    const double *row = y + sid * ld;
    int st = ar_shape_status(n, P, I);
    double beta[K];
#pragma unroll
    for (int j = 0; j < K; ++j) beta[j] = __builtin_nan("");
    double ll = __builtin_nan("");
    uint8_t fl = 0;
    if (st == ARIMA_ST_OK) {
        double b[K];
        ARGen<P, I> gen;
        gen.y = row;
        st = stream_ols<K>(gen, row, n, n - P, b);
        if (st == ARIMA_ST_OK) {
#pragma unroll
            for (int j = 0; j < K; ++j) beta[j] = b[j];
            double css, g[K];
            css_pass<P, 0, I, false, false>(row, n, beta, css, g);
            ll = css_to_loglik(css, n);
            fl = model_flags<P, 0, I>(beta);
        }
    }
#pragma unroll
    for (int j = 0; j < K; ++j) coef_out[sid * K + j] = beta[j];
    ll_out[sid] = ll;
    status_out[sid] = st;
    if (n_eval_out) n_eval_out[sid] = 0;
    if (n_grad_out) n_grad_out[sid] = 0;
    if (flags_out) flags_out[sid] = fl;
}

// =======================================================================================================
// Persistent CSS-CGD fit kernel
// =======================================================================================================
template <int K>
__device__ __forceinline__ void write_fit(int64_t sid, int status, const double (&coef)[K], double ll, int n_eval,
                                          int n_grad, uint8_t flags, double *coef_out, double *ll_out,
                                          int32_t *status_out, int32_t *n_eval_out, int32_t *n_grad_out,
                                          uint8_t *flags_out) {
    const bool ok = status == ARIMA_ST_OK;
#pragma unroll
    for (int j = 0; j < K; ++j) coef_out[sid * K + j] = ok ? coef[j] : __builtin_nan("");
    ll_out[sid] = ok ? ll : __builtin_nan("");
    status_out[sid] = status;
    if (n_eval_out) n_eval_out[sid] = n_eval;
    if (n_grad_out) n_grad_out[sid] = n_grad;
    if (flags_out) flags_out[sid] = ok ? flags : 0;
}

// Persistent fit kernel: one workgroup of 64 * WAVES lanes per CU (WAVES = cg_waves<K, NS>(), up to two waves
// per SIMD). Every lane's optimizer state lives in LDS (LaneSlot), so the registers are free for the pass.
// Per wave iteration: (1) every lane with a response advances its state machine to its next request (finished
// lanes write their result and start the next series, whose id and initial point were fetched one series
// ahead); (2) the wave runs one pass over every served lane's own series. A gradient pass costs several
// objective passes, so lanes that want G sit out objective-only passes until at least g_permille/1000 of the
// active lanes want G (or nobody wants F); a G pass also yields the objective, so F lanes are served by it too.
template <int P, int Q, int I, bool SMEAR, int WAVES>
__global__ __launch_bounds__(64 * WAVES, (WAVES + 3) / 4) void k_cg_fit(
    const double *__restrict__ y, int64_t ld, int n, int64_t N, const double *__restrict__ init,
    const int32_t *__restrict__ init_status, double *__restrict__ coef_out, double *__restrict__ ll_out,
    int32_t *__restrict__ status_out, int32_t *__restrict__ n_eval_out, int32_t *__restrict__ n_grad_out,
    uint8_t *__restrict__ flags_out, unsigned long long *__restrict__ ctl, int g_permille) {
    // ctl[0] = work counter, ctl[1] = lane F passes, ctl[2] = lane G passes, ctl[3] = wave F-only passes,
    // ctl[4] = wave G passes, ctl[5] = objective evaluations, ctl[6] = gradient evaluations, ctl[7] = spec
    // hits, ctl[8] = wave multi-point passes, ctl[10..14] = STS_TIMING diagnostics
    constexpr int K = I + P + Q;
    constexpr int NS = spec_slots<K>();
    __shared__ LaneSlot<K, NS> slots[64 * WAVES];
    CGLane<K, NS> &L = slots[threadIdx.x].s;
    int64_t sid = -1;
    bool idle = false, need_new = true;
    const double *row = y;
    unsigned long long lane_f = 0, lane_g = 0, wave_f = 0, wave_g = 0, wave_m = 0, evals = 0, grads = 0, hits = 0;
    const bool lane0 = (threadIdx.x & 63) == 0;
    // response of the last served request (registers)
    double resp_f = 0.0, resp_g[K];
#pragma unroll
    for (int j = 0; j < K; ++j) resp_g[j] = 0.0;
    // next series of this lane, fetched one series ahead (id, then its status and initial point)
    int64_t nxt = (int64_t)atomicAdd(&ctl[0], 1ull);
    bool nxt_loaded = false;
    int nxt_st = ARIMA_ST_OK;
    double nxt_x0[K];
    L.req = REQ_NONE;
#ifdef STS_TIMING
    unsigned long long t_adv = 0, t_pass = 0, t_g = 0, t_m = 0;
    int kind = 0;
    const unsigned long long t_birth = __builtin_amdgcn_s_memtime();
#endif
    for (;;) {
#ifdef STS_TIMING
        const unsigned long long t_a0 = __builtin_amdgcn_s_memtime();
#endif
        if (!nxt_loaded && nxt < N) {                 // prefetch the next series' initial point
            nxt_st = init_status ? init_status[nxt] : ARIMA_ST_OK;
#pragma unroll
            for (int j = 0; j < K; ++j) nxt_x0[j] = init[nxt * K + j];
            nxt_loaded = true;
        }
        // ---- per lane: advance the state machine to its next request (refilling finished lanes) ----
        while (!idle) {
            if (need_new) {
                if (nxt >= N) { idle = true; break; }
                sid = nxt;
                const int st0 = nxt_st;
                double x0[K];
#pragma unroll
                for (int j = 0; j < K; ++j) x0[j] = nxt_x0[j];
                nxt = (int64_t)atomicAdd(&ctl[0], 1ull);
                nxt_loaded = false;
                need_new = false;
                row = y + sid * ld;
                if (st0 != ARIMA_ST_OK) {
                    double nanc[K];
#pragma unroll
                    for (int j = 0; j < K; ++j) nanc[j] = __builtin_nan("");
                    write_fit<K>(sid, st0, nanc, 0.0, 0, 0, 0, coef_out, ll_out, status_out, n_eval_out,
                                 n_grad_out, flags_out);
                    need_new = true;
                    if (nxt < N) {                    // (rare) the next one is needed right away
                        nxt_st = init_status ? init_status[nxt] : ARIMA_ST_OK;
#pragma unroll
                        for (int j = 0; j < K; ++j) nxt_x0[j] = init[nxt * K + j];
                        nxt_loaded = true;
                    }
                    continue;
                }
                L.start(x0);
            }
            if (L.req != REQ_NONE) break;        // request still pending (deferred G): nothing to advance
            L.advance(resp_f, resp_g);
            if (L.done()) {
                double pt[K];
#pragma unroll
                for (int j = 0; j < K; ++j) pt[j] = L.point[j];
                write_fit<K>(sid, L.status, pt, L.prev_obj, L.n_eval, L.n_grad,
                             L.status == ARIMA_ST_OK ? model_flags<P, Q, I>(pt) : (uint8_t)0, coef_out, ll_out,
                             status_out, n_eval_out, n_grad_out, flags_out);
                evals += L.n_eval;
                grads += L.n_grad;
                hits += L.spec_hits;
                need_new = true;
                if (!nxt_loaded && nxt < N) {
                    nxt_st = init_status ? init_status[nxt] : ARIMA_ST_OK;
#pragma unroll
                    for (int j = 0; j < K; ++j) nxt_x0[j] = init[nxt * K + j];
                    nxt_loaded = true;
                }
                continue;
            }
            break;
        }
        // ---- per wave: one pass serving the posted requests ----
        const unsigned long long act = __ballot(!idle);
#ifdef STS_TIMING
        const unsigned long long t_p0 = __builtin_amdgcn_s_memtime();
        t_adv += t_p0 - t_a0;
#endif
        if (act == 0ull) break;
        const int req = idle ? REQ_NONE : L.req;
        const unsigned long long wantG = __ballot(req == REQ_G);
        const int nG = __popcll(wantG), nA = __popcll(act);
        const bool anyG = nG > 0 && (nG == nA || nG * 1000 >= g_permille * nA);
        // lanes not served by this pass stream a shared row (L2-resident) instead of their own
        const bool served = !idle && (anyG || req == REQ_F);
        const double *prow = served ? row : y;
        double c[K], css, g[K];
        if (served) {
            L.request_point(c);
        } else {
#pragma unroll
            for (int j = 0; j < K; ++j) c[j] = 0.0;
        }
        const int nspec = (served && req == REQ_F) ? L.rq_nspec : 0;
        const bool anySpec = NS > 0 && !anyG && __ballot(nspec > 0) != 0ull;
        if (anyG) {
            css_pass<P, Q, I, true, SMEAR>(prow, n, c, css, g);
            wave_g += lane0;
#ifdef STS_TIMING
            kind = 1;
#endif
        } else if constexpr (NS > 0) {
            if (anySpec) {
                // primary point + the lane's speculative points (lanes with fewer repeat the primary)
                double cm[NS + 1][K], cssm[NS + 1];
#pragma unroll
                for (int j = 0; j < K; ++j) cm[0][j] = c[j];
#pragma unroll
                for (int h = 0; h < NS; ++h) {
                    const bool use = h < nspec;
                    const double al = use ? L.rq_spec[h] : 0.0;
#pragma unroll
                    for (int j = 0; j < K; ++j) cm[h + 1][j] = use ? L.point[j] + al * L.dir[j] : c[j];
                }
                css_pass_multi<P, Q, I, NS + 1>(prow, n, cm, cssm);
                css = cssm[0];
#pragma unroll
                for (int h = 0; h < NS; ++h) {
                    if (h < nspec) {
                        L.sp_alpha[h] = L.rq_spec[h];
                        L.sp_f[h] = css_to_loglik(cssm[h + 1], n);
                    }
                }
                if (nspec > 0) L.sp_n = (uint8_t)nspec;
                wave_m += lane0;
#ifdef STS_TIMING
                kind = 2;
#endif
            } else {
                css_pass<P, Q, I, false, SMEAR>(prow, n, c, css, g);
                wave_f += lane0;
            }
        } else {
            css_pass<P, Q, I, false, SMEAR>(prow, n, c, css, g);
            wave_f += lane0;
        }
        if (served) {
            resp_f = css_to_loglik(css, n);
            if (req == REQ_G) {
#pragma unroll
                for (int j = 0; j < K; ++j) resp_g[j] = g[j];
                lane_g++;
            } else {
                lane_f++;
            }
            L.req = REQ_NONE;
        }
#ifdef STS_TIMING
        {
            const unsigned long long dt = __builtin_amdgcn_s_memtime() - t_p0;
            t_pass += dt;
            if (kind == 1) t_g += dt;
            if (kind == 2) t_m += dt;
            kind = 0;
        }
#endif
    }
#ifdef STS_TIMING
    if (lane0) {
        atomicAdd(&ctl[10], t_adv);
        atomicAdd(&ctl[11], t_pass);
        atomicAdd(&ctl[12], __builtin_amdgcn_s_memtime() - t_birth);
        atomicAdd(&ctl[13], t_g);
        atomicAdd(&ctl[14], t_m);
    }
#endif
    atomicAdd(&ctl[1], lane_f);
    atomicAdd(&ctl[2], lane_g);
    if (lane0) {
        atomicAdd(&ctl[3], wave_f);
        atomicAdd(&ctl[4], wave_g);
    }
    atomicAdd(&ctl[5], evals);
    atomicAdd(&ctl[6], grads);
    atomicAdd(&ctl[7], hits);
    if (lane0) atomicAdd(&ctl[8], wave_m);
}

// =======================================================================================================
// Building blocks at given coefficients
// =======================================================================================================
template <int P, int Q, int I>
__global__ __launch_bounds__(256) void k_css_loglik(const double *__restrict__ y, int64_t ld, int n, int64_t N,
                                                    const double *__restrict__ coef, double *__restrict__ ll_out) {
    constexpr int K = I + P + Q;
    constexpr int KA = K > 0 ? K : 1;
    const int64_t sid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sid >= N) return;
    double c[KA], g[KA], css;
#pragma unroll
    for (int j = 0; j < KA; ++j) c[j] = (j < K) ? coef[sid * K + j] : 0.0;
    css_pass<P, Q, I, false, false>(y + sid * ld, n, c, css, g);
    ll_out[sid] = css_to_loglik(css, n);
}

template <int P, int Q, int I, bool SMEAR>
__global__ __launch_bounds__(256) void k_css_grad(const double *__restrict__ y, int64_t ld, int n, int64_t N,
                                                  const double *__restrict__ coef, double *__restrict__ g_out) {
    constexpr int K = I + P + Q;
    constexpr int KA = K > 0 ? K : 1;
    const int64_t sid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sid >= N) return;
    double c[KA], g[KA], css;
#pragma unroll
    for (int j = 0; j < KA; ++j) c[j] = (j < K) ? coef[sid * K + j] : 0.0;
    css_pass<P, Q, I, true, SMEAR>(y + sid * ld, n, c, css, g);
#pragma unroll
    for (int j = 0; j < K; ++j) g_out[sid * K + j] = g[j];
}

template <int P, int Q, int I>
__global__ __launch_bounds__(256) void k_model_flags(const double *__restrict__ coef, int64_t N,
                                                     uint8_t *__restrict__ flags_out) {
    constexpr int K = I + P + Q;
    constexpr int KA = K > 0 ? K : 1;
    const int64_t sid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sid >= N) return;
    double c[KA];
#pragma unroll
    for (int j = 0; j < KA; ++j) c[j] = (j < K) ? coef[sid * K + j] : 0.0;
    flags_out[sid] = model_flags<P, Q, I>(c);
}


// =======================================================================================================
// per-P launchers (explicitly instantiated one P per translation unit: arima_inst_p{0..5}.hip)
// =======================================================================================================
template <int V>
using IC = std::integral_constant<int, V>;

#ifdef STS_DEV
// dev build (make dev): only q = STS_DEV_Q, smear off -- fast compiles for kernel experiments
template <class Fn>
int with_order(int v, Fn &&fn) {
    return v == STS_DEV_Q ? fn(IC<STS_DEV_Q>{}) : ARIMA_E_UNSUPPORTED;
}
template <class Fn>
int with_smear(int v, Fn &&fn) {
    return v ? ARIMA_E_UNSUPPORTED : fn(IC<0>{});
}
#else
template <class Fn>
int with_order(int v, Fn &&fn) {
    switch (v) {
    case 0: return fn(IC<0>{});
    case 1: return fn(IC<1>{});
    case 2: return fn(IC<2>{});
    case 3: return fn(IC<3>{});
    case 4: return fn(IC<4>{});
    case 5: return fn(IC<5>{});
    default: return ARIMA_E_UNSUPPORTED;
    }
}
#endif
template <class Fn>
int with_bool(int v, Fn &&fn) {
    return v ? fn(IC<1>{}) : fn(IC<0>{});
}
#ifndef STS_DEV
template <class Fn>
int with_smear(int v, Fn &&fn) {
    return with_bool(v, fn);
}
#endif

inline unsigned grid_for(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }

#define STS_CHECK_LAUNCH()                                                                                 \
    do {                                                                                                   \
        hipError_t e_ = hipGetLastError();                                                                 \
        if (e_ != hipSuccess) return ARIMA_E_DEVICE;                                                       \
    } while (0)

template <int P>
int launch_hr_init_P(const double *y, int64_t ld, int n, int64_t N, int q, int I, double *init_out,
                     int32_t *status_out, hipStream_t s) {
    return with_order(q, [&](auto Qc) {
        return with_bool(I, [&](auto Ic) {
            constexpr int Q = decltype(Qc)::value, II = decltype(Ic)::value;
            hipLaunchKernelGGL((k_hr_init<P, Q, II>), dim3(grid_for(N, 256)), dim3(256), 0, s, y, ld, n, N, init_out,
                               status_out);
            STS_CHECK_LAUNCH();
            return ARIMA_OK;
        });
    });
}

template <int P>
int launch_ar_fit_P(const double *y, int64_t ld, int n, int64_t N, int I, double *coef_out, double *ll_out,
                    int32_t *status_out, int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out,
                    hipStream_t s) {
    if constexpr (P == 0) {
        return ARIMA_E_INVALID_ARG;
    } else {
        return with_bool(I, [&](auto Ic) {
            constexpr int II = decltype(Ic)::value;
            hipLaunchKernelGGL((k_ar_fit<P, II>), dim3(grid_for(N, 256)), dim3(256), 0, s, y, ld, n, N, coef_out,
                               ll_out, status_out, n_eval_out, n_grad_out, flags_out);
            STS_CHECK_LAUNCH();
            return ARIMA_OK;
        });
    }
}

template <int P>
int launch_cg_fit_P(const double *y, int64_t ld, int n, int64_t N, int q, int I, int smear, const double *init,
                    const int32_t *init_status, double *coef_out, double *ll_out, int32_t *status_out,
                    int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out, unsigned long long *ctl,
                    int grid_blocks, int g_permille, hipStream_t s) {
    return with_order(q, [&](auto Qc) {
        return with_bool(I, [&](auto Ic) {
            return with_smear(smear, [&](auto Sc) {
                constexpr int Q = decltype(Qc)::value, II = decltype(Ic)::value;
                constexpr bool S = decltype(Sc)::value != 0;
                if constexpr (P + Q + II == 0) {
                    return ARIMA_E_INVALID_ARG;
                } else {
                    constexpr int W = cg_waves<P + Q + II, spec_slots<P + Q + II>()>();
                    hipLaunchKernelGGL((k_cg_fit<P, Q, II, S, W>), dim3(grid_blocks), dim3(64 * W), 0, s, y, ld, n, N,
                                       init, init_status, coef_out, ll_out, status_out, n_eval_out, n_grad_out,
                                       flags_out, ctl, g_permille);
                    STS_CHECK_LAUNCH();
                    return ARIMA_OK;
                }
            });
        });
    });
}

template <int P>
int cg_fit_occupancy_blocks_P(int q, int I, int smear) {
    int blocks = 0;
    with_order(q, [&](auto Qc) {
        return with_bool(I, [&](auto Ic) {
            return with_smear(smear, [&](auto Sc) {
                constexpr int Q = decltype(Qc)::value, II = decltype(Ic)::value;
                constexpr bool S = decltype(Sc)::value != 0;
                if constexpr (P + Q + II > 0) {
                    constexpr int W = cg_waves<P + Q + II, spec_slots<P + Q + II>()>();
                    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_cg_fit<P, Q, II, S, W>, 64 * W, 0);
                }
                return 0;
            });
        });
    });
    return blocks;
}

template <int P>
int launch_css_loglik_P(const double *y, int64_t ld, int n, int64_t N, int q, int I, const double *coef,
                        double *ll_out, hipStream_t s) {
    return with_order(q, [&](auto Qc) {
        return with_bool(I, [&](auto Ic) {
            constexpr int Q = decltype(Qc)::value, II = decltype(Ic)::value;
            hipLaunchKernelGGL((k_css_loglik<P, Q, II>), dim3(grid_for(N, 256)), dim3(256), 0, s, y, ld, n, N, coef,
                               ll_out);
            STS_CHECK_LAUNCH();
            return ARIMA_OK;
        });
    });
}

template <int P>
int launch_css_grad_P(const double *y, int64_t ld, int n, int64_t N, int q, int I, int smear, const double *coef,
                      double *g_out, hipStream_t s) {
    return with_order(q, [&](auto Qc) {
        return with_bool(I, [&](auto Ic) {
            return with_smear(smear, [&](auto Sc) {
                constexpr int Q = decltype(Qc)::value, II = decltype(Ic)::value;
                constexpr bool S = decltype(Sc)::value != 0;
                hipLaunchKernelGGL((k_css_grad<P, Q, II, S>), dim3(grid_for(N, 256)), dim3(256), 0, s, y, ld, n, N,
                                   coef, g_out);
                STS_CHECK_LAUNCH();
                return ARIMA_OK;
            });
        });
    });
}

template <int P>
int launch_model_flags_P(const double *coef, int64_t N, int q, int I, uint8_t *flags_out, hipStream_t s) {
    return with_order(q, [&](auto Qc) {
        return with_bool(I, [&](auto Ic) {
            constexpr int Q = decltype(Qc)::value, II = decltype(Ic)::value;
            hipLaunchKernelGGL((k_model_flags<P, Q, II>), dim3(grid_for(N, 256)), dim3(256), 0, s, coef, N, flags_out);
            STS_CHECK_LAUNCH();
            return ARIMA_OK;
        });
    });
}

#define STS_DECLARE_P(PP, EXT)                                                                                  \
    EXT template int launch_hr_init_P<PP>(const double *, int64_t, int, int64_t, int, int, double *, int32_t *,  \
                                          hipStream_t);                                                         \
    EXT template int launch_ar_fit_P<PP>(const double *, int64_t, int, int64_t, int, double *, double *,         \
                                         int32_t *, int32_t *, int32_t *, uint8_t *, hipStream_t);              \
    EXT template int launch_cg_fit_P<PP>(const double *, int64_t, int, int64_t, int, int, int, const double *,   \
                                         const int32_t *, double *, double *, int32_t *, int32_t *, int32_t *,  \
                                         uint8_t *, unsigned long long *, int, int, hipStream_t);                \
    EXT template int cg_fit_occupancy_blocks_P<PP>(int, int, int);                                              \
    EXT template int launch_css_loglik_P<PP>(const double *, int64_t, int, int64_t, int, int, const double *,    \
                                             double *, hipStream_t);                                            \
    EXT template int launch_css_grad_P<PP>(const double *, int64_t, int, int64_t, int, int, int, const double *, \
                                           double *, hipStream_t);                                              \
    EXT template int launch_model_flags_P<PP>(const double *, int64_t, int, int, uint8_t *, hipStream_t);

}  // namespace sts
