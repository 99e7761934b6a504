// arima_bobyqa.hip — css-bobyqa on the device: ARIMA.fitWithCSSBOBYQA (ARIMA.scala:130-160) over a batch, and autoFit's
// css-bobyqa retries. The algorithm and its kernels are templates in arima_bobyqa_impl.hpp; each dimension K = 2..11 is
// instantiated in its own translation unit (arima_bobyqa_k<K>.hip) so the build compiles them in parallel; this file
// holds the dimension dispatch, the K < 2 instantiations (BOBYQAOptimizer.setup rejects them) and the retry list.
#include <algorithm>

#include "arima_bobyqa_impl.hpp"

namespace sts {

STS_BQ_DECLARE(2, extern) STS_BQ_DECLARE(3, extern) STS_BQ_DECLARE(4, extern) STS_BQ_DECLARE(5, extern)
STS_BQ_DECLARE(6, extern) STS_BQ_DECLARE(7, extern) STS_BQ_DECLARE(8, extern) STS_BQ_DECLARE(9, extern)
STS_BQ_DECLARE(10, extern) STS_BQ_DECLARE(11, extern)

// The round's retry list, bucketed by dimension K = p + q + intercept: bucket K holds its rows at list[K * stride ..],
// counts[K] of them (the runtime launches each dimension's kernel for its bucket)
__global__ __launch_bounds__(64) void k_af_refit_list(const int32_t *__restrict__ status, int64_t total,
                                                      const int64_t *__restrict__ off, int ncombos,
                                                      int32_t *__restrict__ list, int64_t stride,
                                                      unsigned *__restrict__ counts) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= total || !bq_refit_wanted(status[r])) return;
    const int cb = af_row_combo(off, ncombos, r);
    const int p = (cb / 2) / 3, q = (cb / 2) % 3, I = cb % 2, k = p + q + I;
    if (p > 0 && q == 0) return;                   // the AR-only shortcut never reaches a method (ARIMA.scala:90-96)
    const unsigned slot = atomicAdd(&counts[k], 1u);
    list[(int64_t)k * stride + slot] = (int32_t)r;
}

int launch_bobyqa_refit_list(const int64_t *off, int ncombos, int64_t total, const int32_t *status, int32_t *list,
                             int64_t stride, unsigned *counts, hipStream_t s) {
    if (hipMemsetAsync(counts, 0, kBqRefitBuckets * sizeof(unsigned), s) != hipSuccess) return ARIMA_E_DEVICE;
    if (total == 0) return ARIMA_OK;
    hipLaunchKernelGGL(k_af_refit_list, dim3((unsigned)((total + 63) / 64)), dim3(64), 0, s, status, total, off, ncombos,
                       list, stride, counts);
    return hipGetLastError() == hipSuccess ? ARIMA_OK : ARIMA_E_DEVICE;
}

int launch_bobyqa_refit_dim(int k, const double *rows_, int64_t ld, int n, const int32_t *lists, int64_t N,
                            const int64_t *off, int ncombos, int kc, const int32_t *list, const unsigned *counts,
                            int64_t rows, const double *init, const int32_t *init_status, double *coef, double *ll,
                            int32_t *status, uint8_t *flags, bool wave, hipStream_t s) {
#define BQ_REFIT(K)                                                                                                   \
    case K:                                                                                                           \
        return launch_bobyqa_refit_k<K>(rows_, ld, n, lists, N, off, ncombos, kc, list, counts, rows, init,           \
                                        init_status, coef, ll, status, flags, wave, s);
    switch (k) {
        BQ_REFIT(2) BQ_REFIT(3) BQ_REFIT(4) BQ_REFIT(5) BQ_REFIT(6) BQ_REFIT(7) BQ_REFIT(8) BQ_REFIT(9) BQ_REFIT(10)
        BQ_REFIT(11)
    default:
        return ARIMA_E_UNSUPPORTED;
    }
#undef BQ_REFIT
}

int launch_bobyqa_fit(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, const double *init,
                      const int32_t *init_status, const int32_t *refit_status, double *coef_out, double *ll_out,
                      int32_t *status_out, int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out, bool wave,
                      hipStream_t s) {
    if (N == 0) return ARIMA_OK;
    if (!gen_orders_ok(p, q) || I + p + q > BQ_KMAX) return ARIMA_E_UNSUPPORTED;
    // one instantiation per dimension k = I + p + q: Powell's loops get compile-time bounds
#define BQ_LAUNCH(K)                                                                                                  \
    case K:                                                                                                           \
        return launch_bobyqa_fit_k<K>(y, ld, n, N, p, q, I, init, init_status, refit_status, coef_out, ll_out,        \
                                      status_out, n_eval_out, n_grad_out, flags_out, wave, s);
    switch (I + p + q) {
        BQ_LAUNCH(0) BQ_LAUNCH(1) BQ_LAUNCH(2) BQ_LAUNCH(3) BQ_LAUNCH(4) BQ_LAUNCH(5) BQ_LAUNCH(6) BQ_LAUNCH(7)
        BQ_LAUNCH(8) BQ_LAUNCH(9) BQ_LAUNCH(10) BQ_LAUNCH(11)
    default:
        return ARIMA_E_UNSUPPORTED;
    }
#undef BQ_LAUNCH
}

}  // namespace sts
