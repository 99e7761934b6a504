// arima_runtime.cpp — the C ABI (include/sparkts_arima.h) over the HIP kernels: one handle per device, a
// private stream, grow-only device workspaces, per-call HIP-event timing and aggregate pass counters.
//
// Call flow of arima_fit_batch_device (the drop-in for ARIMA.fitModel over one Spark partition,
// ARIMA.scala:79-116):
//   k_difference (differencesOfOrderD(ts, d).drop(d), :88)  ->  p>0 && q==0 ? k_ar_fit (:90-96)
//   : [k_hr_init (:99-103, unless user init)] -> k_cg_fit (fitWithCSSCGD, :105-109, :174-200)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/sparkts_arima.h"
#include "arima_launch.hpp"

namespace {

struct DevBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    int ensure(size_t need) {
        if (need <= bytes) return ARIMA_OK;
        if (ptr) hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
        if (need == 0) return ARIMA_OK;
        if (hipMalloc(&ptr, need) != hipSuccess) return ARIMA_E_OOM;
        bytes = need;
        return ARIMA_OK;
    }
    void release() {
        if (ptr) hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    template <class T>
    T *as() const { return static_cast<T *>(ptr); }
};

constexpr int kNumEvents = 5;
constexpr int kCtlWords = 32;     // device counters of the fit kernel (k_cg_fit's ctl[])

// What arima_get_last_stats needs to turn the device counters of the last fit into arima_fit_stats. The fit
// entry points do not wait for the device (the `*_device` contract): the counters are copied to pinned host
// memory in stream order and the stats are computed when they are asked for.
struct PendingStats {
    bool valid = false;
    int64_t N = 0;
    int n = 0, p = 0, q = 0, I = 0;
    bool ar_only = false, user_init = false, cg = false;
    int64_t grid = 0, express = 0;
};

// Device workspace of one fit in flight: Hannan-Rissanen init, the fit kernel's counters and its express ring.
struct FitWs {
    DevBuf init, hr_status, ctl, xring, xready;
};

// One lane of the order search's concurrent fits (arima_order_search_batch*): its own stream, workspace and
// candidate outputs. Fits of consecutive grid points run on different lanes, so the tail of one fit kernel (its
// slowest series) overlaps the next fits; the select steps stay in grid order on the call's stream.
struct SearchLane {
    hipStream_t stream = nullptr;
    hipEvent_t ev_fit = nullptr, ev_sel = nullptr;
    bool sel_recorded = false;
    FitWs ws;
    DevBuf coef, ll, status, neval, ngrad, flags;
};

constexpr int kMaxSearchLanes = 8;
constexpr int kMaxD = 16;

}  // namespace

struct arima_handle {
    int device = 0;
    int num_cus = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[kNumEvents] = {};
    hipEvent_t ev_done = nullptr;     // end of the last call's device work (serialises workspace reuse across streams)
    bool has_done = false;
    mutable std::mutex mu;
    std::string err;
    arima_fit_stats stats{};
    PendingStats pending;
    bool fit_ctl = false;          // ctl_host holds (or will hold, in stream order) the last fit's kernel counters
    int smear = 1;            // Breeze 0.12 overlap semantics at ARIMA.scala:526: element-wise copy
    int grid_blocks_override = 0;
    int express_blocks = -1;       // k_cg_fit express workgroups (-1: num_cus / 16)
    int64_t last_express = 0;
    int64_t last_grid = 0;
    int search_lanes = 4;          // concurrent fits of the order search
    // device workspaces
    DevBuf diff;
    FitWs ws;
    // host-API staging
    DevBuf h_series, h_coef, h_ll, h_status, h_neval, h_ngrad, h_flags, h_uinit, h_aux;
    // order search: the differenced series per d, the concurrent fit lanes, host-API staging of the orders
    DevBuf os_diff[kMaxD + 1];
    hipEvent_t ev_diff[kMaxD + 1] = {};
    SearchLane lanes[kMaxSearchLanes];
    DevBuf os_order;
    unsigned long long *ctl_host = nullptr;   // pinned
};

namespace {

int set_err(arima_handle *h, int code, const char *msg) {
    if (h) h->err = msg ? msg : "";
    return code;
}

#define HIPCHK(h, expr)                                                                                    \
    do {                                                                                                   \
        hipError_t e_ = (expr);                                                                            \
        if (e_ != hipSuccess) return set_err((h), ARIMA_E_DEVICE, hipGetErrorString(e_));                  \
    } while (0)

#define RCCHK(h, expr, what)                                                                               \
    do {                                                                                                   \
        int rc_ = (expr);                                                                                  \
        if (rc_ != ARIMA_OK) return set_err((h), rc_, what);                                               \
    } while (0)

inline int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// uniform-per-call status fill (unsupported method, zero parameters, shape errors)
__global__ void k_fill_status(int64_t N, int k, const int32_t *__restrict__ prior, int32_t code,
                              double *__restrict__ coef_out, double *__restrict__ ll_out,
                              int32_t *__restrict__ status_out, int32_t *__restrict__ n_eval_out,
                              int32_t *__restrict__ n_grad_out, uint8_t *__restrict__ flags_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    int st = code;
    if (prior && prior[i] != ARIMA_ST_OK) st = prior[i];
    for (int j = 0; j < k; ++j) coef_out[i * k + j] = __builtin_nan("");
    ll_out[i] = __builtin_nan("");
    status_out[i] = st;
    if (n_eval_out) n_eval_out[i] = 0;
    if (n_grad_out) n_grad_out[i] = 0;
    if (flags_out) flags_out[i] = 0;
}

int check_orders(arima_handle *h, int p, int d, int q, int I) {
    if (p < 0 || q < 0 || d < 0 || (I != 0 && I != 1)) return set_err(h, ARIMA_E_INVALID_ARG, "bad order");
    if (p > 5 || q > 5) return set_err(h, ARIMA_E_UNSUPPORTED, "p, q <= 5 are compiled in this build");
    if (d > 16) return set_err(h, ARIMA_E_UNSUPPORTED, "d <= 16");
    return ARIMA_OK;
}

}  // namespace

namespace sts {
int hr_shape_status_host(int n, int p, int q, int I);
}

extern "C" {

int arima_num_params(int p, int q, int include_intercept) { return p + q + (include_intercept ? 1 : 0); }

const char *arima_status_name(int s) {
    switch (s) {
    case ARIMA_ST_OK: return "OK";
    case ARIMA_ST_MAX_EVAL: return "MAX_EVAL";
    case ARIMA_ST_BRACKET_MAX_EVAL: return "BRACKET_MAX_EVAL";
    case ARIMA_ST_MAX_ITER: return "MAX_ITER";
    case ARIMA_ST_SINGULAR: return "SINGULAR";
    case ARIMA_ST_NOT_ENOUGH_DATA: return "NOT_ENOUGH_DATA";
    case ARIMA_ST_NO_DATA: return "NO_DATA";
    case ARIMA_ST_BAD_INTERVAL: return "BAD_INTERVAL";
    case ARIMA_ST_ZERO_PARAMS: return "ZERO_PARAMS";
    case ARIMA_ST_UNSUPPORTED_METHOD: return "UNSUPPORTED_METHOD";
    case ARIMA_ST_SERIES_TOO_SHORT: return "SERIES_TOO_SHORT";
    default: return "UNKNOWN";
    }
}

int arima_create(int device, arima_handle **out) {
    if (!out) return ARIMA_E_INVALID_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return ARIMA_E_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return ARIMA_E_DEVICE;
    arima_handle *h = new arima_handle();
    h->device = device;
    hipDeviceGetAttribute(&h->num_cus, hipDeviceAttributeMultiprocessorCount, device);
    int rc = ARIMA_OK;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) rc = ARIMA_E_DEVICE;
    for (auto &e : h->ev)
        if (rc == ARIMA_OK && hipEventCreate(&e) != hipSuccess) rc = ARIMA_E_DEVICE;
    if (rc == ARIMA_OK && hipEventCreateWithFlags(&h->ev_done, hipEventDisableTiming) != hipSuccess) rc = ARIMA_E_DEVICE;
    if (rc == ARIMA_OK && hipHostMalloc((void **)&h->ctl_host, kCtlWords * sizeof(unsigned long long), 0) != hipSuccess)
        rc = ARIMA_E_OOM;
    if (rc != ARIMA_OK) {
        arima_destroy(h);
        return rc;
    }
    *out = h;
    return ARIMA_OK;
}

int arima_destroy(arima_handle *h) {
    if (!h) return ARIMA_E_INVALID_ARG;
    hipSetDevice(h->device);
    if (h->stream) hipStreamSynchronize(h->stream);
    if (h->has_done) hipEventSynchronize(h->ev_done);
    for (auto &l : h->lanes) {
        if (l.stream) {
            hipStreamSynchronize(l.stream);
            hipStreamDestroy(l.stream);
        }
        if (l.ev_fit) hipEventDestroy(l.ev_fit);
        if (l.ev_sel) hipEventDestroy(l.ev_sel);
    }
    for (auto &e : h->ev_diff)
        if (e) hipEventDestroy(e);
    for (auto &e : h->ev)
        if (e) hipEventDestroy(e);
    if (h->ev_done) hipEventDestroy(h->ev_done);
    if (h->ctl_host) hipHostFree(h->ctl_host);
    if (h->stream) hipStreamDestroy(h->stream);
    delete h;                                  // every DevBuf workspace frees itself
    return ARIMA_OK;
}

const char *arima_last_error(const arima_handle *h) { return h ? h->err.c_str() : "null handle"; }

static void finish_stats(arima_handle *h);

int arima_get_last_stats(const arima_handle *hc, arima_fit_stats *out) {
    if (!hc || !out) return ARIMA_E_INVALID_ARG;
    arima_handle *h = const_cast<arima_handle *>(hc);   // the lazy completion below only fills h->stats
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->pending.valid) {
        hipSetDevice(h->device);
        if (hipEventSynchronize(h->ev_done) != hipSuccess) return set_err(h, ARIMA_E_DEVICE, "stats: device error");
        finish_stats(h);
    }
    *out = h->stats;
    return ARIMA_OK;
}

// The last fit's kernel recorded a watchdog fault (k_cg_fit's hand-off): its results are incomplete.
static int check_fault(arima_handle *h) {
    if (h->fit_ctl && h->ctl_host[26] != 0) {
        h->fit_ctl = false;                      // reported once
        char msg[160];
        snprintf(msg, sizeof msg, "fit kernel watchdog fault %llu (info %llu %llu %llu %llu %llu)", h->ctl_host[26],
                 h->ctl_host[27], h->ctl_host[28], h->ctl_host[29], h->ctl_host[30], h->ctl_host[31]);
        return set_err(h, ARIMA_E_DEVICE, msg);
    }
    return ARIMA_OK;
}

int arima_synchronize(arima_handle *h) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    HIPCHK(h, hipSetDevice(h->device));
    if (h->has_done) HIPCHK(h, hipEventSynchronize(h->ev_done));
    return check_fault(h);
}

int arima_set_option(arima_handle *h, const char *name, int64_t value) {
    if (!h || !name) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (!strcmp(name, "smear")) { h->smear = value ? 1 : 0; return ARIMA_OK; }
    if (!strcmp(name, "express_blocks")) { h->express_blocks = (int)std::max<int64_t>(-1, value); return ARIMA_OK; }
    if (!strcmp(name, "grid_blocks")) { h->grid_blocks_override = (int)std::max<int64_t>(0, value); return ARIMA_OK; }
    if (!strcmp(name, "search_lanes")) {
        h->search_lanes = (int)std::min<int64_t>(kMaxSearchLanes, std::max<int64_t>(1, value));
        return ARIMA_OK;
    }
    return set_err(h, ARIMA_E_INVALID_ARG, "unknown option");
}

// ---------------------------------------------------------------------------------------------------------
// Every device call waits (on the device, not the host) for the previous call's work: the handle's workspaces are
// shared by all calls, whichever stream they are issued on.
static void begin_call(arima_handle *h, hipStream_t s) {
    if (h->has_done) hipStreamWaitEvent(s, h->ev_done, 0);
}

static hipError_t end_call(arima_handle *h, hipStream_t s) {
    hipError_t e = hipEventRecord(h->ev_done, s);
    if (e == hipSuccess) h->has_done = true;
    return e;
}

// Hannan-Rissanen init (unless user init) and the fit kernel -- or the AR-only shortcut, or a uniform per-series
// status -- over already-differenced rows y (N x n, leading dimension ldn), on stream s with workspace ws.
// ev_mid (optional) is recorded between the init and the fit kernel. shared_gpu: other fits run concurrently (the
// order search's lanes), so the fit kernel's drained workgroups exit instead of joining its express pool.
static int fit_kernels(arima_handle *h, FitWs &ws, const double *y, int64_t ldn, int n, int64_t N, int32_t p,
                       int32_t q, int32_t I, int32_t method, const double *d_user_init, double *d_coef, double *d_ll,
                       int32_t *d_status, int32_t *d_neval, int32_t *d_ngrad, uint8_t *d_flags, hipStream_t s,
                       hipEvent_t ev_mid, int64_t *grid_out, int64_t *express_out, bool shared_gpu = false) {
    const int k = I + p + q;
    *grid_out = 0;
    *express_out = 0;
    RCCHK(h, ws.ctl.ensure(kCtlWords * sizeof(unsigned long long)), "workspace");
    HIPCHK(h, hipMemsetAsync(ws.ctl.ptr, 0, kCtlWords * sizeof(unsigned long long), s));
    HIPCHK(h, hipMemsetAsync(ws.ctl.as<unsigned long long>() + 15, 0xff, sizeof(unsigned long long), s));
    if (p > 0 && q == 0) {                                     // AR-only shortcut, method never checked
        if (ev_mid) HIPCHK(h, hipEventRecord(ev_mid, s));
        RCCHK(h, sts::launch_ar_fit(y, ldn, n, N, p, I, d_coef, d_ll, d_status, d_neval, d_ngrad, d_flags, s),
              "ar_fit");
        return ARIMA_OK;
    }
    const double *init = d_user_init;
    const int32_t *init_status = nullptr;
    if (!d_user_init) {
        RCCHK(h, ws.init.ensure((size_t)N * std::max(k, 1) * sizeof(double)), "workspace");
        RCCHK(h, ws.hr_status.ensure((size_t)N * sizeof(int32_t)), "workspace");
        RCCHK(h, sts::launch_hr_init(y, ldn, n, N, p, q, I, ws.init.as<double>(), ws.hr_status.as<int32_t>(), s),
              "hr_init");
        init = ws.init.as<double>();
        init_status = ws.hr_status.as<int32_t>();
    }
    if (ev_mid) HIPCHK(h, hipEventRecord(ev_mid, s));
    if (method != ARIMA_METHOD_CSS_CGD || k == 0) {
        const unsigned grid = (unsigned)((N + 255) / 256);
        const int32_t code = (method != ARIMA_METHOD_CSS_CGD) ? ARIMA_ST_UNSUPPORTED_METHOD : ARIMA_ST_ZERO_PARAMS;
        hipLaunchKernelGGL(k_fill_status, dim3(grid), dim3(256), 0, s, N, k, init_status, code, d_coef, d_ll,
                           d_status, d_neval, d_ngrad, d_flags);
        HIPCHK(h, hipGetLastError());
        return ARIMA_OK;
    }
    // one persistent workgroup per CU (4 waves x the kernel's optimizer slots), the last num_cus/16 of them express
    // workgroups (k_cg_fit's long-series path); fewer bulk blocks when the batch cannot fill them
    const int cus = std::max(1, h->num_cus);
    int xblocks = h->express_blocks >= 0 ? h->express_blocks : std::max(1, cus / 16);
    if (xblocks >= cus) xblocks = cus - 1;
    int blocks = h->grid_blocks_override;
    if (blocks <= 0) blocks = std::max(1, cus - xblocks);
    const int per_block = std::max(1, sts::cg_fit_series_per_block(p, q, I));
    const int64_t need = (N + per_block - 1) / per_block;
    if (blocks > need) blocks = (int)need;
    if (xblocks > 0) {
        RCCHK(h, ws.xring.ensure(sts::kExpressRingBytes), "workspace");
        RCCHK(h, ws.xready.ensure(sts::kExpressReadyBytes), "workspace");
        HIPCHK(h, hipMemsetAsync(ws.xready.ptr, 0, sts::kExpressReadyBytes, s));
    }
    *grid_out = blocks;
    *express_out = xblocks;
    RCCHK(h, sts::launch_cg_fit(y, ldn, n, N, p, q, I, h->smear, init, init_status, d_coef, d_ll, d_status, d_neval,
                                d_ngrad, d_flags, ws.ctl.as<unsigned long long>(), blocks, xblocks,
                                ws.xring.as<unsigned char>(), ws.xready.as<unsigned>(), shared_gpu ? 0 : 1, s),
          "cg_fit");
    return ARIMA_OK;
}

static int fit_device_locked(arima_handle *h, const double *d_series, int64_t N, int32_t T, int64_t ld, int32_t p,
                             int32_t d, int32_t q, int32_t I, int32_t method, const double *d_user_init,
                             double *d_coef, double *d_ll, int32_t *d_status, int32_t *d_neval, int32_t *d_ngrad,
                             uint8_t *d_flags, hipStream_t s) {
    RCCHK(h, check_orders(h, p, d, q, I), "orders");
    if (N < 0 || T < 0 || ld < T) return set_err(h, ARIMA_E_INVALID_ARG, "bad shape");
    if (!d_coef || !d_ll || !d_status) return set_err(h, ARIMA_E_INVALID_ARG, "null output");
    HIPCHK(h, hipSetDevice(h->device));
    const int k = I + p + q;
    const int n = std::max(T - d, 0);
    const int64_t ldn = round_up(std::max(n, 1), 16);
    h->pending = PendingStats{};
    h->stats = arima_fit_stats{};
    if (N == 0) return ARIMA_OK;
    begin_call(h, s);

    RCCHK(h, h->diff.ensure((size_t)N * ldn * sizeof(double)), "workspace");
    HIPCHK(h, hipEventRecord(h->ev[0], s));
    RCCHK(h, sts::launch_difference(d_series, ld, h->diff.as<double>(), ldn, N, T, d, 1, s), "difference");
    HIPCHK(h, hipEventRecord(h->ev[1], s));
    int64_t grid = 0, xblocks = 0;
    RCCHK(h, fit_kernels(h, h->ws, h->diff.as<double>(), ldn, n, N, p, q, I, method, d_user_init, d_coef, d_ll,
                         d_status, d_neval, d_ngrad, d_flags, s, h->ev[2], &grid, &xblocks), "fit");
    HIPCHK(h, hipEventRecord(h->ev[3], s));
    h->last_grid = grid;
    h->last_express = xblocks;
    HIPCHK(h, hipMemcpyAsync(h->ctl_host, h->ws.ctl.ptr, kCtlWords * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    h->fit_ctl = true;
    HIPCHK(h, end_call(h, s));
    PendingStats &ps = h->pending;
    ps.N = N;
    ps.n = n;
    ps.p = p;
    ps.q = q;
    ps.I = I;
    ps.ar_only = p > 0 && q == 0;
    ps.user_init = d_user_init != nullptr;
    ps.cg = !ps.ar_only && method == ARIMA_METHOD_CSS_CGD && k > 0;
    ps.grid = h->last_grid;
    ps.express = h->last_express;
    ps.valid = true;
    return ARIMA_OK;
}

// Completes the stats of the last fit once its device work has finished (arima_get_last_stats).
static void finish_stats(arima_handle *h) {
    const PendingStats &ps = h->pending;
    arima_fit_stats st{};
    const int64_t N = ps.N;
    const int n = ps.n, p = ps.p, q = ps.q, I = ps.I, k = I + p + q;
    float ms = 0;
    hipEventElapsedTime(&ms, h->ev[0], h->ev[1]);
    st.ms_difference = ms;
    hipEventElapsedTime(&ms, h->ev[1], h->ev[2]);
    st.ms_hr_init = ms;
    hipEventElapsedTime(&ms, h->ev[2], h->ev[3]);
    st.ms_cg_fit = ms;
    hipEventElapsedTime(&ms, h->ev[0], h->ev[3]);
    st.ms_total = ms;
    const unsigned long long *c = h->ctl_host;
    st.f_passes = (int64_t)c[1];
    st.g_passes = (int64_t)c[2];
    st.n_eval = (int64_t)c[5];
    st.n_grad = (int64_t)c[6];
    st.wave_f_passes = (int64_t)c[3];
    st.wave_g_passes = (int64_t)c[4];
    st.spec_hits = (int64_t)c[7];
    st.wave_multi_passes = (int64_t)c[8];
    st.spec_chains = (int64_t)c[9];
    st.express_series = (int64_t)c[23];
    st.express_f_passes = (int64_t)c[24];
    st.express_g_passes = (int64_t)c[25];
    st.express_blocks = ps.express;
    st.fault = (int64_t)c[26];
    for (int i = 0; i < 5; ++i) st.fault_info[i] = (int64_t)c[27 + i];
    // STS_TIMING builds: F-pass, G-pass, advance, select cycles (summed over waves), kernel span, drained time
    st.diag[0] = (int64_t)c[10];
    st.diag[1] = (int64_t)c[11];
    st.diag[2] = (int64_t)c[12];
    st.diag[3] = (int64_t)c[13];
    st.diag[4] = c[14] ? (int64_t)(c[14] - c[15]) : 0;
    st.diag[5] = (int64_t)c[16];
    st.grid_blocks = ps.grid;
    // HR passes: 2 per column of each of the two least squares, minus the norm pass of an intercept column (the
    // sum of ones needs no stream; arima_device.hpp ols_stage)
    const int M = std::max(p, q), m = M + 1;
    if (ps.ar_only) st.hr_passes = N * (int64_t)(2 * (I + p) - I);
    else if (!ps.user_init) st.hr_passes = N * (int64_t)(2 * (1 + m) - 1 + 2 * k - I);
    // algorithmic flops: U*S*(2(p+q)+4) + G*S*(2(p+q)+4 + 2kq + 1+p+q + 2k) + W_HR
    const double S = std::max(n - M, 0);
    const double ff = 2.0 * (p + q) + 4, fg = ff + 2.0 * k * q + 1 + p + q + 2.0 * k;
    const double whr = (double)N * (3.0 * std::max(n - m, 0) * (m + 1) * (m + 1) +
                                    3.0 * std::max(n - 2 * M - 1, 0) * k * k + 2.0 * std::max(n - m, 0) * m);
    st.flops = (double)st.f_passes * S * ff + (double)st.g_passes * S * fg + (ps.user_init ? 0.0 : whr);
    st.n_series = N;
    h->stats = st;
    h->pending.valid = false;
}

int arima_fit_batch_device(arima_handle *h, const double *d_series, int64_t n_series, int32_t T, int64_t ld,
                           int32_t p, int32_t d, int32_t q, int32_t include_intercept, int32_t method,
                           const double *d_user_init, double *d_coef_out, double *d_css_ll_out,
                           int32_t *d_status_out, int32_t *d_n_eval_out, int32_t *d_n_grad_out,
                           uint8_t *d_flags_out, void *stream) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    begin_call(h, s);
    return fit_device_locked(h, d_series, n_series, T, ld, p, d, q, include_intercept, method, d_user_init,
                             d_coef_out, d_css_ll_out, d_status_out, d_n_eval_out, d_n_grad_out, d_flags_out, s);
}

int arima_fit_batch(arima_handle *h, const double *series, int64_t N, int32_t T, int32_t p, int32_t d, int32_t q,
                    int32_t I, int32_t method, const double *user_init, double *coef_out, double *css_ll_out,
                    int32_t *status_out, int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    RCCHK(h, check_orders(h, p, d, q, I), "orders");
    if (N < 0 || T < 0 || (N > 0 && (!series || !coef_out || !css_ll_out || !status_out)))
        return set_err(h, ARIMA_E_INVALID_ARG, "bad arguments");
    if (N == 0) return ARIMA_OK;
    HIPCHK(h, hipSetDevice(h->device));
    const int k = I + p + q;
    const size_t kk = (size_t)std::max(k, 1);
    hipStream_t s = h->stream;
    begin_call(h, s);
    RCCHK(h, h->h_series.ensure((size_t)N * std::max(T, 1) * sizeof(double)), "staging");
    RCCHK(h, h->h_coef.ensure((size_t)N * kk * sizeof(double)), "staging");
    RCCHK(h, h->h_ll.ensure((size_t)N * sizeof(double)), "staging");
    RCCHK(h, h->h_status.ensure((size_t)N * sizeof(int32_t)), "staging");
    RCCHK(h, h->h_neval.ensure((size_t)N * sizeof(int32_t)), "staging");
    RCCHK(h, h->h_ngrad.ensure((size_t)N * sizeof(int32_t)), "staging");
    RCCHK(h, h->h_flags.ensure((size_t)N), "staging");
    if (T > 0) HIPCHK(h, hipMemcpyAsync(h->h_series.ptr, series, (size_t)N * T * sizeof(double), hipMemcpyHostToDevice, s));
    const double *d_ui = nullptr;
    if (user_init && k > 0) {
        RCCHK(h, h->h_uinit.ensure((size_t)N * k * sizeof(double)), "staging");
        HIPCHK(h, hipMemcpyAsync(h->h_uinit.ptr, user_init, (size_t)N * k * sizeof(double), hipMemcpyHostToDevice, s));
        d_ui = h->h_uinit.as<double>();
    } else if (user_init) {
        RCCHK(h, h->h_uinit.ensure(8), "staging");
        d_ui = h->h_uinit.as<double>();
    }
    int rc = fit_device_locked(h, h->h_series.as<double>(), N, T, T, p, d, q, I, method, d_ui, h->h_coef.as<double>(),
                               h->h_ll.as<double>(), h->h_status.as<int32_t>(), h->h_neval.as<int32_t>(),
                               h->h_ngrad.as<int32_t>(), h->h_flags.as<uint8_t>(), s);
    if (rc != ARIMA_OK) return rc;
    if (k > 0) HIPCHK(h, hipMemcpyAsync(coef_out, h->h_coef.ptr, (size_t)N * k * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipMemcpyAsync(css_ll_out, h->h_ll.ptr, (size_t)N * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipMemcpyAsync(status_out, h->h_status.ptr, (size_t)N * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (n_eval_out) HIPCHK(h, hipMemcpyAsync(n_eval_out, h->h_neval.ptr, (size_t)N * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (n_grad_out) HIPCHK(h, hipMemcpyAsync(n_grad_out, h->h_ngrad.ptr, (size_t)N * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (flags_out) HIPCHK(h, hipMemcpyAsync(flags_out, h->h_flags.ptr, (size_t)N, hipMemcpyDeviceToHost, s));
    HIPCHK(h, end_call(h, s));
    HIPCHK(h, hipStreamSynchronize(s));
    return check_fault(h);
}

// ---------------------------------------------------------------------------------------------------------
// building blocks (host buffers)
// ---------------------------------------------------------------------------------------------------------
int arima_difference_batch(arima_handle *h, const double *series, int64_t N, int32_t T, int32_t d, double *out) {
    if (!h || N < 0 || T < 0 || d < 0) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (N == 0 || T == 0) return ARIMA_OK;
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t s = h->stream;
    begin_call(h, s);
    const size_t bytes = (size_t)N * T * sizeof(double);
    RCCHK(h, h->h_series.ensure(bytes), "staging");
    RCCHK(h, h->h_aux.ensure(bytes), "staging");
    HIPCHK(h, hipMemcpyAsync(h->h_series.ptr, series, bytes, hipMemcpyHostToDevice, s));
    RCCHK(h, sts::launch_difference(h->h_series.as<double>(), T, h->h_aux.as<double>(), T, N, T, d, 0, s), "difference");
    HIPCHK(h, hipMemcpyAsync(out, h->h_aux.ptr, bytes, hipMemcpyDeviceToHost, s));
    HIPCHK(h, end_call(h, s));
    HIPCHK(h, hipStreamSynchronize(s));
    return ARIMA_OK;
}

int arima_inverse_difference_batch(arima_handle *h, const double *series, int64_t N, int32_t T, int32_t d,
                                   double *out) {
    if (!h || N < 0 || T < 0 || d < 0) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (N == 0 || T == 0) return ARIMA_OK;
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t s = h->stream;
    begin_call(h, s);
    const size_t bytes = (size_t)N * T * sizeof(double);
    RCCHK(h, h->h_series.ensure(bytes), "staging");
    RCCHK(h, h->h_aux.ensure(bytes), "staging");
    HIPCHK(h, hipMemcpyAsync(h->h_series.ptr, series, bytes, hipMemcpyHostToDevice, s));
    RCCHK(h, sts::launch_inverse_difference(h->h_series.as<double>(), T, h->h_aux.as<double>(), T, N, T, d, s),
          "inverse_difference");
    HIPCHK(h, hipMemcpyAsync(out, h->h_aux.ptr, bytes, hipMemcpyDeviceToHost, s));
    HIPCHK(h, end_call(h, s));
    HIPCHK(h, hipStreamSynchronize(s));
    return ARIMA_OK;
}

// upload N rows of length n into the padded (ld multiple of 16) workspace h->diff
static int upload_padded(arima_handle *h, const double *src, int64_t N, int32_t n, int64_t *ld_out, hipStream_t s) {
    const int64_t ld = round_up(std::max(n, 1), 16);
    RCCHK(h, h->diff.ensure((size_t)N * ld * sizeof(double)), "workspace");
    if (n > 0)
        HIPCHK(h, hipMemcpy2DAsync(h->diff.ptr, ld * sizeof(double), src, (size_t)n * sizeof(double),
                                   (size_t)n * sizeof(double), N, hipMemcpyHostToDevice, s));
    *ld_out = ld;
    return ARIMA_OK;
}

int arima_css_loglik_batch(arima_handle *h, const double *series, int64_t N, int32_t T, int32_t p, int32_t d,
                           int32_t q, int32_t I, const double *coef, double *ll_out) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    RCCHK(h, check_orders(h, p, d, q, I), "orders");
    if (N < 0 || T < 0) return set_err(h, ARIMA_E_INVALID_ARG, "bad shape");
    if (N == 0) return ARIMA_OK;
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t s = h->stream;
    begin_call(h, s);
    const int k = I + p + q;
    const int n = std::max(T - d, 0);
    const int64_t ldn = round_up(std::max(n, 1), 16);
    RCCHK(h, h->h_series.ensure((size_t)N * std::max(T, 1) * sizeof(double)), "staging");
    RCCHK(h, h->diff.ensure((size_t)N * ldn * sizeof(double)), "workspace");
    RCCHK(h, h->h_coef.ensure((size_t)N * std::max(k, 1) * sizeof(double)), "staging");
    RCCHK(h, h->h_ll.ensure((size_t)N * sizeof(double)), "staging");
    if (T > 0) HIPCHK(h, hipMemcpyAsync(h->h_series.ptr, series, (size_t)N * T * sizeof(double), hipMemcpyHostToDevice, s));
    if (k > 0) HIPCHK(h, hipMemcpyAsync(h->h_coef.ptr, coef, (size_t)N * k * sizeof(double), hipMemcpyHostToDevice, s));
    RCCHK(h, sts::launch_difference(h->h_series.as<double>(), T, h->diff.as<double>(), ldn, N, T, d, 1, s), "difference");
    RCCHK(h, sts::launch_css_loglik(h->diff.as<double>(), ldn, n, N, p, q, I, h->h_coef.as<double>(),
                                    h->h_ll.as<double>(), s), "css_loglik");
    HIPCHK(h, hipMemcpyAsync(ll_out, h->h_ll.ptr, (size_t)N * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(h, end_call(h, s));
    HIPCHK(h, hipStreamSynchronize(s));
    return ARIMA_OK;
}

int arima_css_gradient_batch(arima_handle *h, const double *diffed, int64_t N, int32_t n, int32_t p, int32_t q,
                             int32_t I, const double *coef, double *grad_out) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    RCCHK(h, check_orders(h, p, 0, q, I), "orders");
    if (N < 0 || n < 0) return set_err(h, ARIMA_E_INVALID_ARG, "bad shape");
    const int k = I + p + q;
    if (N == 0 || k == 0) return ARIMA_OK;
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t s = h->stream;
    begin_call(h, s);
    int64_t ld = 0;
    RCCHK(h, upload_padded(h, diffed, N, n, &ld, s), "upload");
    RCCHK(h, h->h_coef.ensure((size_t)N * k * sizeof(double)), "staging");
    RCCHK(h, h->h_aux.ensure((size_t)N * k * sizeof(double)), "staging");
    HIPCHK(h, hipMemcpyAsync(h->h_coef.ptr, coef, (size_t)N * k * sizeof(double), hipMemcpyHostToDevice, s));
    RCCHK(h, sts::launch_css_grad(h->diff.as<double>(), ld, n, N, p, q, I, h->smear, h->h_coef.as<double>(),
                                  h->h_aux.as<double>(), s), "css_grad");
    HIPCHK(h, hipMemcpyAsync(grad_out, h->h_aux.ptr, (size_t)N * k * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(h, end_call(h, s));
    HIPCHK(h, hipStreamSynchronize(s));
    return ARIMA_OK;
}

int arima_hannan_rissanen_batch(arima_handle *h, const double *diffed, int64_t N, int32_t n, int32_t p, int32_t q,
                                int32_t I, double *init_out, int32_t *status_out) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    RCCHK(h, check_orders(h, p, 0, q, I), "orders");
    if (N < 0 || n < 0) return set_err(h, ARIMA_E_INVALID_ARG, "bad shape");
    if (N == 0) return ARIMA_OK;
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t s = h->stream;
    begin_call(h, s);
    const int k = I + p + q;
    int64_t ld = 0;
    RCCHK(h, upload_padded(h, diffed, N, n, &ld, s), "upload");
    RCCHK(h, h->h_coef.ensure((size_t)N * std::max(k, 1) * sizeof(double)), "staging");
    RCCHK(h, h->h_status.ensure((size_t)N * sizeof(int32_t)), "staging");
    RCCHK(h, sts::launch_hr_init(h->diff.as<double>(), ld, n, N, p, q, I, h->h_coef.as<double>(),
                                 h->h_status.as<int32_t>(), s), "hr_init");
    if (k > 0) HIPCHK(h, hipMemcpyAsync(init_out, h->h_coef.ptr, (size_t)N * k * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipMemcpyAsync(status_out, h->h_status.ptr, (size_t)N * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(h, end_call(h, s));
    HIPCHK(h, hipStreamSynchronize(s));
    return ARIMA_OK;
}

int arima_model_flags_batch(arima_handle *h, const double *coef, int64_t N, int32_t p, int32_t q, int32_t I,
                            uint8_t *flags_out) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    RCCHK(h, check_orders(h, p, 0, q, I), "orders");
    if (N <= 0) return ARIMA_OK;
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t s = h->stream;
    begin_call(h, s);
    const int k = I + p + q;
    RCCHK(h, h->h_coef.ensure((size_t)N * std::max(k, 1) * sizeof(double)), "staging");
    RCCHK(h, h->h_flags.ensure((size_t)N), "staging");
    if (k > 0) HIPCHK(h, hipMemcpyAsync(h->h_coef.ptr, coef, (size_t)N * k * sizeof(double), hipMemcpyHostToDevice, s));
    RCCHK(h, sts::launch_model_flags(h->h_coef.as<double>(), N, p, q, I, h->h_flags.as<uint8_t>(), s), "flags");
    HIPCHK(h, hipMemcpyAsync(flags_out, h->h_flags.ptr, (size_t)N, hipMemcpyDeviceToHost, s));
    HIPCHK(h, end_call(h, s));
    HIPCHK(h, hipStreamSynchronize(s));
    return ARIMA_OK;
}

int arima_forecast_batch(arima_handle *h, const double *series, int64_t N, int32_t T, int32_t p, int32_t d,
                         int32_t q, int32_t I, const double *coef, int32_t n_future, double *out) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    RCCHK(h, check_orders(h, p, d, q, I), "orders");
    if (N < 0 || T < d || n_future < 0) return set_err(h, ARIMA_E_INVALID_ARG, "bad shape");
    if (N == 0) return ARIMA_OK;
    if (!series || !coef || !out) return set_err(h, ARIMA_E_INVALID_ARG, "null buffer");
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t s = h->stream;
    begin_call(h, s);
    const int k = I + p + q;
    const int64_t L = (int64_t)T + n_future;
    RCCHK(h, h->h_series.ensure((size_t)N * std::max(T, 1) * sizeof(double)), "staging");
    RCCHK(h, h->h_coef.ensure((size_t)N * std::max(k, 1) * sizeof(double)), "staging");
    RCCHK(h, h->h_aux.ensure((size_t)N * std::max<int64_t>(L, 1) * sizeof(double)), "staging");
    if (T > 0) HIPCHK(h, hipMemcpyAsync(h->h_series.ptr, series, (size_t)N * T * sizeof(double), hipMemcpyHostToDevice, s));
    if (k > 0) HIPCHK(h, hipMemcpyAsync(h->h_coef.ptr, coef, (size_t)N * k * sizeof(double), hipMemcpyHostToDevice, s));
    RCCHK(h, sts::launch_forecast(h->h_series.as<double>(), T, h->h_coef.as<double>(), k, h->h_aux.as<double>(), L, N,
                                  T, p, d, q, I, n_future, s), "forecast");
    if (L > 0) HIPCHK(h, hipMemcpyAsync(out, h->h_aux.ptr, (size_t)N * L * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(h, end_call(h, s));
    HIPCHK(h, hipStreamSynchronize(s));
    return ARIMA_OK;
}

int arima_forecast_batch_device(arima_handle *h, const double *d_series, int64_t N, int32_t T, int64_t ld,
                                int32_t p, int32_t d, int32_t q, int32_t I, const double *d_coef, int32_t n_future,
                                double *d_out, int64_t ld_out, void *stream) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    RCCHK(h, check_orders(h, p, d, q, I), "orders");
    if (N < 0 || T < d || n_future < 0 || ld < T || ld_out < (int64_t)T + n_future)
        return set_err(h, ARIMA_E_INVALID_ARG, "bad shape");
    if (N == 0) return ARIMA_OK;
    if (!d_series || !d_coef || !d_out) return set_err(h, ARIMA_E_INVALID_ARG, "null buffer");
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    begin_call(h, s);
    RCCHK(h, sts::launch_forecast(d_series, ld, d_coef, I + p + q, d_out, ld_out, N, T, p, d, q, I, n_future, s),
          "forecast");
    HIPCHK(h, end_call(h, s));
    return ARIMA_OK;
}

// ---------------------------------------------------------------------------------------------------------
// order search over (d, p, q, intercept) — SURVEY.md 8(f) row 2 (config C5)
// ---------------------------------------------------------------------------------------------------------
static int order_search_locked(arima_handle *h, const double *d_series, int64_t N, int32_t T, int64_t ld,
                               int32_t max_p, int32_t max_d, int32_t max_q, int32_t intercept_mode, int32_t method,
                               int32_t *d_order, double *d_coef, double *d_aic, int64_t *n_fits, hipStream_t s) {
    if (max_p < 0 || max_q < 0 || max_d < 0 || intercept_mode < 0 || intercept_mode > 2)
        return set_err(h, ARIMA_E_INVALID_ARG, "bad search bounds");
    if (max_p > 5 || max_q > 5 || max_d > kMaxD) return set_err(h, ARIMA_E_UNSUPPORTED, "p, q <= 5, d <= 16");
    if (N < 0 || T < 0 || ld < T || !d_order || !d_coef || !d_aic) return set_err(h, ARIMA_E_INVALID_ARG, "bad shape");
    h->pending = PendingStats{};
    h->stats = arima_fit_stats{};
    if (N == 0) return ARIMA_OK;
    HIPCHK(h, hipSetDevice(h->device));
    const int L = h->search_lanes;
    for (int j = 0; j < L; ++j) {
        SearchLane &ln = h->lanes[j];
        if (!ln.stream) {
            HIPCHK(h, hipStreamCreateWithFlags(&ln.stream, hipStreamNonBlocking));
            HIPCHK(h, hipEventCreateWithFlags(&ln.ev_fit, hipEventDisableTiming));
            HIPCHK(h, hipEventCreateWithFlags(&ln.ev_sel, hipEventDisableTiming));
        }
        RCCHK(h, ln.coef.ensure((size_t)N * 11 * sizeof(double)), "workspace");
        RCCHK(h, ln.ll.ensure((size_t)N * sizeof(double)), "workspace");
        RCCHK(h, ln.status.ensure((size_t)N * sizeof(int32_t)), "workspace");
        RCCHK(h, ln.neval.ensure((size_t)N * sizeof(int32_t)), "workspace");
        RCCHK(h, ln.ngrad.ensure((size_t)N * sizeof(int32_t)), "workspace");
        RCCHK(h, ln.flags.ensure((size_t)N), "workspace");
        // every workspace at its largest size before anything is enqueued: a growing DevBuf frees (hipFree
        // synchronises the device) and would serialise the host loop below with the fits already in flight
        RCCHK(h, ln.ws.init.ensure((size_t)N * 11 * sizeof(double)), "workspace");
        RCCHK(h, ln.ws.hr_status.ensure((size_t)N * sizeof(int32_t)), "workspace");
        RCCHK(h, ln.ws.ctl.ensure(kCtlWords * sizeof(unsigned long long)), "workspace");
        RCCHK(h, ln.ws.xring.ensure(sts::kExpressRingBytes), "workspace");
        RCCHK(h, ln.ws.xready.ensure(sts::kExpressReadyBytes), "workspace");
    }
    for (int d = 0; d <= max_d; ++d)
        RCCHK(h, h->os_diff[d].ensure((size_t)N * round_up(std::max(T - d, 1), 16) * sizeof(double)), "workspace");
    HIPCHK(h, hipEventRecord(h->ev[0], s));
    RCCHK(h, sts::launch_search_init(d_aic, d_order, d_coef, N, s), "search_init");
    const int i_lo = intercept_mode == 1 ? 1 : 0, i_hi = intercept_mode == 0 ? 0 : 1;
    int64_t fits = 0;
    for (int d = 0; d <= max_d; ++d) {
        // differencesOfOrderD once per d (ARIMA.scala:88), shared read-only by that d's fits on every lane
        const int n = std::max(T - d, 0);
        const int64_t ldn = round_up(std::max(n, 1), 16);
        RCCHK(h, h->os_diff[d].ensure((size_t)N * ldn * sizeof(double)), "workspace");
        if (!h->ev_diff[d]) HIPCHK(h, hipEventCreateWithFlags(&h->ev_diff[d], hipEventDisableTiming));
        RCCHK(h, sts::launch_difference(d_series, ld, h->os_diff[d].as<double>(), ldn, N, T, d, 1, s), "difference");
        HIPCHK(h, hipEventRecord(h->ev_diff[d], s));
        for (int p = 0; p <= max_p; ++p)
            for (int q = 0; q <= max_q; ++q)
                for (int I = i_lo; I <= i_hi; ++I) {
                    // ARIMA(0,d,0) without intercept has no parameters: the reference throws (NoDataException);
                    // fit_kernels reports it per series and the select step skips it.
                    SearchLane &ln = h->lanes[fits % L];
                    HIPCHK(h, hipStreamWaitEvent(ln.stream, h->ev_diff[d], 0));
                    if (ln.sel_recorded) HIPCHK(h, hipStreamWaitEvent(ln.stream, ln.ev_sel, 0));  // outputs read
                    int64_t grid = 0, xb = 0;
                    RCCHK(h, fit_kernels(h, ln.ws, h->os_diff[d].as<double>(), ldn, n, N, p, q, I, method, nullptr,
                                         ln.coef.as<double>(), ln.ll.as<double>(), ln.status.as<int32_t>(),
                                         ln.neval.as<int32_t>(), ln.ngrad.as<int32_t>(), ln.flags.as<uint8_t>(),
                                         ln.stream, nullptr, &grid, &xb, L > 1), "fit");
                    HIPCHK(h, hipEventRecord(ln.ev_fit, ln.stream));
                    // candidates are merged in grid order on the call's stream (first minimum wins, as minBy)
                    HIPCHK(h, hipStreamWaitEvent(s, ln.ev_fit, 0));
                    RCCHK(h, sts::launch_search_select(ln.coef.as<double>(), ln.ll.as<double>(),
                                                       ln.status.as<int32_t>(), ln.flags.as<uint8_t>(), N, p, d, q, I,
                                                       d_aic, d_order, d_coef, s),
                          "search_select");
                    HIPCHK(h, hipEventRecord(ln.ev_sel, s));
                    ln.sel_recorded = true;
                    ++fits;
                }
    }
    HIPCHK(h, hipEventRecord(h->ev[3], s));
    if (n_fits) *n_fits = fits;
    return ARIMA_OK;
}

int arima_order_search_batch_device(arima_handle *h, const double *d_series, int64_t n_series, int32_t T,
                                    int64_t ld, int32_t max_p, int32_t max_d, int32_t max_q,
                                    int32_t intercept_mode, int32_t method, int32_t *d_order_out,
                                    double *d_coef_out, double *d_aic_out, void *stream) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    begin_call(h, s);
    const int rc = order_search_locked(h, d_series, n_series, T, ld, max_p, max_d, max_q, intercept_mode, method,
                                       d_order_out, d_coef_out, d_aic_out, nullptr, s);
    if (rc != ARIMA_OK) return rc;
    HIPCHK(h, end_call(h, s));
    return ARIMA_OK;
}

int arima_order_search_batch(arima_handle *h, const double *series, int64_t N, int32_t T, int32_t max_p,
                             int32_t max_d, int32_t max_q, int32_t intercept_mode, int32_t method,
                             int32_t *order_out, double *coef_out, double *aic_out) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (N < 0 || T < 0) return set_err(h, ARIMA_E_INVALID_ARG, "bad shape");
    if (N == 0) return ARIMA_OK;
    if (!series || !order_out || !coef_out || !aic_out) return set_err(h, ARIMA_E_INVALID_ARG, "null buffer");
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t s = h->stream;
    begin_call(h, s);
    RCCHK(h, h->h_series.ensure((size_t)N * std::max(T, 1) * sizeof(double)), "staging");
    RCCHK(h, h->h_aux.ensure((size_t)N * 11 * sizeof(double)), "staging");
    RCCHK(h, h->h_ll.ensure((size_t)N * sizeof(double)), "staging");
    RCCHK(h, h->os_order.ensure((size_t)N * 4 * sizeof(int32_t)), "staging");
    if (T > 0) HIPCHK(h, hipMemcpyAsync(h->h_series.ptr, series, (size_t)N * T * sizeof(double), hipMemcpyHostToDevice, s));
    int rc = order_search_locked(h, h->h_series.as<double>(), N, T, T, max_p, max_d, max_q, intercept_mode, method,
                                 h->os_order.as<int32_t>(), h->h_aux.as<double>(), h->h_ll.as<double>(), nullptr, s);
    if (rc != ARIMA_OK) return rc;
    HIPCHK(h, hipMemcpyAsync(order_out, h->os_order.ptr, (size_t)N * 4 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipMemcpyAsync(coef_out, h->h_aux.ptr, (size_t)N * 11 * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipMemcpyAsync(aic_out, h->h_ll.ptr, (size_t)N * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(h, end_call(h, s));
    HIPCHK(h, hipStreamSynchronize(s));
    return ARIMA_OK;
}

int arima_sample_batch_device(arima_handle *h, double *d_series, int64_t N, int32_t T, int64_t ld, int32_t p,
                              int32_t d, int32_t q, int32_t I, const double *base_coef, double jitter,
                              uint64_t seed, int64_t first_series, void *stream) {
    if (!h || !base_coef || N < 0 || T < 0 || ld < T) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    RCCHK(h, check_orders(h, p, d, q, I), "orders");
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    begin_call(h, s);
    RCCHK(h, sts::launch_sample(d_series, ld, N, T, p, d, q, I, base_coef, jitter, seed, first_series, s), "sample");
    HIPCHK(h, end_call(h, s));
    return ARIMA_OK;
}

}  // extern "C"
