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
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

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
constexpr int kCtlWords = sts::kFitCtlWords;   // device counters of the fit kernel (k_cg_fit's ctl[]; ctl[32] = series written)

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
    DevBuf best_aic, best_order, best_coef;    // this lane's best candidate per series (merged at the end)
    DevBuf acc;                                // kCtlWords counter sums over the lane's fits + their flops (double)
};

// A device fit larger than one slice (option "fit_slice_bytes" of differenced workspace; default 0 = 60 % of the free
// HBM over the fit contexts) runs as consecutive slices over the fit contexts: the workspaces stay bounded whatever
// the batch (C3's 8M series on one GPU), and the slices pipeline like consecutive calls. Every slice takes the next slot of a ring with
// its own timing events and its own pinned copy of the kernel counters, so the call's stats cover every slice. A
// slot is reused only once its previous slice's copy has landed (host check on its last event).
constexpr int kSliceSlots = 64;
struct SliceSlot {
    hipEvent_t ev[5] = {};                 // start, after differencing, after init, after fit, after the counter copy
    bool used = false;
    PendingStats ps;
};

constexpr int kMaxSearchLanes = sts::kSearchMaxLanes;
constexpr int kMaxD = 16;
constexpr int kMaxPipeline = 8;
constexpr int64_t kBobyqaWaveMaxN = 4096;     // css-bobyqa fits up to this many series: a wave per series

// One fit context: what a fit call needs for itself (stream, differenced-series workspace, HR init, kernel counters,
// timing events, pinned counter copy, host-path staging). Fit calls rotate over h->pipeline contexts, so with
// pipeline > 1 consecutive fits run concurrently and the tail of one fit kernel (its slowest series) overlaps the
// next fit's differencing, init and bulk work; a context is reused only after its previous call has finished.
// One device-fit call's caller buffers as byte ranges [lo, hi) (series rows and user inits read; the six outputs
// written) -- fit_pipeline > 1 hazard tracking
struct CallSpans {
    uintptr_t in[2][2] = {}, out[6][2] = {};
};
constexpr int kInflightMax = 16;   // tracked calls per context; beyond, every later call waits for that context
struct Inflight {                  // the device-fit calls on one context that may not have finished yet
    CallSpans call[kInflightMax];
    hipEvent_t ev[kInflightMax] = {};   // each call's end (a hazard waits for exactly that call)
    int n = 0;
    bool overflow = false;
};

struct FitCtx {
    hipStream_t stream = nullptr;
    hipEvent_t ev[kNumEvents] = {};
    hipEvent_t ev_done = nullptr;             // end of this context's last call
    bool has_done = false;
    Inflight inflight;                        // its device-fit calls' caller buffers (fit_pipeline > 1)
    DevBuf diff;
    FitWs ws;
    unsigned long long *ctl_host = nullptr;   // pinned
    PendingStats pending;
    bool fit_ctl = false;                     // ctl_host holds (or will hold, in stream order) the kernel counters
    // host path (arima_fit_batch): device copies of one chunk and pinned staging of its input and outputs
    DevBuf d_series, d_coef, d_ll, d_status, d_neval, d_ngrad, d_flags, d_uinit;
    void *pin = nullptr;
    size_t pin_bytes = 0;
    int64_t chunk_first = -1, chunk_n = 0;    // the chunk whose results wait in `pin`
};

inline void set_span(uintptr_t (&sp)[2], const void *p, int64_t bytes) {
    sp[0] = (uintptr_t)p;
    sp[1] = p && bytes > 0 ? (uintptr_t)p + (uintptr_t)bytes : (uintptr_t)p;
}

inline bool spans_meet(const uintptr_t (&a)[2], const uintptr_t (&b)[2]) {
    return a[0] < a[1] && b[0] < b[1] && a[0] < b[1] && b[0] < a[1];
}

}  // namespace

struct arima_handle {
    int device = 0;
    int num_cus = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[kNumEvents] = {};
    hipEvent_t ev_done = nullptr;     // end of the last non-fit call's device work
    bool has_done = false;
    mutable std::mutex mu;
    std::string err;
    arima_fit_stats stats{};
    int smear = 1;           // Breeze 0.12 overlap semantics at ARIMA.scala:526: element-wise copy
    int grid_blocks_override = 0;
    int express_blocks = -1;       // k_cg_fit express workgroups (-1: num_cus / 16)
    int express_ring = 0;          // express hand-offs per launch (0: the whole ring, sts::kExpressRingEntries)
    int merge_live = sts::kMergeLiveDefault;    // k_cg_fit drain merge: hand over at <= this many live slots (0: off)
    // express CUs of the order search's concurrent fits (-1: as "express_blocks"). 0 by default: with 16 lanes in
    // flight each fit's express workgroups held whole CUs for the fit's duration, mostly waiting (C5 262 144:
    // 14 728 series/s with them, 16 659 without; profiles/r04/g_merge)
    int search_express_blocks = 0;
    int donate_evals = 0;          // k_cg_fit: evaluations before a slot may go to an express wave (0: kernel default)
    int donate_evals_drained = 0;  // ... once the batch's work counter has run out (0: kernel default)
    int chain_overhead = 0;        // k_cg_fit's objective-pass width model, 1/16 chains per step (0: kernel default 6)
    // k_hr_init: 0 = a lane per series; > 0 = that many single-wave workgroups (grid-stride); -1 (default) = 1 024
    // for pipelined device fits (fit_pipeline > 1: C2 9.47-9.55 -> 9.68-9.75 M series/s, profiles/r04/m_hrgrid),
    // else 0 (alone it is 25.2 vs 26.9 ms at C2)
    int hr_grid = -1;
    int row_pad = 0;               // doubles (multiple of 16) added to the differenced rows' stride
    // css-bobyqa layout: 1 = a wave per series (state in LDS), 0 = a lane per series, -1 (default) = a wave per series
    // for autoFit's retries and for fits of <= kBobyqaWaveMaxN series, else a lane per series. Bit-identical; measured
    // on C2 series: 1 024 fits 0.20 (wave) vs 0.62 s (lane), 16 384 fits ~1.6 (8 x the 1 024-series wave time: 2 048
    // series resident) vs 0.96 s, 65 536 fits 3.56 vs 1.79 s, autoFit of 65 536 series 11.98 vs 35.0 s
    // (profiles/r05/q_wave, r_occ2, g_tmpl). An objective parallel in time over the row in LDS (css_pit_lds) was
    // slower in this kernel: autoFit 19.3 s, 1 024 fits 0.27 s (s_pit)
    int bobyqa_wave = -1;
    // 1: device fits of d <= 1 difference into the k_difference workspace as before round 6 instead of reading the
    // caller's rows (option "fuse_diff" 0; results are identical, tests compare the two)
    int fuse_mode = 1;             // option "fuse_diff": 0 never, 1 where it pays (sts::fuse_pays), 2 always
    int64_t last_express = 0;
    int64_t last_grid = 0;
    int search_lanes = 8;          // concurrent fits of the order search (2/4/8: 1269/1303/1408 series/s, profiles/r02/g_c5)
    // fit contexts in rotation for device fits (option "fit_pipeline"). Default 3: consecutive asynchronous calls
    // overlap (one call's tail with the next one's differencing, init and bulk passes) and calls that share buffers
    // stay ordered (order_after_overlapping_fits). On the box's 4 hardware queues at C2 1M x 1024, 5 consecutive
    // calls: 1 / 2 / 3 / 4 contexts 6.68 / 8.30 / 10.02 / 9.97 M series/s; one call alone 151 ms at 1, 162 ms at 3
    // (drained bulk waves leave instead of turning express) -- profiles/r05/k_defp
    int pipeline = 3;
    // (Cutting ONE call into slices over several contexts was measured on the box's 4 queues at C2 1M x 1024 and
    // removed: 1 / 2 / 3 / 4 slices 6.91 / 6.39 / 6.35 / 4.47 M series/s, every slice ends with its own slowest
    // series; profiles/r05/c_af2/default_cs*.json.)
    // host path (arima_fit_batch): chunks of host_chunk series over host_pipeline fit contexts, the last ones halved
    // (host_tail). C2 1M x 1024 from pageable memory, 8 hardware queues: 262144 x 3 contexts 3.86 M series/s,
    // 131072 x 6 4.47-4.65, 65536 x 6 3.65 (profiles/r06/g_e2e); the upload runs at the link's 56 GB/s either way
    // (tools/h2d_bw.py, profiles/r06/d_ab/h2d.json), so the call is bound by the uploads plus its last fit's tail
    static constexpr int64_t kHostTailMin = 16384;
    int host_pipeline = 3;         // contexts the chunked host path rotates over (option "host_pipeline"; arima_create)
    int64_t host_chunk = 1 << 18;  // series per chunk of the host path (option "host_chunk"; arima_create)
    int host_tail = 1;             // halve the last chunks (option "host_tail")
    // host path uploads: with host_copy_threads > 0 the caller's pageable rows are copied by that many threads into a
    // ring of pinned blocks, each block DMA'd while the threads fill the next (upload_staged); 0 (default) uploads
    // straight from pageable memory through the HIP runtime's own staging. Both reach the link's ~56 GB/s on the box
    // (tools/h2d_bw.py), and the runtime's staging measured slightly faster end to end (4.65 vs 4.47 M series/s at
    // C2, profiles/r06/g_e2e), so the staged ring stays an option for hosts whose pageable path is slower.
    int host_copy_threads = 0;
    static constexpr int kStageSlots = 3;
    static constexpr size_t kStageBytes = size_t(128) << 20;
    void *stage[kStageSlots] = {};
    hipEvent_t stage_ev[kStageSlots] = {};
    bool stage_used[kStageSlots] = {};
    unsigned stage_next = 0;
    int64_t fit_slice_bytes = 0;   // differenced workspace of one device-fit slice (option "fit_slice_bytes"; 0: from free HBM)
    SliceSlot slot[kSliceSlots];
    unsigned long long *slot_ctl = nullptr;     // pinned, kCtlWords per slot
    unsigned slot_seq = 0;                      // slots taken so far
    unsigned slice_first = 0, slice_n = 0;      // slots of the last sliced fit call still pending (stats_ctx == -2)
    arima_fit_stats slice_acc{};                // ... and the stats of its slices whose slots were already reused
    DevBuf dev_fault;                           // sticky device record of the first fit-kernel fault (6 words)
    unsigned fit_seq = 0;          // fit calls so far (selects the context)
    int stats_ctx = -1;            // context of the last fit (arima_get_last_stats), -1: none
    arima_fit_stats host_acc{};    // host path: counters summed over its chunks
    FitCtx fctx[kMaxPipeline];
    // device workspaces of the building blocks
    DevBuf diff;
    DevBuf fc_ws;                  // the runtime-order forecast's per-series arrays (forecast_any)
    // host-API staging
    DevBuf h_series, h_coef, h_ll, h_status, h_neval, h_ngrad, h_flags, h_uinit, h_aux;
    // order search: the differenced series per d, the concurrent fit lanes, host-API staging of the orders
    DevBuf os_diff[kMaxD + 1];
    hipEvent_t ev_diff[kMaxD + 1] = {};
    SearchLane lanes[kMaxSearchLanes];
    DevBuf os_order;
    unsigned long long *search_acc_host = nullptr;   // pinned: (kCtlWords + 1) words per lane of the last search
    // autoFit (arima_autofit_batch*): the differenced rows, the walk state, the rounds' per-order lists and results
    DevBuf af_rows, af_dsel, af_state, af_best, af_counts, af_lists, af_off, af_coef, af_ll, af_status, af_flags;
    DevBuf af_init, af_hrst, af_rlist, af_rcount;     // the round's inits and the css-bobyqa retry list
    DevBuf af_out_order, af_out_coef, af_out_aic, af_out_status, af_out_nfits;   // host-API staging
    int64_t *af_host = nullptr;                      // pinned: kAfCombosMax counts, kAfCombosMax row offsets, the retry count
    hipEvent_t ev_af = nullptr;
    int search_lanes_used = 0;
    int64_t search_n = 0, search_fits = 0;
    int64_t autofit_slice = 0;     // autoFit series per slice (option "autofit_slice"; 0 = from free HBM)
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
// Leading dimension of a differenced-row workspace: 128-B aligned rows of n doubles plus the handle's row_pad
static int64_t row_stride(const arima_handle *h, int64_t n) { return round_up(std::max<int64_t>(n, 1), 16) + h->row_pad; }

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

// Take (read and clear) the sticky fault record rec[0..5] into rec[8..13] with atomic exchanges: a fault that a
// concurrent k_fault_merge records after the exchange of rec[0] stays for the next take instead of being cleared
// unseen (a plain read followed by a memset could lose it).
__global__ void k_fault_take(unsigned long long *__restrict__ rec) {
    if (threadIdx.x != 0) return;
    const unsigned long long code = atomicExch(&rec[0], 0ull);
    rec[8] = code;
    for (int i = 1; i < 6; ++i) rec[8 + i] = code ? atomicExch(&rec[i], 0ull) : 0ull;
}

// One grid point's fit into its search lane's counter sums (order-search stats, arima_get_last_stats): every kernel
// counter word, and the fit's algorithmic flops by compute_stats' formula. cg = 0: the AR-only
// shortcut or a uniform status (no counters; every series written). The fault words ctl[26..31] are not summed: the
// lane keeps the first fault any of its fits recorded.
__global__ void k_search_acc(const unsigned long long *__restrict__ ctl, unsigned long long *__restrict__ acc,
                             int64_t N, int n, int p, int q, int I, int cg) {
    if (threadIdx.x != 0) return;
    for (int i = 0; i < kCtlWords; ++i)
        if (i < 26 || i > 31) acc[i] += ctl[i];
    if (acc[26] == 0 && ctl[26] != 0)
        for (int i = 26; i <= 31; ++i) acc[i] = ctl[i];
    if (!cg) acc[32] += (unsigned long long)N;
    const int k = I + p + q, M = p > q ? p : q, m = M + 1;
    const double S = n - M > 0 ? n - M : 0;
    const double ff = 2.0 * (p + q) + 4, fg = ff + 2.0 * k * q + 1 + p + q + 2.0 * k;
    const double U = (double)(ctl[1] + ctl[18] + ctl[24] + ctl[7]), G = (double)(ctl[2] - ctl[18] + ctl[25]);
    // the AR-only shortcut (p > 0, q == 0) runs one OLS, not the Hannan-Rissanen init
    const bool ar_only = p > 0 && q == 0;
    const double whr = ar_only ? 0.0
                               : (double)N * (3.0 * (n - m > 0 ? n - m : 0) * (m + 1) * (m + 1) +
                                              3.0 * (n - 2 * M - 1 > 0 ? n - 2 * M - 1 : 0) * k * k +
                                              2.0 * (n - m > 0 ? n - m : 0) * m);
    double *fl = reinterpret_cast<double *>(acc + kCtlWords);
    *fl = *fl + U * S * ff + G * S * fg + whr;
}

// the first watchdog fault of a fit kernel (its ctl[26..31]) into the handle's sticky device record
__global__ void k_fault_merge(const unsigned long long *__restrict__ ctl, unsigned long long *__restrict__ rec) {
    if (threadIdx.x != 0 || ctl[26] == 0) return;
    if (atomicCAS(&rec[0], 0ull, ctl[26]) == 0ull)
        for (int i = 1; i < 6; ++i) rec[i] = ctl[26 + i];
}

// p, q <= 5: the order-specialised kernels; 5 < p, q <= kGenMaxOrder (20): the runtime-order path (arima_generic.hip)
int check_orders(arima_handle *h, int p, int d, int q, int I) {
    if (p < 0 || q < 0 || d < 0 || (I != 0 && I != 1)) return set_err(h, ARIMA_E_INVALID_ARG, "bad order");
    if (!sts::gen_orders_ok(p, q)) return set_err(h, ARIMA_E_UNSUPPORTED, "p, q <= 20");
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
    case ARIMA_ST_NOT_STATIONARY: return "NOT_STATIONARY";
    case ARIMA_ST_NO_MODEL: return "NO_MODEL";
    case ARIMA_ST_TOO_FEW_PARAMS: return "TOO_FEW_PARAMS";
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
    // the host path's contexts need hardware queues of their own (HIP maps a process's streams onto
    // GPU_MAX_HW_QUEUES of them, default 4): 6 contexts of 131072-series chunks with 8 or more queues, else 3 of 262144
    // (profiles/r06/e_split, g_e2e: on 4 queues 4+ contexts serialise and run slower than 3)
    if (const char *q = getenv("GPU_MAX_HW_QUEUES")) {
        if (atoi(q) >= 8) {
            h->host_pipeline = 6;
            h->host_chunk = 1 << 17;
        }
    }
    hipDeviceGetAttribute(&h->num_cus, hipDeviceAttributeMultiprocessorCount, device);
    int rc = ARIMA_OK;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) rc = ARIMA_E_DEVICE;
    for (auto &e : h->ev)
        if (rc == ARIMA_OK && hipEventCreate(&e) != hipSuccess) rc = ARIMA_E_DEVICE;
    if (rc == ARIMA_OK && hipEventCreateWithFlags(&h->ev_done, hipEventDisableTiming) != hipSuccess) rc = ARIMA_E_DEVICE;
    for (auto &c : h->fctx) {
        if (rc == ARIMA_OK && hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking) != hipSuccess) rc = ARIMA_E_DEVICE;
        for (auto &e : c.ev)
            if (rc == ARIMA_OK && hipEventCreate(&e) != hipSuccess) rc = ARIMA_E_DEVICE;
        if (rc == ARIMA_OK && hipEventCreateWithFlags(&c.ev_done, hipEventDisableTiming) != hipSuccess) rc = ARIMA_E_DEVICE;
        if (rc == ARIMA_OK && hipHostMalloc((void **)&c.ctl_host, kCtlWords * sizeof(unsigned long long), 0) != hipSuccess)
            rc = ARIMA_E_OOM;
    }
    if (rc == ARIMA_OK &&
        hipHostMalloc((void **)&h->slot_ctl, (size_t)kSliceSlots * kCtlWords * sizeof(unsigned long long), 0) != hipSuccess)
        rc = ARIMA_E_OOM;
    if (rc == ARIMA_OK && hipHostMalloc((void **)&h->search_acc_host,
                                        (size_t)kMaxSearchLanes * (kCtlWords + 1) * sizeof(unsigned long long), 0) != hipSuccess)
        rc = ARIMA_E_OOM;
    if (rc == ARIMA_OK && h->dev_fault.ensure(16 * sizeof(unsigned long long)) != ARIMA_OK) rc = ARIMA_E_OOM;
    if (rc == ARIMA_OK && hipMemset(h->dev_fault.ptr, 0, 16 * sizeof(unsigned long long)) != hipSuccess) rc = ARIMA_E_DEVICE;
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
    for (auto &c : h->fctx) {
        if (c.stream) {
            hipStreamSynchronize(c.stream);
            hipStreamDestroy(c.stream);
        }
        for (auto &e : c.ev)
            if (e) hipEventDestroy(e);
        if (c.ev_done) hipEventDestroy(c.ev_done);
        for (auto &e : c.inflight.ev)
            if (e) hipEventDestroy(e);
        if (c.ctl_host) hipHostFree(c.ctl_host);
        if (c.pin) hipHostFree(c.pin);
    }
    for (auto &e : h->ev_diff)
        if (e) hipEventDestroy(e);
    for (auto &sl : h->slot)
        for (auto &e : sl.ev)
            if (e) hipEventDestroy(e);
    for (int j = 0; j < arima_handle::kStageSlots; ++j) {
        if (h->stage_ev[j]) {
            hipEventSynchronize(h->stage_ev[j]);
            hipEventDestroy(h->stage_ev[j]);
        }
        if (h->stage[j]) hipHostFree(h->stage[j]);
    }
    if (h->slot_ctl) hipHostFree(h->slot_ctl);
    if (h->search_acc_host) hipHostFree(h->search_acc_host);
    if (h->af_host) hipHostFree(h->af_host);
    if (h->ev_af) hipEventDestroy(h->ev_af);
    for (auto &e : h->ev)
        if (e) hipEventDestroy(e);
    if (h->ev_done) hipEventDestroy(h->ev_done);
    if (h->stream) hipStreamDestroy(h->stream);
    delete h;                                  // every DevBuf workspace frees itself
    return ARIMA_OK;
}

const char *arima_last_error(const arima_handle *h) { return h ? h->err.c_str() : "null handle"; }

static void finish_stats(arima_handle *h, FitCtx &c);
static arima_fit_stats compute_stats(const PendingStats &ps, const unsigned long long *cc, const hipEvent_t *ev);
static void acc_stats(arima_fit_stats &a, const arima_fit_stats &s);

int arima_get_last_stats(const arima_handle *hc, arima_fit_stats *out) {
    if (!hc || !out) return ARIMA_E_INVALID_ARG;
    arima_handle *h = const_cast<arima_handle *>(hc);   // the lazy completion below only fills h->stats
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->stats_ctx >= 0 && h->fctx[h->stats_ctx].pending.valid) {
        FitCtx &c = h->fctx[h->stats_ctx];
        hipSetDevice(h->device);
        if (hipEventSynchronize(c.ev_done) != hipSuccess) return set_err(h, ARIMA_E_DEVICE, "stats: device error");
        finish_stats(h, c);
    } else if (h->stats_ctx == -2 && h->slice_n > 0) {   // a sliced fit: the sum over its slices
        hipSetDevice(h->device);
        arima_fit_stats acc = h->slice_acc;
        for (unsigned j = 0; j < h->slice_n; ++j) {
            const unsigned sl = (h->slice_first + j) % kSliceSlots;
            SliceSlot &ss = h->slot[sl];
            if (hipEventSynchronize(ss.ev[4]) != hipSuccess) return set_err(h, ARIMA_E_DEVICE, "stats: device error");
            acc_stats(acc, compute_stats(ss.ps, h->slot_ctl + (size_t)sl * kCtlWords, ss.ev));
        }
        h->stats = acc;
        h->slice_n = 0;
        h->slice_acc = arima_fit_stats{};
    } else if (h->stats_ctx == -3 && h->search_lanes_used > 0) {   // an order search: the sums over its fits
        hipSetDevice(h->device);
        if (hipEventSynchronize(h->ev[4]) != hipSuccess) return set_err(h, ARIMA_E_DEVICE, "stats: device error");
        arima_fit_stats st{};
        double flops = 0.0;
        unsigned long long w[kCtlWords] = {};
        for (int j = 0; j < h->search_lanes_used; ++j) {
            const unsigned long long *a = h->search_acc_host + (size_t)j * (kCtlWords + 1);
            for (int i = 0; i < kCtlWords; ++i)
                if (i < 26 || i > 31) w[i] += a[i];
            if (w[26] == 0 && a[26] != 0)                    // the first lane's recorded fault
                for (int i = 26; i <= 31; ++i) w[i] = a[i];
            double f;
            memcpy(&f, a + kCtlWords, sizeof f);
            flops += f;
        }
        st.n_series = h->search_n * h->search_fits;          // fits (series x grid points)
        st.f_passes = (int64_t)w[1];
        st.g_passes = (int64_t)w[2];
        st.wave_f_passes = (int64_t)w[3];
        st.wave_g_passes = (int64_t)w[4];
        st.n_eval = (int64_t)w[5];
        st.n_grad = (int64_t)w[6];
        st.spec_hits = (int64_t)w[7];
        st.wave_multi_passes = (int64_t)w[8];
        st.spec_chains = (int64_t)w[9];
        st.ride_passes = (int64_t)w[18];
        st.express_series = (int64_t)w[23];
        st.express_f_passes = (int64_t)w[24];
        st.express_g_passes = (int64_t)w[25];
        st.series_done = (int64_t)w[32];
        st.express_pit_passes = (int64_t)w[33];
        st.express_pit_sweeps = (int64_t)w[34];
        st.express_pit_g_passes = (int64_t)w[35];
        st.wave_chains = (int64_t)w[36];
        st.low_util_passes = (int64_t)w[37];
        st.merge_series = (int64_t)w[41];
        st.merge_waves = (int64_t)w[42];
        st.fault = (int64_t)w[26];
        for (int i = 0; i < 5; ++i) st.fault_info[i] = (int64_t)w[27 + i];
        st.grid_blocks = h->last_grid;
        st.express_blocks = h->last_express;
        st.flops = flops;
        float ms = 0;
        hipEventElapsedTime(&ms, h->ev[0], h->ev[3]);
        st.ms_cg_fit = ms;
        st.ms_total = ms;
        h->stats = st;
        h->search_lanes_used = 0;
    }
    *out = h->stats;
    return ARIMA_OK;
}

// A finished fit kernel of context c recorded a watchdog fault (k_cg_fit's hand-off): its results are incomplete.
static int check_fault(arima_handle *h, FitCtx &c) {
    if (c.fit_ctl && c.ctl_host[26] != 0) {
        c.fit_ctl = false;                      // reported once
        char msg[160];
        snprintf(msg, sizeof msg, "fit kernel watchdog fault %llu (info %llu %llu %llu %llu %llu)", c.ctl_host[26],
                 c.ctl_host[27], c.ctl_host[28], c.ctl_host[29], c.ctl_host[30], c.ctl_host[31]);
        return set_err(h, ARIMA_E_DEVICE, msg);
    }
    return ARIMA_OK;
}

static int take_fault(arima_handle *h);

int arima_synchronize(arima_handle *h) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    HIPCHK(h, hipSetDevice(h->device));
    if (h->has_done) HIPCHK(h, hipEventSynchronize(h->ev_done));
    int rc = ARIMA_OK;
    for (auto &c : h->fctx) {
        if (c.has_done) HIPCHK(h, hipEventSynchronize(c.ev_done));
        if (rc == ARIMA_OK) rc = check_fault(h, c);
    }
    for (auto &l : h->lanes)
        if (l.stream) HIPCHK(h, hipStreamSynchronize(l.stream));
    // the sticky record every fit kernel's counters are merged into (sliced fits, order-search lanes, contexts whose
    // pinned counters a later call has already overwritten)
    const int rf = take_fault(h);
    if (rc == ARIMA_OK) rc = rf;
    return rc;
}

int arima_set_option(arima_handle *h, const char *name, int64_t value) {
    if (!h || !name) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (!strcmp(name, "smear")) { h->smear = value ? 1 : 0; return ARIMA_OK; }
    if (!strcmp(name, "bobyqa_wave")) { h->bobyqa_wave = value < 0 ? -1 : (value ? 1 : 0); return ARIMA_OK; }
    if (!strcmp(name, "fuse_diff")) { h->fuse_mode = (int)std::min<int64_t>(2, std::max<int64_t>(0, value)); return ARIMA_OK; }
    if (!strcmp(name, "chain_overhead")) { h->chain_overhead = (int)std::min<int64_t>(4096, std::max<int64_t>(0, value)); return ARIMA_OK; }
    if (!strcmp(name, "autofit_slice")) { h->autofit_slice = std::max<int64_t>(0, value); return ARIMA_OK; }
    if (!strcmp(name, "row_pad")) {                 // doubles, rounded up to whole 128-B lines
        h->row_pad = (int)round_up(std::min<int64_t>(4096, std::max<int64_t>(0, value)), 16);
        return ARIMA_OK;
    }
    if (!strcmp(name, "hr_grid")) { h->hr_grid = (int)std::min<int64_t>(1 << 20, std::max<int64_t>(-1, value)); return ARIMA_OK; }
    if (!strcmp(name, "express_ring")) {
        h->express_ring = (int)std::min<int64_t>(sts::kExpressRingEntries, std::max<int64_t>(0, value));
        return ARIMA_OK;
    }
    if (!strcmp(name, "search_express_blocks")) {
        h->search_express_blocks = (int)std::max<int64_t>(-1, value);
        return ARIMA_OK;
    }
    if (!strcmp(name, "donate_evals")) { h->donate_evals = (int)std::max<int64_t>(0, value); return ARIMA_OK; }
    if (!strcmp(name, "donate_evals_drained")) {
        h->donate_evals_drained = (int)std::max<int64_t>(0, value);
        return ARIMA_OK;
    }
    if (!strcmp(name, "merge_live")) { h->merge_live = (int)std::min<int64_t>(64, std::max<int64_t>(0, value)); return ARIMA_OK; }
    if (!strcmp(name, "express_blocks")) { h->express_blocks = (int)std::max<int64_t>(-1, value); return ARIMA_OK; }
    if (!strcmp(name, "grid_blocks")) { h->grid_blocks_override = (int)std::max<int64_t>(0, value); return ARIMA_OK; }
    if (!strcmp(name, "search_lanes")) {
        h->search_lanes = (int)std::min<int64_t>(kMaxSearchLanes, std::max<int64_t>(1, value));
        return ARIMA_OK;
    }
    if (!strcmp(name, "fit_pipeline")) {
        h->pipeline = (int)std::min<int64_t>(kMaxPipeline, std::max<int64_t>(1, value));
        return ARIMA_OK;
    }
    if (!strcmp(name, "host_pipeline")) {
        h->host_pipeline = (int)std::min<int64_t>(kMaxPipeline, std::max<int64_t>(1, value));
        return ARIMA_OK;
    }
    if (!strcmp(name, "host_chunk")) { h->host_chunk = std::max<int64_t>(1, value); return ARIMA_OK; }
    if (!strcmp(name, "host_tail")) { h->host_tail = value ? 1 : 0; return ARIMA_OK; }
    if (!strcmp(name, "host_copy_threads")) {
        h->host_copy_threads = (int)std::min<int64_t>(64, std::max<int64_t>(0, value));
        return ARIMA_OK;
    }
    if (!strcmp(name, "fit_slice_bytes")) { h->fit_slice_bytes = std::max<int64_t>(0, value); return ARIMA_OK; }
    return set_err(h, ARIMA_E_INVALID_ARG, "unknown option");
}

int arima_get_option(const arima_handle *hc, const char *name, int64_t *value) {
    if (!hc || !name || !value) return ARIMA_E_INVALID_ARG;
    const arima_handle *h = hc;
    std::lock_guard<std::mutex> lk(h->mu);
    const struct { const char *n; int64_t v; } opts[] = {
        {"smear", h->smear}, {"express_blocks", h->express_blocks}, {"grid_blocks", h->grid_blocks_override},
        {"search_lanes", h->search_lanes}, {"fit_pipeline", h->pipeline}, {"host_pipeline", h->host_pipeline},
        {"host_chunk", h->host_chunk}, {"fit_slice_bytes", h->fit_slice_bytes}, {"express_ring", h->express_ring},
        {"hr_grid", h->hr_grid}, {"row_pad", h->row_pad}, {"bobyqa_wave", h->bobyqa_wave}, {"merge_live", h->merge_live},
        {"search_express_blocks", h->search_express_blocks}, {"donate_evals", h->donate_evals},
        {"donate_evals_drained", h->donate_evals_drained}, {"fuse_diff", h->fuse_mode}, {"autofit_slice", h->autofit_slice},
        {"host_copy_threads", h->host_copy_threads}, {"chain_overhead", h->chain_overhead}, {"host_tail", h->host_tail}};
    for (const auto &o : opts)
        if (!strcmp(name, o.n)) {
            *value = o.v;
            return ARIMA_OK;
        }
    return ARIMA_E_INVALID_ARG;
}

// ---------------------------------------------------------------------------------------------------------
// Ordering. A non-fit call waits (on the device, not the host) for every earlier call: the building blocks share
// the handle's workspaces, and any call may read an earlier call's outputs. A fit call waits for the earlier
// non-fit calls (e.g. the sampler that wrote its input), for the previous call on its own context and, with
// fit_pipeline > 1 (default 3), for any in-flight fit whose buffers its own overlap (order_after_overlapping_fits);
// with fit_pipeline = 1 the previous call on its context is the previous fit, so calls run in issue order.
static void begin_call(arima_handle *h, hipStream_t s) {
    if (h->has_done) hipStreamWaitEvent(s, h->ev_done, 0);
    for (auto &c : h->fctx)
        if (c.has_done) hipStreamWaitEvent(s, c.ev_done, 0);
}

static hipError_t end_call(arima_handle *h, hipStream_t s) {
    hipError_t e = hipEventRecord(h->ev_done, s);
    if (e == hipSuccess) h->has_done = true;
    return e;
}

static void begin_fit(arima_handle *h, FitCtx &c, hipStream_t s) {
    if (h->has_done) hipStreamWaitEvent(s, h->ev_done, 0);
    if (c.has_done) hipStreamWaitEvent(s, c.ev_done, 0);
}

// fit_pipeline > 1: consecutive fit calls run concurrently on different contexts, unless one reads what an in-flight
// call writes, writes what it reads, or writes the same memory -- then the new call waits for that call's end (so a
// caller may chain fits, e.g. one fit's coefficients as the next one's user inits, or reuse one output buffer,
// without synchronising: the same results as fit_pipeline 1)
static bool calls_meet(const CallSpans &x, const CallSpans &y) {
    for (int a = 0; a < 6; ++a) {
        for (int b = 0; b < 2; ++b)
            if (spans_meet(x.out[a], y.in[b])) return true;
        for (int b = 0; b < 6; ++b)
            if (spans_meet(x.out[a], y.out[b])) return true;
    }
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 6; ++b)
            if (spans_meet(x.in[a], y.out[b])) return true;
    return false;
}

// Returns the event to record at the new call's end (nullptr once its context tracks kInflightMax calls).
static hipEvent_t order_after_overlapping_fits(arima_handle *h, int ci, const CallSpans &cs, hipStream_t s) {
    for (int j = 0; j < kMaxPipeline; ++j) {
        FitCtx &o = h->fctx[j];
        if (!o.has_done || hipEventQuery(o.ev_done) == hipSuccess) {   // everything issued there has finished
            o.inflight.n = 0;
            o.inflight.overflow = false;
            continue;
        }
        if (j == ci) continue;                     // begin_fit already orders the call after its context's last one
        if (o.inflight.overflow) {
            hipStreamWaitEvent(s, o.ev_done, 0);
            continue;
        }
        for (int e = 0; e < o.inflight.n; ++e)
            if (calls_meet(cs, o.inflight.call[e])) hipStreamWaitEvent(s, o.inflight.ev[e], 0);
    }
    Inflight &f = h->fctx[ci].inflight;
    if (f.n == kInflightMax) {
        f.overflow = true;
        return nullptr;
    }
    if (!f.ev[f.n] && hipEventCreateWithFlags(&f.ev[f.n], hipEventDisableTiming) != hipSuccess) {
        f.overflow = true;
        return nullptr;
    }
    f.call[f.n] = cs;
    return f.ev[f.n++];
}

static CallSpans call_spans(const double *series, int64_t N, int32_t T, int64_t ld, int k, const double *uinit,
                            const double *coef, const double *ll, const int32_t *st, const int32_t *ne,
                            const int32_t *ng, const uint8_t *fl) {
    CallSpans cs;
    if (N <= 0) return cs;
    set_span(cs.in[0], series, ((N - 1) * ld + std::max<int64_t>(T, 0)) * (int64_t)sizeof(double));
    set_span(cs.in[1], uinit, N * k * (int64_t)sizeof(double));
    set_span(cs.out[0], coef, N * k * (int64_t)sizeof(double));
    set_span(cs.out[1], ll, N * (int64_t)sizeof(double));
    set_span(cs.out[2], st, N * (int64_t)sizeof(int32_t));
    set_span(cs.out[3], ne, N * (int64_t)sizeof(int32_t));
    set_span(cs.out[4], ng, N * (int64_t)sizeof(int32_t));
    set_span(cs.out[5], fl, N);
    return cs;
}

static hipError_t end_fit(FitCtx &c, hipStream_t s) {
    hipError_t e = hipEventRecord(c.ev_done, s);
    if (e == hipSuccess) c.has_done = true;
    return e;
}

// Hannan-Rissanen init (unless user init) and the fit kernel -- or the AR-only shortcut, or a uniform per-series
// status -- over already-differenced rows y (N x n, leading dimension ldn), on stream s with workspace ws.
// ev_mid (optional) is recorded between the init and the fit kernel. shared_gpu: other fits run concurrently (the
// order search's lanes), so the fit kernel's drained workgroups exit instead of joining its express pool.
// dd = 1: y holds the caller's RAW rows (leading dimension ldn) of a d = 1 fit, differenced inside every pass (fused
// differencing, arima_device.hpp stream_row); dd = 0: y holds differenced rows.
static int fit_kernels(arima_handle *h, FitWs &ws, const double *y, int64_t ldn, int n, int64_t N, int32_t p,
                       int32_t q, int32_t I, int32_t method, const double *d_user_init, double *d_coef, double *d_ll,
                       int32_t *d_status, int32_t *d_neval, int32_t *d_ngrad, uint8_t *d_flags, hipStream_t s,
                       hipEvent_t ev_mid, int64_t *grid_out, int64_t *express_out, bool shared_gpu = false,
                       int express_cus = -2, bool search = false, int dd = 0) {
    const int k = I + p + q;
    *grid_out = 0;
    *express_out = 0;
    // every workspace before the first launch (a growing DevBuf frees, and hipFree synchronises the device)
    RCCHK(h, ws.ctl.ensure(kCtlWords * sizeof(unsigned long long)), "workspace");
    RCCHK(h, ws.xring.ensure(sts::kExpressRingBytes), "workspace");
    RCCHK(h, ws.xready.ensure(sts::kExpressReadyBytes), "workspace");
    // the fit kernel's counters and express-ring ready words, initialised by the kernel that runs before it
    // (k_hr_init, or one k_fit_prep dispatch) instead of up to six fill dispatches (round 6)
    sts::FitPrep prep;
    prep.ctl = ws.ctl.as<unsigned long long>();
    prep.xready = ws.xready.as<unsigned>();
    prep.xready_words = sts::kExpressReadyBytes / 4;
    prep.v19 = (unsigned long long)std::max(h->express_ring, 0);
    prep.v44 = (unsigned long long)std::max(h->merge_live, 0);
    prep.v45 = (unsigned long long)std::max(h->donate_evals, 0);
    prep.v46 = (unsigned long long)std::max(h->donate_evals_drained, 0);
    prep.v47 = (unsigned long long)std::max(h->chain_overhead, 0);
    const bool cg = !(p > 0 && q == 0) && method == ARIMA_METHOD_CSS_CGD && k > 0;
    const bool gen = sts::gen_order(p, q);                     // above the compiled orders: arima_generic.hip
    if (!cg || gen) prep.xready_words = 0;                     // no express ring: only the counters are read
    if (p > 0 && q == 0) {                                     // AR-only shortcut, method never checked
        RCCHK(h, sts::launch_fit_prep(prep, s), "fit_prep");
        if (ev_mid) HIPCHK(h, hipEventRecord(ev_mid, s));
        if (gen)
            RCCHK(h, sts::launch_gen_ar_fit(y, ldn, n, N, p, I, d_coef, d_ll, d_status, d_neval, d_ngrad, d_flags, dd,
                                            s), "ar_fit");
        else
            RCCHK(h, sts::launch_ar_fit(y, ldn, n, N, p, I, d_coef, d_ll, d_status, d_neval, d_ngrad, d_flags, s, dd),
                  "ar_fit");
        return ARIMA_OK;
    }
    const double *init = d_user_init;
    const int32_t *init_status = nullptr;
    if (!d_user_init) {
        RCCHK(h, ws.init.ensure((size_t)N * std::max(k, 1) * sizeof(double)), "workspace");
        RCCHK(h, ws.hr_status.ensure((size_t)N * sizeof(int32_t)), "workspace");
        if (gen)
            RCCHK(h, sts::launch_gen_hr_init(y, ldn, n, N, p, q, I, ws.init.as<double>(), ws.hr_status.as<int32_t>(),
                                             dd, prep, s), "hr_init");
        else
            RCCHK(h, sts::launch_hr_init(y, ldn, n, N, p, q, I, ws.init.as<double>(), ws.hr_status.as<int32_t>(), s,
                                         h->hr_grid >= 0 ? h->hr_grid : (shared_gpu && !search ? 1024 : 0), dd, prep),
                  "hr_init");
        init = ws.init.as<double>();
        init_status = ws.hr_status.as<int32_t>();
    } else {
        RCCHK(h, sts::launch_fit_prep(prep, s), "fit_prep");
    }
    if (ev_mid) HIPCHK(h, hipEventRecord(ev_mid, s));
    if (method == ARIMA_METHOD_CSS_BOBYQA && k > 0) {           // fitWithCSSBOBYQA, ARIMA.scala:106, :130-160
        RCCHK(h, sts::launch_bobyqa_fit(y, ldn, n, N, p, q, I, init, init_status, nullptr, d_coef, d_ll, d_status,
                                        d_neval, d_ngrad, d_flags,
                                        h->bobyqa_wave < 0 ? N <= kBobyqaWaveMaxN : h->bobyqa_wave != 0, s),
              "bobyqa_fit");
        return ARIMA_OK;
    }
    if (method != ARIMA_METHOD_CSS_CGD || k == 0) {
        const unsigned grid = (unsigned)((N + 255) / 256);
        const int32_t code = (method != ARIMA_METHOD_CSS_CGD) ? ARIMA_ST_UNSUPPORTED_METHOD : ARIMA_ST_ZERO_PARAMS;
        hipLaunchKernelGGL(k_fill_status, dim3(grid), dim3(256), 0, s, N, k, init_status, code, d_coef, d_ll,
                           d_status, d_neval, d_ngrad, d_flags);
        HIPCHK(h, hipGetLastError());
        return ARIMA_OK;
    }
    if (gen) {                                                  // fitWithCSSCGD at runtime orders, a lane per series
        RCCHK(h, sts::launch_gen_fit(y, ldn, n, N, p, q, I, h->smear, init, init_status, d_coef, d_ll, d_status,
                                     d_neval, d_ngrad, d_flags, ws.ctl.as<unsigned long long>(), dd, s), "gen_fit");
        return ARIMA_OK;
    }
    // one persistent workgroup per CU (4 waves x the kernel's optimizer slots), the last num_cus/16 of them express
    // workgroups (k_cg_fit's long-series path); fewer bulk blocks when the batch cannot fill them
    // (express_blocks and grid_blocks count CUs' worth of workgroups: x kFitBlocksPerCU single-wave workgroups)
    const int cus = std::max(1, h->num_cus);
    // (express_cus: the caller's count, -2 = the "express_blocks" option; the order search passes its own)
    const int xopt = express_cus >= -1 ? express_cus : h->express_blocks;
    int xcus = xopt >= 0 ? xopt : std::max(1, cus / 16);
    if (xcus >= cus) xcus = cus - 1;
    int bcus = h->grid_blocks_override;
    if (bcus <= 0) bcus = std::max(1, cus - xcus);
    const int bpc = sts::kFitBlocksPerCU;
    int xblocks = xcus * bpc;
    int blocks = bcus * bpc;
    const int per_block = std::max(1, sts::cg_fit_series_per_block(p, q, I));
    const int64_t need = (N + per_block - 1) / per_block;
    if (blocks > need) blocks = (int)need;
    *grid_out = blocks;
    *express_out = xcus;                    // in CUs, the unit of the "express_blocks" option
    RCCHK(h, sts::launch_cg_fit(y, ldn, n, N, p, q, I, h->smear, init, init_status, d_coef, d_ll, d_status, d_neval,
                                d_ngrad, d_flags, ws.ctl.as<unsigned long long>(), blocks, xblocks,
                                ws.xring.as<unsigned char>(), ws.xready.as<unsigned>(), shared_gpu ? 0 : 1, s, dd),
          "cg_fit");
    hipLaunchKernelGGL(k_fault_merge, dim3(1), dim3(64), 0, s, ws.ctl.as<unsigned long long>(),
                       h->dev_fault.as<unsigned long long>());
    HIPCHK(h, hipGetLastError());
    return ARIMA_OK;
}

// Grow the workspaces of the first `count` contexts to an N x ldn batch with k parameters at once, so that no
// workspace grows (hipFree synchronises the device) while fits of other contexts are in flight.
static int reserve_fit_ws(arima_handle *h, int count, int64_t N, int64_t ldn, int k, bool diff_ws = true) {
    for (int j = 0; j < count; ++j) {
        FitCtx &c = h->fctx[j];
        if (diff_ws) RCCHK(h, c.diff.ensure((size_t)N * ldn * sizeof(double)), "workspace");
        RCCHK(h, c.ws.init.ensure((size_t)N * std::max(k, 1) * sizeof(double)), "workspace");
        RCCHK(h, c.ws.hr_status.ensure((size_t)N * sizeof(int32_t)), "workspace");
        RCCHK(h, c.ws.ctl.ensure(kCtlWords * sizeof(unsigned long long)), "workspace");
        RCCHK(h, c.ws.xring.ensure(sts::kExpressRingBytes), "workspace");
        RCCHK(h, c.ws.xready.ensure(sts::kExpressReadyBytes), "workspace");
    }
    return ARIMA_OK;
}

// One fit on context c, enqueued on stream s (the caller has ordered s after what the fit depends on).
// shared_gpu: fits of other contexts may run concurrently, so the fit kernel's drained workgroups exit (making room
// for the next fit) instead of joining its express pool.
// slot >= 0: one slice of a sliced call -- timing events and the counter copy go to that slice slot, and the
// context keeps no pending stats of its own.
static int fit_device_locked(arima_handle *h, FitCtx &c, int ci, int reserve, const double *d_series, int64_t N,
                             int32_t T, int64_t ld, int32_t p, int32_t d, int32_t q, int32_t I, int32_t method,
                             const double *d_user_init, double *d_coef, double *d_ll, int32_t *d_status,
                             int32_t *d_neval, int32_t *d_ngrad, uint8_t *d_flags, hipStream_t s, bool shared_gpu,
                             int slot = -1) {
    RCCHK(h, check_orders(h, p, d, q, I), "orders");
    if (N < 0 || T < 0 || ld < T) return set_err(h, ARIMA_E_INVALID_ARG, "bad shape");
    if (!d_coef || !d_ll || !d_status) return set_err(h, ARIMA_E_INVALID_ARG, "null output");
    HIPCHK(h, hipSetDevice(h->device));
    const int k = I + p + q;
    const int n = std::max(T - d, 0);
    c.pending = PendingStats{};
    if (slot < 0) {
        h->stats = arima_fit_stats{};
        h->stats_ctx = ci;
    }
    if (N == 0) return ARIMA_OK;
    // Fused differencing (round 6): css-cgd fits (and the AR-only shortcut) of d <= 1 read the caller's rows directly
    // -- d = 0 as they are, d = 1 differenced inside every pass (arima_device.hpp stream_row) -- instead of a
    // differenced copy written by k_difference (17 GB of HBM traffic per 1M x 1024 fit, a pipeline stage of its own,
    // and an N x T workspace per fit context). d >= 2 and css-bobyqa keep the copy.
    const bool fused = d <= 1 && (method == ARIMA_METHOD_CSS_CGD || (p > 0 && q == 0)) &&
                       (h->fuse_mode == 2 || (h->fuse_mode == 1 && sts::fuse_pays(p, q)));
    const int64_t ldn = fused ? ld : row_stride(h, n);
    const double *rows = fused ? d_series : nullptr;

    SliceSlot *ss = slot >= 0 ? &h->slot[slot] : nullptr;
    hipEvent_t *ev = ss ? ss->ev : c.ev;
    unsigned long long *ctl_dst = ss ? h->slot_ctl + (size_t)slot * kCtlWords : c.ctl_host;
    RCCHK(h, reserve_fit_ws(h, reserve, N, ldn, k, !fused), "workspace");
    HIPCHK(h, hipEventRecord(ev[0], s));
    if (!fused) {
        RCCHK(h, sts::launch_difference(d_series, ld, c.diff.as<double>(), ldn, N, T, d, 1, s), "difference");
        rows = c.diff.as<double>();
    }
    HIPCHK(h, hipEventRecord(ev[1], s));
    int64_t grid = 0, xblocks = 0;
    RCCHK(h, fit_kernels(h, c.ws, rows, ldn, n, N, p, q, I, method, d_user_init, d_coef, d_ll,
                         d_status, d_neval, d_ngrad, d_flags, s, ev[2], &grid, &xblocks, shared_gpu, -2, false,
                         fused ? d : 0), "fit");
    HIPCHK(h, hipEventRecord(ev[3], s));
    h->last_grid = grid;
    h->last_express = xblocks;
    HIPCHK(h, hipMemcpyAsync(ctl_dst, c.ws.ctl.ptr, kCtlWords * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    if (ss) HIPCHK(h, hipEventRecord(ss->ev[4], s));
    c.fit_ctl = !ss;
    PendingStats &ps = ss ? ss->ps : c.pending;
    ps.N = N;
    ps.n = n;
    ps.p = p;
    ps.q = q;
    ps.I = I;
    ps.ar_only = p > 0 && q == 0;
    ps.user_init = d_user_init != nullptr;
    ps.cg = !ps.ar_only && method == ARIMA_METHOD_CSS_CGD && k > 0;
    ps.grid = grid;
    ps.express = xblocks;
    ps.valid = true;
    return ARIMA_OK;
}

// The stats of one finished fit (or slice) from its pending shape, its counter copy and its timing events.
static arima_fit_stats compute_stats(const PendingStats &ps, const unsigned long long *cc, const hipEvent_t *ev) {
    arima_fit_stats st{};
    if (!ps.valid) return st;
    const int64_t N = ps.N;
    const int n = ps.n, p = ps.p, q = ps.q, I = ps.I, k = I + p + q;
    float ms = 0;
    hipEventElapsedTime(&ms, ev[0], ev[1]);
    st.ms_difference = ms;
    hipEventElapsedTime(&ms, ev[1], ev[2]);
    st.ms_hr_init = ms;
    hipEventElapsedTime(&ms, ev[2], ev[3]);
    st.ms_cg_fit = ms;
    hipEventElapsedTime(&ms, ev[0], ev[3]);
    st.ms_total = ms;
    st.f_passes = (int64_t)cc[1];
    st.g_passes = (int64_t)cc[2];
    st.n_eval = (int64_t)cc[5];
    st.n_grad = (int64_t)cc[6];
    st.wave_f_passes = (int64_t)cc[3];
    st.wave_g_passes = (int64_t)cc[4];
    st.spec_hits = (int64_t)cc[7];
    st.wave_multi_passes = (int64_t)cc[8];
    st.spec_chains = (int64_t)cc[9];
    st.ride_passes = (int64_t)cc[18];
    // series the kernels wrote; the AR-only shortcut, user-uniform statuses and an empty fit write every series
    st.series_done = ps.cg ? (int64_t)cc[32] : N;
    st.express_series = (int64_t)cc[23];
    st.express_f_passes = (int64_t)cc[24];
    st.express_g_passes = (int64_t)cc[25];
    st.express_pit_passes = (int64_t)cc[33];
    st.express_pit_sweeps = (int64_t)cc[34];
    st.express_pit_g_passes = (int64_t)cc[35];
    st.wave_chains = (int64_t)cc[36];
    st.low_util_passes = (int64_t)cc[37];
    st.diag_step_cycles = (int64_t)cc[38];
    st.diag_refill_cycles = (int64_t)cc[39];
    st.merge_series = (int64_t)cc[41];
    st.merge_waves = (int64_t)cc[42];
    st.express_blocks = ps.express;
    st.fault = (int64_t)cc[26];
    for (int i = 0; i < 5; ++i) st.fault_info[i] = (int64_t)cc[27 + i];
    // STS_TIMING builds: F-pass, G-pass, advance, select cycles (summed over waves), kernel span, drained time
    st.diag[0] = (int64_t)cc[10];
    st.diag[1] = (int64_t)cc[11];
    st.diag[2] = (int64_t)cc[12];
    st.diag[3] = (int64_t)cc[13];
    st.diag[4] = cc[14] ? (int64_t)(cc[14] - cc[15]) : 0;
    st.diag[5] = (int64_t)cc[16];
    st.grid_blocks = ps.grid;
    // HR passes: 2 per column of each of the two least squares, minus the norm pass of an intercept column (the
    // sum of ones needs no stream; arima_device.hpp ols_stage)
    const int M = std::max(p, q), m = M + 1;
    if (ps.ar_only) st.hr_passes = N * (int64_t)(2 * (I + p) - I);
    else if (!ps.user_init) st.hr_passes = N * (int64_t)(2 * (1 + m) - 1 + 2 * k - I);
    // algorithmic flops: U*S*(2(p+q)+4) + G*S*(2(p+q)+4 + 2kq + 1+p+q + 2k) + W_HR, with
    // U = distinct objective points evaluated by a pass (bulk objective passes, objective requests served by
    // gradient passes, express objective passes, and the speculative points the optimizer then used) and
    // G = gradient evaluations that ran a pass (bulk gradient passes without the objective riders, express ones)
    const double S = std::max(n - M, 0);
    const double ff = 2.0 * (p + q) + 4, fg = ff + 2.0 * k * q + 1 + p + q + 2.0 * k;
    const double whr = (double)N * (3.0 * std::max(n - m, 0) * (m + 1) * (m + 1) +
                                    3.0 * std::max(n - 2 * M - 1, 0) * k * k + 2.0 * std::max(n - m, 0) * m);
    const double U = (double)(st.f_passes + st.ride_passes + st.express_f_passes + st.spec_hits);
    const double G = (double)(st.g_passes - st.ride_passes + st.express_g_passes);
    st.flops = U * S * ff + G * S * fg + (ps.user_init ? 0.0 : whr);
    st.n_series = N;
    return st;
}

// Completes the stats of context c's last fit once its device work has finished.
static void finish_stats(arima_handle *h, FitCtx &c) {
    h->stats = compute_stats(c.pending, c.ctl_host, c.ev);
    c.pending.valid = false;
}

int arima_fit_batch_device(arima_handle *h, const double *d_series, int64_t n_series, int32_t T, int64_t ld,
                           int32_t p, int32_t d, int32_t q, int32_t include_intercept, int32_t method,
                           const double *d_user_init, double *d_coef_out, double *d_css_ll_out,
                           int32_t *d_status_out, int32_t *d_n_eval_out, int32_t *d_n_grad_out,
                           uint8_t *d_flags_out, void *stream) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    const int P = h->pipeline;
    HIPCHK(h, hipSetDevice(h->device));
    const int64_t ldn = row_stride(h, T - d);
    // Slice size: option fit_slice_bytes, or (0, the default) as large as the free HBM allows for P contexts. Every
    // slice ends with its own slowest series (the launch's critical path), so fewer, larger slices are faster (C4 at
    // 1M x 4096 in 262k-series slices: 2.9 s per fit alone, one slice: 1.2 s).
    int64_t slice_bytes = h->fit_slice_bytes;
    if (slice_bytes <= 0) {
        size_t free_b = 0, total_b = 0;
        HIPCHK(h, hipMemGetInfo(&free_b, &total_b));
        size_t held = 0;                           // the contexts' differenced workspaces are reused
        for (int j = 0; j < P; ++j) held += h->fctx[j].diff.bytes;
        slice_bytes = std::max<int64_t>(1ll << 30, (int64_t)((free_b + held) / 10 * 6 / (size_t)std::max(P, 1)));
    }
    int64_t slice = std::max<int64_t>(1024, slice_bytes / (ldn * (int64_t)sizeof(double)) / 1024 * 1024);
    if (n_series <= slice || T < 0 || ld < T || n_series < 0) {
        const int ci = (int)(h->fit_seq++ % (unsigned)P);
        FitCtx &c = h->fctx[ci];
        hipStream_t s = stream ? (hipStream_t)stream : c.stream;
        begin_fit(h, c, s);
        // hazards against in-flight fits of every context, whatever P is now: fits issued under a larger
        // fit_pipeline may still run on other contexts
        hipEvent_t ev_call = order_after_overlapping_fits(h, ci, call_spans(d_series, n_series, T, ld,
                                                                     include_intercept + p + q, d_user_init,
                                                                     d_coef_out, d_css_ll_out, d_status_out,
                                                                     d_n_eval_out, d_n_grad_out, d_flags_out), s);
        const int rc = fit_device_locked(h, c, ci, P, d_series, n_series, T, ld, p, d, q, include_intercept, method,
                                         d_user_init, d_coef_out, d_css_ll_out, d_status_out, d_n_eval_out,
                                         d_n_grad_out, d_flags_out, s, P > 1);
        HIPCHK(h, end_fit(c, s));
        if (ev_call) HIPCHK(h, hipEventRecord(ev_call, s));
        return rc;
    }
    // sliced: slice j of the batch runs on the next fit context (its own outputs' rows), exactly as consecutive calls
    RCCHK(h, check_orders(h, p, d, q, include_intercept), "orders");
    if (!d_coef_out || !d_css_ll_out || !d_status_out) return set_err(h, ARIMA_E_INVALID_ARG, "null output");
    const int k = include_intercept + p + q;
    const int64_t nslices = (n_series + slice - 1) / slice;
    h->stats = arima_fit_stats{};
    h->stats_ctx = -2;
    h->slice_first = h->slot_seq % kSliceSlots;
    h->slice_n = 0;
    h->slice_acc = arima_fit_stats{};
    for (int64_t j = 0; j < nslices; ++j) {
        const int sl = (int)(h->slot_seq++ % kSliceSlots);
        SliceSlot &ss = h->slot[sl];
        if (!ss.used) {
            for (auto &e : ss.ev) HIPCHK(h, hipEventCreate(&e));
            ss.used = true;
        } else if (hipEventQuery(ss.ev[4]) != hipSuccess) {
            HIPCHK(h, hipEventSynchronize(ss.ev[4]));       // its previous slice's counter copy must have landed
        }
        if (h->slice_n == (unsigned)kSliceSlots) {
            // more slices than slots: the oldest pending slice of THIS call is the one in slot sl; fold its stats
            // into the call's running total before the slot is overwritten
            acc_stats(h->slice_acc, compute_stats(ss.ps, h->slot_ctl + (size_t)sl * kCtlWords, ss.ev));
            h->slice_first = (h->slice_first + 1) % kSliceSlots;
            h->slice_n--;
        }
        ss.ps = PendingStats{};
        const int64_t f = j * slice, ns = std::min(slice, n_series - f);
        const int ci = (int)(h->fit_seq++ % (unsigned)P);             // the next context in the rotation
        FitCtx &c = h->fctx[ci];
        hipStream_t s = stream ? (hipStream_t)stream : c.stream;
        begin_fit(h, c, s);
        hipEvent_t ev_call = order_after_overlapping_fits(
                h, ci, call_spans(d_series + f * ld, ns, T, ld, k, d_user_init ? d_user_init + f * k : nullptr,
                                  d_coef_out + f * k, d_css_ll_out + f, d_status_out + f,
                                  d_n_eval_out ? d_n_eval_out + f : nullptr, d_n_grad_out ? d_n_grad_out + f : nullptr,
                                  d_flags_out ? d_flags_out + f : nullptr), s);
        const int rc = fit_device_locked(
            h, c, ci, P, d_series + f * ld, ns, T, ld, p, d, q, include_intercept, method,
            d_user_init ? d_user_init + f * k : nullptr, d_coef_out + f * k, d_css_ll_out + f, d_status_out + f,
            d_n_eval_out ? d_n_eval_out + f : nullptr, d_n_grad_out ? d_n_grad_out + f : nullptr,
            d_flags_out ? d_flags_out + f : nullptr, s, P > 1, sl);
        HIPCHK(h, end_fit(c, s));
        if (ev_call) HIPCHK(h, hipEventRecord(ev_call, s));
        h->slice_n++;
        if (rc != ARIMA_OK) return rc;
    }
    return ARIMA_OK;
}

// ---------------------------------------------------------------------------------------------------------
// Host path (end to end from host memory). The batch is cut into chunks of h->host_chunk
// series that rotate over h->host_pipeline contexts: chunk j's upload (from the caller's pageable buffer, staged by
// the HIP runtime) runs while the fits of chunks j-1, j-2 are still on the device, so PCIe and compute overlap and
// the tail of one chunk's fit kernel overlaps the next chunk's work. Results come back through pinned staging and
// are copied to the caller's arrays when the context is reused (or at the end).
// ---------------------------------------------------------------------------------------------------------
namespace {
struct HostOut {
    double *coef, *ll;
    int32_t *status, *n_eval, *n_grad;
    uint8_t *flags;
};

// bytes of one chunk's results in pinned staging: coef (n*k), ll, status, n_eval, n_grad, flags
inline size_t pin_layout(int64_t n, int k, size_t off[6]) {
    size_t o = 0;
    off[0] = o; o += round_up((int64_t)n * std::max(k, 1) * 8, 256);
    off[1] = o; o += round_up(n * 8, 256);
    off[2] = o; o += round_up(n * 4, 256);
    off[3] = o; o += round_up(n * 4, 256);
    off[4] = o; o += round_up(n * 4, 256);
    off[5] = o; o += round_up(n, 256);
    return o;
}
}  // namespace

static void acc_stats(arima_fit_stats &a, const arima_fit_stats &s) {
    a.ms_difference += s.ms_difference;
    a.ms_hr_init += s.ms_hr_init;
    a.ms_cg_fit += s.ms_cg_fit;
    a.ms_total += s.ms_total;
    a.f_passes += s.f_passes;
    a.g_passes += s.g_passes;
    a.hr_passes += s.hr_passes;
    a.n_eval += s.n_eval;
    a.n_grad += s.n_grad;
    a.flops += s.flops;
    a.n_series += s.n_series;
    a.wave_f_passes += s.wave_f_passes;
    a.wave_g_passes += s.wave_g_passes;
    a.wave_multi_passes += s.wave_multi_passes;
    a.spec_hits += s.spec_hits;
    a.spec_chains += s.spec_chains;
    a.ride_passes += s.ride_passes;
    a.series_done += s.series_done;
    a.express_series += s.express_series;
    a.express_f_passes += s.express_f_passes;
    a.express_g_passes += s.express_g_passes;
    a.express_pit_passes += s.express_pit_passes;
    a.express_pit_sweeps += s.express_pit_sweeps;
    a.express_pit_g_passes += s.express_pit_g_passes;
    a.wave_chains += s.wave_chains;
    a.low_util_passes += s.low_util_passes;
    a.merge_series += s.merge_series;
    a.merge_waves += s.merge_waves;
    a.grid_blocks = s.grid_blocks;
    a.express_blocks = s.express_blocks;
    if (!a.fault && s.fault) {
        a.fault = s.fault;
        for (int i = 0; i < 5; ++i) a.fault_info[i] = s.fault_info[i];
    }
}

// memcpy with `threads` host threads (the caller's pageable rows into a pinned block: one thread copies at a fraction
// of the host's memory bandwidth, a PCIe Gen5 x16 link needs several)
static void par_memcpy(void *dst, const void *src, size_t bytes, int threads) {
    const size_t min_part = size_t(4) << 20;
    const int t = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(threads, 1), bytes / min_part));
    if (t <= 1) {
        memcpy(dst, src, bytes);
        return;
    }
    std::vector<std::thread> pool;
    const size_t part = (bytes + t - 1) / t / 64 * 64 + 64;
    for (int i = 0; i < t; ++i) {
        const size_t off = (size_t)i * part;
        if (off >= bytes) break;
        const size_t len = std::min(part, bytes - off);
        pool.emplace_back([=] { memcpy((char *)dst + off, (const char *)src + off, len); });
    }
    for (auto &th : pool) th.join();
}

// Host rows -> device on stream s through the handle's ring of pinned blocks: block i is filled by the copy threads
// while block i-1's DMA runs; a block is refilled only after its previous DMA has finished (its event). The caller's
// buffer is fully read when this returns (as a pageable hipMemcpyAsync's is).
static int upload_staged(arima_handle *h, void *dst, const void *src, size_t bytes, hipStream_t s) {
    if (bytes == 0) return ARIMA_OK;
    if (h->host_copy_threads <= 0) {
        HIPCHK(h, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
        return ARIMA_OK;
    }
    for (size_t off = 0; off < bytes;) {
        const int j = (int)(h->stage_next++ % arima_handle::kStageSlots);
        if (!h->stage[j]) {
            if (hipHostMalloc(&h->stage[j], arima_handle::kStageBytes, 0) != hipSuccess)
                return set_err(h, ARIMA_E_OOM, "pinned staging");
            HIPCHK(h, hipEventCreateWithFlags(&h->stage_ev[j], hipEventDisableTiming));
        } else if (h->stage_used[j]) {
            HIPCHK(h, hipEventSynchronize(h->stage_ev[j]));
        }
        const size_t len = std::min(arima_handle::kStageBytes, bytes - off);
        par_memcpy(h->stage[j], (const char *)src + off, len, h->host_copy_threads);
        HIPCHK(h, hipMemcpyAsync((char *)dst + off, h->stage[j], len, hipMemcpyHostToDevice, s));
        HIPCHK(h, hipEventRecord(h->stage_ev[j], s));
        h->stage_used[j] = true;
        off += len;
    }
    return ARIMA_OK;
}

// Wait for context c's chunk, copy its results to the caller's arrays and add its counters to h->host_acc.
static int drain_chunk(arima_handle *h, FitCtx &c, int k, const HostOut &o) {
    if (c.chunk_n <= 0) return ARIMA_OK;
    HIPCHK(h, hipEventSynchronize(c.ev_done));
    const int64_t f = c.chunk_first, n = c.chunk_n;
    c.chunk_n = 0;
    if (c.pending.valid) finish_stats(h, c);
    acc_stats(h->host_acc, h->stats);
    RCCHK(h, check_fault(h, c), "fault");
    size_t off[6];
    pin_layout(n, k, off);
    const char *b = static_cast<const char *>(c.pin);
    if (k > 0) memcpy(o.coef + f * k, b + off[0], (size_t)n * k * 8);
    memcpy(o.ll + f, b + off[1], (size_t)n * 8);
    memcpy(o.status + f, b + off[2], (size_t)n * 4);
    if (o.n_eval) memcpy(o.n_eval + f, b + off[3], (size_t)n * 4);
    if (o.n_grad) memcpy(o.n_grad + f, b + off[4], (size_t)n * 4);
    if (o.flags) memcpy(o.flags + f, b + off[5], (size_t)n);
    return ARIMA_OK;
}

int arima_fit_batch(arima_handle *h, const double *series, int64_t N, int32_t T, int32_t p, int32_t d, int32_t q,
                    int32_t I, int32_t method, const double *user_init, double *coef_out, double *css_ll_out,
                    int32_t *status_out, int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    RCCHK(h, check_orders(h, p, d, q, I), "orders");
    if (N < 0 || T < 0 || (N > 0 && (!series || !coef_out || !css_ll_out || !status_out)))
        return set_err(h, ARIMA_E_INVALID_ARG, "bad arguments");
    h->stats = arima_fit_stats{};
    h->stats_ctx = -1;
    if (N == 0) return ARIMA_OK;
    HIPCHK(h, hipSetDevice(h->device));
    const int k = I + p + q;
    const int P = h->host_pipeline;
    const int64_t chunk = std::min<int64_t>(h->host_chunk, N);
    // Chunk boundaries: full chunks, then the last two chunks' worth halved again and again (down to 16 384 series).
    // The call ends with the fit of its last chunk, whose duration is that chunk's slowest series: a small last chunk
    // exposes less of it after the final upload (C2 1M x 1024 on 8 queues: profiles/r06/g_e2e, h_e2e)
    std::vector<int64_t> starts;
    for (int64_t f = 0; f < N;) {
        starts.push_back(f);
        const int64_t rem = N - f;
        int64_t n = std::min(chunk, rem);
        if (h->host_tail && rem <= 2 * chunk && rem > arima_handle::kHostTailMin) n = std::max<int64_t>(arima_handle::kHostTailMin, (rem + 1) / 2);
        f += n;
    }
    starts.push_back(N);
    const int64_t nchunks = (int64_t)starts.size() - 1;
    const int used = (int)std::min<int64_t>(P, nchunks);
    const HostOut o{coef_out, css_ll_out, status_out, n_eval_out, n_grad_out, flags_out};
    h->host_acc = arima_fit_stats{};
    // every context the call uses: settle what an earlier call left in it, then size its buffers for a full chunk
    for (int j = 0; j < used; ++j) {
        FitCtx &c = h->fctx[j];
        if (c.has_done) HIPCHK(h, hipEventSynchronize(c.ev_done));
        c.chunk_n = 0;
        RCCHK(h, c.d_series.ensure((size_t)chunk * std::max(T, 1) * sizeof(double)), "staging");
        RCCHK(h, c.d_coef.ensure((size_t)chunk * std::max(k, 1) * sizeof(double)), "staging");
        RCCHK(h, c.d_ll.ensure((size_t)chunk * sizeof(double)), "staging");
        RCCHK(h, c.d_status.ensure((size_t)chunk * sizeof(int32_t)), "staging");
        RCCHK(h, c.d_neval.ensure((size_t)chunk * sizeof(int32_t)), "staging");
        RCCHK(h, c.d_ngrad.ensure((size_t)chunk * sizeof(int32_t)), "staging");
        RCCHK(h, c.d_flags.ensure((size_t)chunk), "staging");
        if (user_init) RCCHK(h, c.d_uinit.ensure((size_t)chunk * std::max(k, 1) * sizeof(double)), "staging");
        size_t off[6];
        const size_t need = pin_layout(chunk, k, off);
        if (c.pin_bytes < need) {
            if (c.pin) hipHostFree(c.pin);
            c.pin = nullptr;
            c.pin_bytes = 0;
            if (hipHostMalloc(&c.pin, need, 0) != hipSuccess) return set_err(h, ARIMA_E_OOM, "pinned staging");
            c.pin_bytes = need;
        }
    }
    int rc = ARIMA_OK;
    for (int64_t j = 0; j < nchunks && rc == ARIMA_OK; ++j) {
        const int ci = (int)(j % P);
        FitCtx &c = h->fctx[ci];
        rc = drain_chunk(h, c, k, o);                       // chunk j - P
        if (rc != ARIMA_OK) break;
        const int64_t first = starts[j], n = starts[j + 1] - starts[j];
        hipStream_t s = c.stream;
        begin_fit(h, c, s);
        if (T > 0) RCCHK(h, upload_staged(h, c.d_series.ptr, series + first * T, (size_t)n * T * sizeof(double), s),
                         "upload");
        const double *d_ui = nullptr;
        if (user_init) {
            if (k > 0)
                HIPCHK(h, hipMemcpyAsync(c.d_uinit.ptr, user_init + first * k, (size_t)n * k * sizeof(double),
                                         hipMemcpyHostToDevice, s));
            d_ui = c.d_uinit.as<double>();
        }
        rc = fit_device_locked(h, c, ci, used, c.d_series.as<double>(), n, T, T, p, d, q, I, method, d_ui,
                               c.d_coef.as<double>(), c.d_ll.as<double>(), c.d_status.as<int32_t>(),
                               c.d_neval.as<int32_t>(), c.d_ngrad.as<int32_t>(), c.d_flags.as<uint8_t>(), s,
                               nchunks > 1);
        if (rc == ARIMA_OK) {
            size_t off[6];
            pin_layout(n, k, off);
            char *b = static_cast<char *>(c.pin);
            if (k > 0) HIPCHK(h, hipMemcpyAsync(b + off[0], c.d_coef.ptr, (size_t)n * k * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(h, hipMemcpyAsync(b + off[1], c.d_ll.ptr, (size_t)n * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(h, hipMemcpyAsync(b + off[2], c.d_status.ptr, (size_t)n * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(h, hipMemcpyAsync(b + off[3], c.d_neval.ptr, (size_t)n * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(h, hipMemcpyAsync(b + off[4], c.d_ngrad.ptr, (size_t)n * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(h, hipMemcpyAsync(b + off[5], c.d_flags.ptr, (size_t)n, hipMemcpyDeviceToHost, s));
            c.chunk_first = first;
            c.chunk_n = n;
        }
        HIPCHK(h, end_fit(c, s));
    }
    for (int j = 0; j < used; ++j) {                        // the last chunks (every context, even after an error)
        const int r = drain_chunk(h, h->fctx[j], k, o);
        if (rc == ARIMA_OK) rc = r;
    }
    h->stats = h->host_acc;
    h->stats_ctx = -1;
    const int rf = take_fault(h);          // already reported per chunk when set: clear the sticky record
    return rc != ARIMA_OK ? rc : rf;
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
    const int64_t ld = row_stride(h, n);
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
    const int64_t ldn = row_stride(h, n);
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
                                 h->h_status.as<int32_t>(), s, std::max(h->hr_grid, 0)), "hr_init");
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

// ARIMAModel.forecast over a device batch: k_forecast (p, q <= 5, d <= 8, the streaming kernel) or the runtime-order
// k_gen_forecast for every other order, in slices whose per-series arrays fit a bounded workspace (h->fc_ws)
static int forecast_any(arima_handle *h, const double *ts, int64_t ld, const double *coef, int k, double *out,
                        int64_t ld_out, int64_t N, int T, int p, int d, int q, int I, int n_future, hipStream_t s) {
    if (!sts::gen_order(p, q) && d <= 8)
        return sts::launch_forecast(ts, ld, coef, k, out, ld_out, N, T, p, d, q, I, n_future, s);
    const int64_t w = sts::gen_forecast_ws_doubles(T, p, d, q, n_future);
    const int64_t chunk = std::max<int64_t>(64, std::min<int64_t>(N, (int64_t(1) << 27) / std::max<int64_t>(w, 1)));
    RCCHK(h, h->fc_ws.ensure((size_t)std::min(chunk, N) * w * sizeof(double)), "forecast workspace");
    for (int64_t f = 0; f < N; f += chunk) {
        const int64_t n = std::min(chunk, N - f);
        RCCHK(h, sts::launch_gen_forecast(ts + f * ld, ld, coef + f * k, k, out + f * ld_out, ld_out, n, T, p, d, q, I,
                                          n_future, h->fc_ws.as<double>(), w, s), "forecast");
    }
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
    RCCHK(h, forecast_any(h, h->h_series.as<double>(), T, h->h_coef.as<double>(), k, h->h_aux.as<double>(), L, N,
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
    RCCHK(h, forecast_any(h, d_series, ld, d_coef, I + p + q, d_out, ld_out, N, T, p, d, q, I, n_future, s),
          "forecast");
    HIPCHK(h, end_call(h, s));
    return ARIMA_OK;
}

// ---------------------------------------------------------------------------------------------------------
// order search over (d, p, q, intercept) — SURVEY.md 8(f) row 2 (config C5)
// ---------------------------------------------------------------------------------------------------------
// stream s waits for everything the first L search lanes have been given so far
static void join_lanes_into(arima_handle *h, hipStream_t s, int L) {
    for (int j = 0; j < L; ++j) {
        SearchLane &ln = h->lanes[j];
        if (!ln.stream) continue;
        if (hipEventRecord(ln.ev_fit, ln.stream) == hipSuccess) hipStreamWaitEvent(s, ln.ev_fit, 0);
    }
}

static int order_search_locked(arima_handle *h, const double *d_series, int64_t N, int32_t T, int64_t ld,
                               int32_t max_p, int32_t max_d, int32_t max_q, int32_t intercept_mode, int32_t method,
                               int32_t *d_order, double *d_coef, double *d_aic, int64_t *n_fits, hipStream_t s) {
    if (max_p < 0 || max_q < 0 || max_d < 0 || intercept_mode < 0 || intercept_mode > 2)
        return set_err(h, ARIMA_E_INVALID_ARG, "bad search bounds");
    if (max_p > 5 || max_q > 5 || max_d > kMaxD) return set_err(h, ARIMA_E_UNSUPPORTED, "p, q <= 5, d <= 16");
    if (N < 0 || T < 0 || ld < T || !d_order || !d_coef || !d_aic) return set_err(h, ARIMA_E_INVALID_ARG, "bad shape");
    h->stats_ctx = -1;
    h->stats = arima_fit_stats{};
    if (N == 0) return ARIMA_OK;
    HIPCHK(h, hipSetDevice(h->device));
    // Differenced copies: one per d, all computed up front, so the lanes run through the d boundaries without
    // draining -- when they fit in HBM next to the lanes' workspaces; otherwise one shared copy, rewritten for each
    // d once every fit of the previous d has finished (max_d up to 16 would not fit).
    size_t diff_bytes = 0;
    for (int d = 0; d <= max_d; ++d) diff_bytes += (size_t)N * row_stride(h, T - d) * sizeof(double);
    const size_t lane_bytes = (size_t)N * (11 * 8 * 2 + 8 + 4 * 4 + 1 + 8 + 16 + 88) + sts::kExpressRingBytes +
                              sts::kExpressReadyBytes;
    size_t free_b = 0, total_b = 0;
    HIPCHK(h, hipMemGetInfo(&free_b, &total_b));
    size_t held = 0;                               // what this handle's search workspaces already hold
    for (int d = 0; d <= kMaxD; ++d) held += h->os_diff[d].bytes;
    const bool per_d = diff_bytes + (size_t)h->search_lanes * lane_bytes <= (free_b + held) / 10 * 9;
    // Lanes: as many of the configured as their workspaces allow (at least one)
    int L = 0;
    for (int j = 0; j < h->search_lanes; ++j) {
        SearchLane &ln = h->lanes[j];
        if (!ln.stream) {
            HIPCHK(h, hipStreamCreateWithFlags(&ln.stream, hipStreamNonBlocking));
            HIPCHK(h, hipEventCreateWithFlags(&ln.ev_fit, hipEventDisableTiming));
            HIPCHK(h, hipEventCreateWithFlags(&ln.ev_sel, hipEventDisableTiming));
        }
        // every workspace at its largest size before anything is enqueued: a growing DevBuf frees (hipFree
        // synchronises the device) and would serialise the host loop below with the fits already in flight
        int rc = ARIMA_OK;
        for (DevBuf *b : {&ln.coef, &ln.ws.init})
            if (rc == ARIMA_OK) rc = b->ensure((size_t)N * 11 * sizeof(double));
        if (rc == ARIMA_OK) rc = ln.ll.ensure((size_t)N * sizeof(double));
        for (DevBuf *b : {&ln.status, &ln.neval, &ln.ngrad, &ln.ws.hr_status})
            if (rc == ARIMA_OK) rc = b->ensure((size_t)N * sizeof(int32_t));
        if (rc == ARIMA_OK) rc = ln.flags.ensure((size_t)N);
        if (rc == ARIMA_OK) rc = ln.best_aic.ensure((size_t)N * sizeof(double));
        if (rc == ARIMA_OK) rc = ln.best_order.ensure((size_t)N * 4 * sizeof(int32_t));
        if (rc == ARIMA_OK) rc = ln.best_coef.ensure((size_t)N * 11 * sizeof(double));
        if (rc == ARIMA_OK) rc = ln.ws.ctl.ensure(kCtlWords * sizeof(unsigned long long));
        if (rc == ARIMA_OK) rc = ln.acc.ensure((kCtlWords + 1) * sizeof(unsigned long long));
        if (rc == ARIMA_OK) rc = ln.ws.xring.ensure(sts::kExpressRingBytes);
        if (rc == ARIMA_OK) rc = ln.ws.xready.ensure(sts::kExpressReadyBytes);
        if (rc != ARIMA_OK) {
            if (j == 0) return set_err(h, rc, "order search workspace");
            break;                                 // fewer lanes instead of failing the call
        }
        L = j + 1;
    }
    if (per_d) {
        for (int d = 0; d <= max_d; ++d)
            RCCHK(h, h->os_diff[d].ensure((size_t)N * row_stride(h, T - d) * sizeof(double)), "workspace");
    } else {
        RCCHK(h, h->os_diff[0].ensure((size_t)N * row_stride(h, T) * sizeof(double)), "workspace");
    }
    HIPCHK(h, hipEventRecord(h->ev[0], s));
    auto diff_into = [&](int d, DevBuf &buf) -> int {
        const int n = std::max(T - d, 0);
        const int64_t ldn = row_stride(h, n);
        if (!h->ev_diff[d]) HIPCHK(h, hipEventCreateWithFlags(&h->ev_diff[d], hipEventDisableTiming));
        RCCHK(h, sts::launch_difference(d_series, ld, buf.as<double>(), ldn, N, T, d, 1, s), "difference");
        HIPCHK(h, hipEventRecord(h->ev_diff[d], s));
        return ARIMA_OK;
    };
    if (per_d)                                     // differencesOfOrderD once per d (ARIMA.scala:88)
        for (int d = 0; d <= max_d; ++d) RCCHK(h, diff_into(d, h->os_diff[d]), "difference");
    // Every lane keeps its own best candidate per series, and candidates compare by (approxAIC, grid position), so
    // the result does not depend on the order the grid points finish in: each lane runs its grid points back to back
    // without waiting for the others (a lane's long fit no longer holds the other lanes' next fits). With one
    // differenced copy per d the grid points go to the lanes by estimated cost, longest first (LPT); with the shared
    // copy they keep the (d, p, q, intercept) order and the lanes join before the copy is rewritten.
    for (int j = 0; j < L; ++j) {
        SearchLane &ln = h->lanes[j];
        HIPCHK(h, hipStreamWaitEvent(ln.stream, h->ev[0], 0));
        RCCHK(h, sts::launch_search_init(ln.best_aic.as<double>(), ln.best_order.as<int32_t>(),
                                         ln.best_coef.as<double>(), N, ln.stream), "search_init");
        HIPCHK(h, hipMemsetAsync(ln.acc.ptr, 0, (kCtlWords + 1) * sizeof(unsigned long long), ln.stream));
    }
    const int i_lo = intercept_mode == 1 ? 1 : 0, i_hi = intercept_mode == 0 ? 0 : 1;
    struct GridPoint { int d, p, q, I; double cost; };
    std::vector<GridPoint> grid;
    for (int d = 0; d <= max_d; ++d)
        for (int p = 0; p <= max_p; ++p)
            for (int q = 0; q <= max_q; ++q)
                for (int I = i_lo; I <= i_hi; ++I)
                    // ms per 65 536 series in profiles/r03/b_c3_c5/grid_65536.jsonl follow (1+p)(1+q) (corr. 0.8);
                    // AR-only fits (q = 0) are a single OLS
                    grid.push_back({d, p, q, I, q == 0 ? 0.1 : (double)(1 + p) * (1 + q)});
    std::vector<std::vector<int>> plan(L);
    if (per_d) {
        std::vector<int> idx(grid.size());
        for (size_t g = 0; g < grid.size(); ++g) idx[g] = (int)g;
        std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return grid[a].cost > grid[b].cost; });
        std::vector<double> load(L, 0.0);
        for (int g : idx) {
            const int j = (int)(std::min_element(load.begin(), load.end()) - load.begin());
            plan[j].push_back(g);
            load[j] += grid[g].cost;
        }
    } else {
        for (size_t g = 0; g < grid.size(); ++g) plan[g % L].push_back((int)g);
    }
    int64_t fits = 0;
    // the shared differenced copy: the fits of one d at a time (plan order is d-major on every lane)
    for (int dd = 0; dd <= (per_d ? 0 : max_d); ++dd) {
        if (!per_d) {
            if (dd > 0) join_lanes_into(h, s, L);   // every fit of d - 1 has read the copy
            RCCHK(h, diff_into(dd, h->os_diff[0]), "difference");
        }
        for (int j = 0; j < L; ++j) {
            SearchLane &ln = h->lanes[j];
            for (int g : plan[j]) {
                const GridPoint &gp = grid[g];
                if (!per_d && gp.d != dd) continue;
                const int d = gp.d, p = gp.p, q = gp.q, I = gp.I;
                const int n = std::max(T - d, 0);
                const int64_t ldn = row_stride(h, n);
                DevBuf &dbuf = per_d ? h->os_diff[d] : h->os_diff[0];
                HIPCHK(h, hipStreamWaitEvent(ln.stream, h->ev_diff[d], 0));
                // ARIMA(0,d,0) without intercept has no parameters: the reference throws (NoDataException);
                // fit_kernels reports it per series and the select step skips it.
                int64_t gridb = 0, xb = 0;
                RCCHK(h, fit_kernels(h, ln.ws, dbuf.as<double>(), ldn, n, N, p, q, I, method, nullptr,
                                     ln.coef.as<double>(), ln.ll.as<double>(), ln.status.as<int32_t>(),
                                     ln.neval.as<int32_t>(), ln.ngrad.as<int32_t>(), ln.flags.as<uint8_t>(), ln.stream,
                                     nullptr, &gridb, &xb, L > 1, L > 1 ? h->search_express_blocks : -2, true), "fit");
                if (gridb > 0) {
                    h->last_grid = gridb;
                    h->last_express = xb;
                }
                hipLaunchKernelGGL(k_search_acc, dim3(1), dim3(64), 0, ln.stream, ln.ws.ctl.as<unsigned long long>(),
                                   ln.acc.as<unsigned long long>(), N, n, p, q, I,
                                   (p > 0 && q == 0) || method != ARIMA_METHOD_CSS_CGD || I + p + q == 0 ? 0 : 1);
                HIPCHK(h, hipGetLastError());
                // a fit whose kernel recorded a watchdog fault contributes nothing (its outputs are incomplete) and
                // the fault reaches the caller through the handle's sticky record (arima_synchronize)
                RCCHK(h, sts::launch_search_select(ln.coef.as<double>(), ln.ll.as<double>(), ln.status.as<int32_t>(),
                                                   ln.flags.as<uint8_t>(), N, p, d, q, I,
                                                   ln.ws.ctl.as<unsigned long long>(), ln.best_aic.as<double>(),
                                                   ln.best_order.as<int32_t>(), ln.best_coef.as<double>(),
                                                   ln.stream),
                      "search_select");
                ++fits;
            }
        }
    }
    join_lanes_into(h, s, L);
    sts::SearchBests bests{};
    for (int j = 0; j < L; ++j) {
        bests.aic[j] = h->lanes[j].best_aic.as<double>();
        bests.order[j] = h->lanes[j].best_order.as<int32_t>();
        bests.coef[j] = h->lanes[j].best_coef.as<double>();
    }
    RCCHK(h, sts::launch_search_merge(bests, L, N, d_aic, d_order, d_coef, s), "search_merge");
    HIPCHK(h, hipEventRecord(h->ev[3], s));
    for (int j = 0; j < L; ++j)                    // the lanes' counter sums, read by arima_get_last_stats
        HIPCHK(h, hipMemcpyAsync(h->search_acc_host + (size_t)j * (kCtlWords + 1), h->lanes[j].acc.ptr,
                                 (kCtlWords + 1) * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipEventRecord(h->ev[4], s));
    h->stats_ctx = -3;
    h->search_lanes_used = L;
    h->search_n = N;
    h->search_fits = fits;
    if (n_fits) *n_fits = fits;
    return ARIMA_OK;
}

// The call's stream waits for everything its lanes have been given (also after an error part-way through the grid,
// ADVICE r2): later calls then wait for the lanes' reads of the search workspaces through h->ev_done.
static void join_lanes(arima_handle *h, hipStream_t s) {
    for (auto &ln : h->lanes) {
        if (!ln.stream) continue;
        if (hipEventRecord(ln.ev_fit, ln.stream) == hipSuccess) hipStreamWaitEvent(s, ln.ev_fit, 0);
    }
}

// Blocking entry points: the fault record covers the lanes' fit kernels (a dropped series must not
// pass as a candidate, and the call reports ARIMA_E_DEVICE).
static int take_fault(arima_handle *h) {
    unsigned long long f[6] = {};
    unsigned long long *rec = h->dev_fault.as<unsigned long long>();
    hipLaunchKernelGGL(k_fault_take, dim3(1), dim3(64), 0, h->stream, rec);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipMemcpyAsync(f, rec + 8, sizeof f, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (f[0] == 0) return ARIMA_OK;
    char msg[160];
    snprintf(msg, sizeof msg, "fit kernel watchdog fault %llu (info %llu %llu %llu %llu %llu)", f[0], f[1], f[2],
             f[3], f[4], f[5]);
    return set_err(h, ARIMA_E_DEVICE, msg);
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
    join_lanes(h, s);
    HIPCHK(h, end_call(h, s));
    return rc;
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
    join_lanes(h, s);
    if (rc == ARIMA_OK) {
        HIPCHK(h, hipMemcpyAsync(order_out, h->os_order.ptr, (size_t)N * 4 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipMemcpyAsync(coef_out, h->h_aux.ptr, (size_t)N * 11 * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipMemcpyAsync(aic_out, h->h_ll.ptr, (size_t)N * sizeof(double), hipMemcpyDeviceToHost, s));
    }
    HIPCHK(h, end_call(h, s));
    HIPCHK(h, hipStreamSynchronize(s));
    if (rc != ARIMA_OK) return rc;
    return take_fault(h);
}

// ---------------------------------------------------------------------------------------------------------
// ARIMA.autoFit over a batch (ARIMA.scala:280-375; arima_autofit.hip has the kernels and the quirks they restate)
// ---------------------------------------------------------------------------------------------------------
// Host loop: (1) the KPSS search over d = 0..max_d (rows of undecided series differenced at d into af_rows, then the
// test; decided rows keep their d); (2) rounds of the stepwise walk: k_af_plan appends every walking series'
// candidates to per-(p, q, intercept) lists, the host reads the list sizes (one small copy per round), and every
// non-empty list is gathered and fitted as one batch (fit_kernels: AR-only OLS or HR init + k_cg_fit) on the fit
// contexts' streams, several orders at once; k_af_update then picks each series' new incumbent and neighbourhood.
// The walk ends when no series has candidates left (at most max_p + 2 rounds after the first).
constexpr int kAfContexts = 4;                     // fit contexts the orders of one round rotate over

// One slice of the batch (every workspace sized for N series of length T). max_p <= sts::kAfMaxP.
static int autofit_slice(arima_handle *h, const double *d_series, int64_t N, int32_t T, int64_t ld, int32_t max_p,
                         int32_t max_d, int32_t max_q, int32_t *d_order, double *d_coef, double *d_aic,
                         int32_t *d_status, int32_t *d_nfits, hipStream_t s, int64_t *fits_out) {
    const int ncombos = sts::af_combos(max_p);
    const int64_t ldT = row_stride(h, T);
    const int64_t rows_max = N * sts::kAfMaxCand;  // candidate fits of one round, at most
    RCCHK(h, h->af_rows.ensure((size_t)N * ldT * sizeof(double)), "autofit workspace");
    RCCHK(h, h->af_dsel.ensure((size_t)N * sizeof(int32_t)), "autofit workspace");
    RCCHK(h, h->af_state.ensure((size_t)N * sizeof(sts::AfSeries)), "autofit workspace");
    RCCHK(h, h->af_best.ensure((size_t)N * 11 * sizeof(double)), "autofit workspace");
    RCCHK(h, h->af_counts.ensure(sts::kAfCombosMax * sizeof(unsigned)), "autofit workspace");
    RCCHK(h, h->af_off.ensure(sts::kAfCombosMax * sizeof(int64_t)), "autofit workspace");
    RCCHK(h, h->af_lists.ensure((size_t)ncombos * N * sizeof(int32_t)), "autofit workspace");
    RCCHK(h, h->af_coef.ensure((size_t)rows_max * 11 * sizeof(double)), "autofit workspace");
    RCCHK(h, h->af_ll.ensure((size_t)rows_max * sizeof(double)), "autofit workspace");
    RCCHK(h, h->af_status.ensure((size_t)rows_max * sizeof(int32_t)), "autofit workspace");
    RCCHK(h, h->af_flags.ensure((size_t)rows_max), "autofit workspace");
    RCCHK(h, h->af_init.ensure((size_t)rows_max * 11 * sizeof(double)), "autofit workspace");
    RCCHK(h, h->af_hrst.ensure((size_t)rows_max * sizeof(int32_t)), "autofit workspace");
    RCCHK(h, h->af_rlist.ensure((size_t)sts::kBqRefitBuckets * rows_max * sizeof(int32_t)), "autofit workspace");
    RCCHK(h, h->af_rcount.ensure(sts::kBqRefitBuckets * sizeof(unsigned)), "autofit workspace");
    if (!h->af_host && hipHostMalloc((void **)&h->af_host, (2 * sts::kAfCombosMax + sts::kBqRefitBuckets) * sizeof(int64_t),
                                     0) != hipSuccess)
        return set_err(h, ARIMA_E_OOM, "pinned");
    if (!h->ev_af) HIPCHK(h, hipEventCreateWithFlags(&h->ev_af, hipEventDisableTiming));
    const int P = std::min(kAfContexts, kMaxPipeline);
    for (int j = 0; j < P; ++j) {                  // every context's gather buffer and fit workspace at full size
        FitCtx &c = h->fctx[j];
        RCCHK(h, c.diff.ensure((size_t)N * ldT * sizeof(double)), "autofit workspace");
        RCCHK(h, c.ws.init.ensure((size_t)N * 11 * sizeof(double)), "workspace");
        RCCHK(h, c.ws.hr_status.ensure((size_t)N * sizeof(int32_t)), "workspace");
        RCCHK(h, c.ws.ctl.ensure(kCtlWords * sizeof(unsigned long long)), "workspace");
        RCCHK(h, c.ws.xring.ensure(sts::kExpressRingBytes), "workspace");
        RCCHK(h, c.ws.xready.ensure(sts::kExpressReadyBytes), "workspace");
        if (c.has_done) HIPCHK(h, hipStreamWaitEvent(s, c.ev_done, 0));
    }
    // (1) d: the first of 0..max_d whose differencesOfOrderD(ts, d) passes kpsstest(_, "c") (ARIMA.scala:287-297)
    const int32_t kpss_st = T <= 0 ? ARIMA_ST_NO_DATA : (T < 2 ? ARIMA_ST_NOT_ENOUGH_DATA : ARIMA_ST_OK);
    int32_t *dsel = h->af_dsel.as<int32_t>();
    HIPCHK(h, hipMemsetAsync(dsel, 0xff, (size_t)N * sizeof(int32_t), s));
    if (kpss_st == ARIMA_ST_OK) {
        for (int d = 0; d <= max_d; ++d) {
            RCCHK(h, sts::launch_difference_sel(d_series, ld, h->af_rows.as<double>(), ldT, N, T, dsel, d, s),
                  "difference");
            RCCHK(h, sts::launch_kpss_c(h->af_rows.as<double>(), ldT, T, N, d, dsel, nullptr, s), "kpss");
        }
    }
    // (2) the stepwise walk (findBestARMAModel, :310-375) on each series' differenced row
    sts::AfSeries *st = h->af_state.as<sts::AfSeries>();
    RCCHK(h, sts::launch_af_init(N, dsel, st, kpss_st, s), "autofit init");
    int64_t fits = 0;
    for (int round = 0; kpss_st == ARIMA_ST_OK; ++round) {
        HIPCHK(h, hipMemsetAsync(h->af_counts.ptr, 0, ncombos * sizeof(unsigned), s));
        RCCHK(h, sts::launch_af_plan(N, st, h->af_counts.as<unsigned>(), h->af_lists.as<int32_t>(), s), "autofit plan");
        unsigned counts[sts::kAfCombosMax];
        HIPCHK(h, hipMemcpyAsync(h->af_host, h->af_counts.ptr, ncombos * sizeof(unsigned), hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipStreamSynchronize(s));
        memcpy(counts, h->af_host, ncombos * sizeof(unsigned));
        int64_t *off = h->af_host + sts::kAfCombosMax;
        int64_t total = 0;
        for (int cb = 0; cb < ncombos; ++cb) {
            off[cb] = total;
            total += counts[cb];
        }
        if (total == 0) break;
        fits += total;
        HIPCHK(h, hipMemcpyAsync(h->af_off.ptr, off, ncombos * sizeof(int64_t), hipMemcpyHostToDevice, s));
        HIPCHK(h, hipEventRecord(h->ev_af, s));
        // the round's orders, largest list first, over the fit contexts (several orders fit at once)
        int order[sts::kAfCombosMax];
        for (int cb = 0; cb < ncombos; ++cb) order[cb] = cb;
        std::stable_sort(order, order + ncombos, [&](int a, int b) { return counts[a] > counts[b]; });
        int used = 0;
        for (int oi = 0; oi < ncombos && counts[order[oi]] > 0; ++oi) {
            const int cb = order[oi];
            const int p = (cb / 2) / 3, q = (cb / 2) % 3, I = cb % 2;
            const int64_t cnt = counts[cb];
            FitCtx &c = h->fctx[used % P];
            HIPCHK(h, hipStreamWaitEvent(c.stream, h->ev_af, 0));
            RCCHK(h, sts::launch_gather_rows(h->af_rows.as<double>(), ldT, h->af_lists.as<int32_t>() + (int64_t)cb * N,
                                             cnt, T, c.diff.as<double>(), c.stream), "gather");
            int64_t gridb = 0, xb = 0;
            // fitModel(p, 0, q, diffedTs, intercept, "css-cgd") (:316); rows of order cb from off[cb] (coef stride k);
            // p > 5: the runtime-order path (fit_kernels dispatches it)
            RCCHK(h, fit_kernels(h, c.ws, c.diff.as<double>(), ldT, T, cnt, p, q, I, ARIMA_METHOD_CSS_CGD, nullptr,
                                 h->af_coef.as<double>() + off[cb] * 11, h->af_ll.as<double>() + off[cb],
                                 h->af_status.as<int32_t>() + off[cb], nullptr, nullptr,
                                 h->af_flags.as<uint8_t>() + off[cb], c.stream, nullptr, &gridb, &xb, P > 1), "fit");
            // the Hannan-Rissanen inits and their status, kept for the round's css-bobyqa retries (below)
            const int k = p + q + I;
            if (!(p > 0 && q == 0) && k > 0) {
                HIPCHK(h, hipMemcpyAsync(h->af_init.as<double>() + off[cb] * 11, c.ws.init.ptr,
                                         (size_t)cnt * k * sizeof(double), hipMemcpyDeviceToDevice, c.stream));
            }
            if (!(p > 0 && q == 0))
                HIPCHK(h, hipMemcpyAsync(h->af_hrst.as<int32_t>() + off[cb], c.ws.hr_status.ptr,
                                         (size_t)cnt * sizeof(int32_t), hipMemcpyDeviceToDevice, c.stream));
            HIPCHK(h, end_fit(c, c.stream));
            ++used;
        }
        for (int j = 0; j < std::min(used, P); ++j) HIPCHK(h, hipStreamWaitEvent(s, h->fctx[j].ev_done, 0));
        // fitTryBothStrategies (:315-319): every row of the round whose css-cgd fit threw in the optimizer, refitted
        // with css-bobyqa from the same Hannan-Rissanen init, in place. The rows are listed per dimension k, the host
        // reads the counts back, and each dimension present runs as one kernel sized by its count (one workgroup per
        // retry, not per candidate row), the dimensions on different streams so they run together
        RCCHK(h, sts::launch_bobyqa_refit_list(h->af_off.as<int64_t>(), ncombos, total, h->af_status.as<int32_t>(),
                                               h->af_rlist.as<int32_t>(), rows_max, h->af_rcount.as<unsigned>(), s),
              "bobyqa list");
        HIPCHK(h, hipMemcpyAsync(h->af_host + 2 * sts::kAfCombosMax, h->af_rcount.ptr,
                                 sts::kBqRefitBuckets * sizeof(unsigned), hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipStreamSynchronize(s));
        unsigned retries[sts::kBqRefitBuckets];
        memcpy(retries, h->af_host + 2 * sts::kAfCombosMax, sizeof retries);
        HIPCHK(h, hipEventRecord(h->ev_af, s));
        int launched = 0;
        for (int k = 2; k < sts::kBqRefitBuckets; ++k) {
            if (retries[k] == 0) continue;
            FitCtx &c = h->fctx[launched % P];
            HIPCHK(h, hipStreamWaitEvent(c.stream, h->ev_af, 0));
            RCCHK(h, sts::launch_bobyqa_refit_dim(k, h->af_rows.as<double>(), ldT, T, h->af_lists.as<int32_t>(), N,
                                                  h->af_off.as<int64_t>(), ncombos, 11,
                                                  h->af_rlist.as<int32_t>() + (int64_t)k * rows_max,
                                                  h->af_rcount.as<unsigned>(), (int64_t)retries[k],
                                                  h->af_init.as<double>(), h->af_hrst.as<int32_t>(),
                                                  h->af_coef.as<double>(), h->af_ll.as<double>(),
                                                  h->af_status.as<int32_t>(), h->af_flags.as<uint8_t>(),
                                                  h->bobyqa_wave != 0, c.stream), "bobyqa refit");
            HIPCHK(h, end_fit(c, c.stream));
            ++launched;
        }
        for (int j = 0; j < std::min(launched, P); ++j) HIPCHK(h, hipStreamWaitEvent(s, h->fctx[j].ev_done, 0));
        RCCHK(h, sts::launch_af_update(N, st, h->af_off.as<int64_t>(), h->af_coef.as<double>(), h->af_ll.as<double>(),
                                       h->af_status.as<int32_t>(), h->af_flags.as<uint8_t>(), h->af_best.as<double>(),
                                       max_p, max_q, s), "autofit update");
        if (round > 64) return set_err(h, ARIMA_E_DEVICE, "autofit: the walk did not end");
    }
    RCCHK(h, sts::launch_af_finish(N, st, h->af_best.as<double>(), d_order, d_coef, d_aic, d_status, d_nfits, s),
          "autofit finish");
    if (fits_out) *fits_out = fits;
    return ARIMA_OK;
}

// ARIMA.autoFit over the batch in slices whose workspaces fit the free HBM (the per-call footprint is ~5x
// the input -- the differenced rows plus one gather buffer per fit context -- so a large batch is cut instead of
// failing with ARIMA_E_OOM); option "autofit_slice" fixes the slice (series), 0 = from free HBM.
static int autofit_locked(arima_handle *h, const double *d_series, int64_t N, int32_t T, int64_t ld, int32_t max_p,
                          int32_t max_d, int32_t max_q, int32_t *d_order, double *d_coef, double *d_aic,
                          int32_t *d_status, int32_t *d_nfits, hipStream_t s, int64_t *fits_out) {
    if (max_p < 0 || max_q < 0 || max_d < 0) return set_err(h, ARIMA_E_INVALID_ARG, "bad autofit bounds");
    if (max_p > sts::kAfMaxP || max_d > kMaxD)
        return set_err(h, ARIMA_E_UNSUPPORTED, "autofit: max_p <= 8 (css-bobyqa retries of <= 11 parameters), d <= 16");
    if (N < 0 || T < 0 || ld < T || (N > 0 && (!d_series || !d_order || !d_coef || !d_aic || !d_status)))
        return set_err(h, ARIMA_E_INVALID_ARG, "bad shape");
    h->stats = arima_fit_stats{};
    h->stats_ctx = -1;
    if (N == 0) return ARIMA_OK;
    HIPCHK(h, hipSetDevice(h->device));
    const int64_t ldT = row_stride(h, T);
    int64_t slice = h->autofit_slice;
    if (slice <= 0) {
        size_t free_b = 0, total_b = 0;
        HIPCHK(h, hipMemGetInfo(&free_b, &total_b));
        size_t held = h->af_rows.bytes;            // workspaces this call reuses
        for (int j = 0; j < kAfContexts; ++j) held += h->fctx[j].diff.bytes;
        const int64_t per = (int64_t)(1 + kAfContexts) * ldT * 8 + sts::kAfMaxCand * (11 * 16 + 16) +
                            (int64_t)sts::kAfCombosMax * 4 + 256;
        slice = std::max<int64_t>(4096, (int64_t)((free_b + held) / 10 * 6) / per);
    }
    HIPCHK(h, hipEventRecord(h->ev[0], s));
    int64_t fits = 0;
    for (int64_t f = 0; f < N; f += slice) {
        const int64_t n = std::min(slice, N - f);
        int64_t fs = 0;
        RCCHK(h, autofit_slice(h, d_series + f * ld, n, T, ld, max_p, max_d, max_q, d_order + f * 4, d_coef + f * 11,
                               d_aic + f, d_status + f, d_nfits ? d_nfits + f : nullptr, s, &fs), "autofit");
        fits += fs;
    }
    HIPCHK(h, hipEventRecord(h->ev[3], s));
    h->stats.n_series = fits;
    if (fits_out) *fits_out = fits;
    return ARIMA_OK;
}

int arima_autofit_batch_device(arima_handle *h, const double *d_series, int64_t n_series, int32_t T, int64_t ld,
                               int32_t max_p, int32_t max_d, int32_t max_q, int32_t *d_order_out,
                               double *d_coef_out, double *d_aic_out, int32_t *d_status_out, int32_t *d_n_fits_out,
                               void *stream) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    HIPCHK(h, hipSetDevice(h->device));          // before any stream work
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    begin_call(h, s);
    const int rc = autofit_locked(h, d_series, n_series, T, ld, max_p, max_d, max_q, d_order_out, d_coef_out,
                                  d_aic_out, d_status_out, d_n_fits_out, s, nullptr);
    HIPCHK(h, end_call(h, s));
    // the walk synchronised with the device once per round, so its fits have finished: a watchdog fault that one of
    // them recorded is reported by this call, not by a later unrelated one
    if (rc != ARIMA_OK) return rc;
    HIPCHK(h, hipStreamSynchronize(s));
    return take_fault(h);
}

int arima_autofit_batch(arima_handle *h, const double *series, int64_t N, int32_t T, int32_t max_p, int32_t max_d,
                        int32_t max_q, int32_t *order_out, double *coef_out, double *aic_out, int32_t *status_out,
                        int32_t *n_fits_out) {
    if (!h) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (N < 0 || T < 0) return set_err(h, ARIMA_E_INVALID_ARG, "bad shape");
    if (N == 0) return ARIMA_OK;
    if (!series || !order_out || !coef_out || !aic_out || !status_out) return set_err(h, ARIMA_E_INVALID_ARG, "null buffer");
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t s = h->stream;
    begin_call(h, s);
    RCCHK(h, h->h_series.ensure((size_t)N * std::max(T, 1) * sizeof(double)), "staging");
    RCCHK(h, h->af_out_order.ensure((size_t)N * 4 * sizeof(int32_t)), "staging");
    RCCHK(h, h->af_out_coef.ensure((size_t)N * 11 * sizeof(double)), "staging");
    RCCHK(h, h->af_out_aic.ensure((size_t)N * sizeof(double)), "staging");
    RCCHK(h, h->af_out_status.ensure((size_t)N * sizeof(int32_t)), "staging");
    RCCHK(h, h->af_out_nfits.ensure((size_t)N * sizeof(int32_t)), "staging");
    if (T > 0) HIPCHK(h, hipMemcpyAsync(h->h_series.ptr, series, (size_t)N * T * sizeof(double), hipMemcpyHostToDevice, s));
    int rc = autofit_locked(h, h->h_series.as<double>(), N, T, T, max_p, max_d, max_q, h->af_out_order.as<int32_t>(),
                            h->af_out_coef.as<double>(), h->af_out_aic.as<double>(), h->af_out_status.as<int32_t>(),
                            h->af_out_nfits.as<int32_t>(), s, nullptr);
    if (rc == ARIMA_OK) {
        HIPCHK(h, hipMemcpyAsync(order_out, h->af_out_order.ptr, (size_t)N * 4 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipMemcpyAsync(coef_out, h->af_out_coef.ptr, (size_t)N * 11 * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipMemcpyAsync(aic_out, h->af_out_aic.ptr, (size_t)N * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipMemcpyAsync(status_out, h->af_out_status.ptr, (size_t)N * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        if (n_fits_out)
            HIPCHK(h, hipMemcpyAsync(n_fits_out, h->af_out_nfits.ptr, (size_t)N * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    }
    HIPCHK(h, end_call(h, s));
    HIPCHK(h, hipStreamSynchronize(s));
    if (rc != ARIMA_OK) return rc;
    return take_fault(h);
}

int arima_kpss_batch(arima_handle *h, const double *series, int64_t N, int32_t T, double *stat_out, int32_t *status_out) {
    if (!h || N < 0 || T < 0) return ARIMA_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (N == 0) return ARIMA_OK;
    if (!series || !stat_out || !status_out) return set_err(h, ARIMA_E_INVALID_ARG, "null buffer");
    const int32_t st = T <= 0 ? ARIMA_ST_NO_DATA : (T < 2 ? ARIMA_ST_NOT_ENOUGH_DATA : ARIMA_ST_OK);
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t s = h->stream;
    begin_call(h, s);
    RCCHK(h, h->h_ll.ensure((size_t)N * sizeof(double)), "staging");
    if (st == ARIMA_ST_OK) {
        int64_t ld = 0;
        RCCHK(h, upload_padded(h, series, N, T, &ld, s), "upload");
        RCCHK(h, sts::launch_kpss_c(h->diff.as<double>(), ld, T, N, 0, nullptr, h->h_ll.as<double>(), s), "kpss");
        HIPCHK(h, hipMemcpyAsync(stat_out, h->h_ll.ptr, (size_t)N * sizeof(double), hipMemcpyDeviceToHost, s));
    }
    HIPCHK(h, end_call(h, s));
    HIPCHK(h, hipStreamSynchronize(s));
    for (int64_t i = 0; i < N; ++i) {
        status_out[i] = st;
        if (st != ARIMA_ST_OK) stat_out[i] = NAN;
    }
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
