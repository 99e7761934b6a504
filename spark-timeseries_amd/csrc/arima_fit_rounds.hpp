#pragma once
// arima_fit_rounds.hpp — the CSS-CGD fit as rounds of streaming passes (fit_kernel = 2; included by
// arima_kernels_impl.hpp after k_cg_fit, which serves the last rounds' long-running series).
//
// Why: a pass over a series is a chain of dependent fp64 ops (the CSS recursion keeps the reference's
// rounding), so a lane-per-series pass is latency-bound unless many waves share each SIMD. k_cg_fit keeps each
// series' optimizer state in LDS next to its passes, which pins it to one wave per SIMD, and its pass lanes idle
// whenever fewer than 64 of a wave's slots want the same kind of pass. Here the optimizer state machine and the passes
// are separate kernels, and every series takes one step per round:
//   k_rounds_init      HR status / initial point -> the state record (CGLane, in HBM), a G request in list G of round 0
//   k_rounds_pass      one pass per listed request: full 64-lane tiles of one kind (G, or F with 1 + nsp chains), no
//                      optimizer state in registers -> several waves per SIMD hide the chains' latency and the row
//                      streams run near HBM bandwidth; responses (objective, predicted objectives, gradient) to HBM
//   k_rounds_advance   each served series applies its response to its record (CGLane::step, the same state machine as
//                      k_cg_fit's slots) and lists its next request for round r + 1 -- or, once few series are left
//                      (tail_at) or the last round is reached, for k_cg_fit, which resumes them from their records
// Every evaluation is the same operation sequence as in k_cg_fit (css_pass / css_pass_multi / css_to_loglik on the
// request's point, predicted points point + alpha * dir as CGLane::spec_point computes them), so results and
// evaluation counts are bit-identical whichever kernel served a request.
//
// Round lists: kRoundLists int32 series-id lists per round, by cost: 0 = G, then F with NS, ..., 0 predicted points.
// Round r reads lists[r & 1]; counts live in rc[r * kRcStride + t], the pass kernel's tile counter in
// rc[r * kRcStride + kRoundLists] (rounds 0 .. max_rounds: the last compaction fills round max_rounds' counts, which
// no pass reads), the tail list's count in rc[(max_rounds + 1) * kRcStride].
// The lists are kept in series order: the advance kernel only marks each series' next list (mark[sid]), and an
// order-preserving compaction (count per range of series -> scan -> scatter) builds round r + 1's lists. A tile of
// 64 requests then covers 64 neighbouring rows (a few 2-MiB pages) instead of 64 scattered ones: with scattered
// rows the passes ran 3-4x slower per request (address translation; profiles/r03/rounds).
// Marks: 0..kRoundLists-1 = the list of the posted request, kMarkTail = hand over to k_cg_fit, kMarkNone = done.
#include "arima_device.hpp"

namespace sts {

template <int K>
using RoundLane = CGLane<K, spec_ns<K>(), spec_nc<K>()>;
template <int K>
constexpr int rounds_rec_stride() { return (int)((sizeof(RoundLane<K>) + 127) / 128 * 128); }
template <int K>
constexpr int rounds_resp_words() { return 1 + spec_ns<K>() + K; }
static_assert(kRoundLists == 2 + spec_ns<5>(), "lists: G and F with 0..NS predictions (arima_launch.hpp)");

#ifndef STS_ROUNDS_PF_F
#define STS_ROUNDS_PF_F 2
#endif
#ifndef STS_ROUNDS_PF_G
#define STS_ROUNDS_PF_G 2
#endif
constexpr int kRoundsPfF = STS_ROUNDS_PF_F;   // 128-B chunks in flight per lane (the other waves of the SIMD hide
constexpr int kRoundsPfG = STS_ROUNDS_PF_G;   // the rest of the latency)

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
constexpr uint8_t kMarkTail = 0xfe, kMarkNone = 0xff;

// Wave-aggregated append of `val` to list[cnt++] for the lanes with want (wave-uniform call).
__device__ __forceinline__ void wave_append(unsigned *cnt, int32_t *list, bool want, int32_t val) {
    const unsigned long long m = __ballot(want);
    if (m == 0ull) return;
    const int lane = lane_id();
    const int leader = __ffsll((long long)m) - 1;
    unsigned base = 0;
    if (lane == leader) base = atomicAdd(cnt, (unsigned)__popcll(m));
    base = __shfl(base, leader);
    if (want) list[base + (unsigned)__popcll(m & ((1ull << lane) - 1ull))] = val;
}

template <int K>
__device__ __forceinline__ RoundLane<K> *rec_at(unsigned char *rec, int64_t sid) {
    return reinterpret_cast<RoundLane<K> *>(rec + sid * (int64_t)rounds_rec_stride<K>());
}

// ---- round 0: initial points (ARIMA.scala:99-109), failed Hannan-Rissanen fits reported at once ----------------
template <int K>
__global__ __launch_bounds__(64) void k_rounds_init(int64_t N, const double *__restrict__ init,
                                                    const int32_t *__restrict__ init_status, unsigned char *rec,
                                                    uint8_t *__restrict__ mark, double *__restrict__ coef_out,
                                                    double *__restrict__ ll_out, int32_t *__restrict__ status_out,
                                                    int32_t *__restrict__ n_eval_out, int32_t *__restrict__ n_grad_out,
                                                    uint8_t *__restrict__ flags_out, unsigned long long *__restrict__ ctl) {
    const int64_t sid = (int64_t)blockIdx.x * 64 + lane_id();
    const bool in = sid < N;
    const int st0 = !in ? ARIMA_ST_OK : (init_status ? init_status[sid] : ARIMA_ST_OK);
    if (in && st0 != ARIMA_ST_OK) {
        double nanc[K];
#pragma unroll
        for (int j = 0; j < K; ++j) nanc[j] = __builtin_nan("");
        write_fit<K>(sid, st0, nanc, 0.0, 0, 0, 0, coef_out, ll_out, status_out, n_eval_out, n_grad_out, flags_out);
    }
    const bool go = in && st0 == ARIMA_ST_OK;
    if (go) {
        double x0[K];
#pragma unroll
        for (int j = 0; j < K; ++j) x0[j] = init[sid * K + j];
        RoundLane<K> S;
        S.start_posted(x0);                    // computeObjectiveGradient(point): a G request
        *rec_at<K>(rec, sid) = S;
    }
    if (in) mark[sid] = go ? (uint8_t)0 : kMarkNone;     // round 0: list 0 (G)
    const unsigned long long failed = __ballot(in && !go);
    if (lane_id() == 0 && failed) atomicAdd(&ctl[32], (unsigned long long)__popcll(failed));
}

// ---- order-preserving compaction of the marks into round ro's lists (and the tail list) ---------------------------
// Ranges of kRangeSeries series; k_rounds_count counts each range's marks per list (+ tail), k_rounds_scan turns the
// counts into offsets (one workgroup) and the list sizes of round ro, k_rounds_scatter writes the series ids.
constexpr int kRangeSeries = 2048;
constexpr int kRangeWords = 8;                         // per range: kRoundLists lists + the tail, padded

static __global__ __launch_bounds__(64) void k_rounds_count(int64_t N, const uint8_t *__restrict__ mark,
                                                     unsigned *__restrict__ counts) {
    const int lane = lane_id();
    const int64_t first = (int64_t)blockIdx.x * kRangeSeries;
    unsigned c[kRoundLists + 1] = {};
    for (int i = 0; i < kRangeSeries; i += 64) {
        const int64_t sid = first + i + lane;
        const int m = sid < N ? mark[sid] : kMarkNone;
#pragma unroll
        for (int t = 0; t <= kRoundLists; ++t)
            c[t] += (unsigned)__popcll(__ballot(m == (t < kRoundLists ? t : kMarkTail)));
    }
    if (lane <= kRoundLists) {
        unsigned v = 0;
#pragma unroll
        for (int t = 0; t <= kRoundLists; ++t) v = lane == t ? c[t] : v;
        counts[(size_t)blockIdx.x * kRangeWords + lane] = v;
    }
}

// one workgroup of 1024 threads: exclusive scan of every column over the ranges (in place), list sizes to rc_out,
// the tail's size added to *tail_n (its offsets start there)
static __global__ __launch_bounds__(1024) void k_rounds_scan(int nranges, unsigned *__restrict__ counts,
                                                      unsigned *__restrict__ rc_out, unsigned *__restrict__ tail_n) {
    __shared__ unsigned part[1024];
    __shared__ unsigned carry;
    const int tid = (int)threadIdx.x;
    for (int t = 0; t <= kRoundLists; ++t) {
        if (tid == 0) carry = t == kRoundLists ? *tail_n : 0u;
        __syncthreads();
        for (int b0 = 0; b0 < nranges; b0 += 1024) {
            const int b = b0 + tid;
            const unsigned v = b < nranges ? counts[(size_t)b * kRangeWords + t] : 0u;
            part[tid] = v;
            __syncthreads();
            for (int off = 1; off < 1024; off <<= 1) {       // inclusive Hillis-Steele scan
                const unsigned add = tid >= off ? part[tid - off] : 0u;
                __syncthreads();
                part[tid] += add;
                __syncthreads();
            }
            if (b < nranges) counts[(size_t)b * kRangeWords + t] = carry + part[tid] - v;
            __syncthreads();
            if (tid == 1023) carry += part[1023];
            __syncthreads();
        }
        if (tid == 0) {
            if (t < kRoundLists) rc_out[t] = carry;
            else *tail_n = carry;
        }
        __syncthreads();
    }
}

static __global__ __launch_bounds__(64) void k_rounds_scatter(int64_t N, uint8_t *__restrict__ mark,
                                                       const unsigned *__restrict__ offsets,
                                                       int32_t *__restrict__ lists, int32_t *__restrict__ tail) {
    const int lane = lane_id();
    const int64_t first = (int64_t)blockIdx.x * kRangeSeries;
    unsigned o[kRoundLists + 1];
#pragma unroll
    for (int t = 0; t <= kRoundLists; ++t) o[t] = offsets[(size_t)blockIdx.x * kRangeWords + t];
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int i = 0; i < kRangeSeries; i += 64) {
        const int64_t sid = first + i + lane;
        const int m = sid < N ? mark[sid] : kMarkNone;
#pragma unroll
        for (int t = 0; t <= kRoundLists; ++t) {
            const bool mine = m == (t < kRoundLists ? t : kMarkTail);
            const unsigned long long bm = __ballot(mine);
            if (mine) {
                const unsigned pos = o[t] + (unsigned)__popcll(bm & below);
                if (t < kRoundLists) lists[(size_t)t * N + pos] = (int32_t)sid;
                else tail[pos] = (int32_t)sid;
            }
            o[t] += (unsigned)__popcll(bm);
        }
        if (m == kMarkTail) mark[sid] = kMarkNone;    // listed once
    }
}

// ---- one pass per listed request ---------------------------------------------------------------------------------
// Persistent: each wave claims 64-entry tiles (G tiles first, then F by decreasing chain count), so a round ends
// with its cheapest tiles. Lanes past the end of a list stream the tile's first row with its coefficients and
// write nothing (uniform control flow, no extra bytes: the row is already being read).
template <int P, int Q, int I, bool SMEAR>
__global__ __launch_bounds__(64) void k_rounds_pass(int r, const double *__restrict__ y, int64_t ld, int n,
                                                    int64_t N, const unsigned char *rec, double *__restrict__ resp,
                                                    const int32_t *__restrict__ lists, unsigned *__restrict__ rc,
                                                    unsigned long long *__restrict__ ctl) {
    constexpr int K = I + P + Q;
    constexpr int NS = spec_ns<K>();
    constexpr int RW = rounds_resp_words<K>();
    using Lane = RoundLane<K>;
    const int lane = lane_id();
    unsigned *rcr = rc + (size_t)r * kRcStride;
    const int32_t *lr = lists + (size_t)(r & 1) * kRoundLists * N;
    unsigned cnt[kRoundLists], tiles[kRoundLists + 1];
    tiles[0] = 0;
#pragma unroll
    for (int t = 0; t < kRoundLists; ++t) {
        cnt[t] = rcr[t];
        tiles[t + 1] = tiles[t] + (cnt[t] + 63u) / 64u;
    }
    const unsigned total = tiles[kRoundLists];
    unsigned long long lane_f = 0, lane_g = 0, wave_f = 0, wave_g = 0, wave_m = 0, chains = 0;
    for (;;) {
        unsigned tile = 0;
        if (lane == 0) tile = atomicAdd(&rcr[kRoundLists], 1u);
        tile = __shfl(tile, 0);
        if (tile >= total) break;
        int t = 0;
#pragma unroll
        for (int u = 1; u < kRoundLists; ++u)
            if (tile >= tiles[u]) t = u;
        const unsigned idx = (tile - tiles[t]) * 64u + (unsigned)lane;
        const bool valid = idx < cnt[t];
        const int32_t *lt = lr + (size_t)t * N;
        const int64_t sid = lt[valid ? idx : (tile - tiles[t]) * 64u];
        const Lane &S = *rec_at<K>(const_cast<unsigned char *>(rec), sid);
        const double *row = y + sid * ld;
        double *out = resp + sid * RW;
        double c[K];
        if (t == 0) {
#pragma unroll
            for (int j = 0; j < K; ++j) c[j] = S.point[j];
            double css, g[K];
            css_pass<P, Q, I, true, SMEAR, kRoundsPfG>(row, n, c, css, g);
            if (valid) {
                out[0] = css_to_loglik(css, n);
#pragma unroll
                for (int j = 0; j < K; ++j) out[1 + NS + j] = g[j];
            }
            wave_g += lane == 0;
            lane_g += valid;
        } else {
            const double al = S.ev_alpha;
#pragma unroll
            for (int j = 0; j < K; ++j) c[j] = S.point[j] + al * S.dir[j];
            auto multi = [&](auto NCHc) {
                constexpr int NCH = decltype(NCHc)::value;
                double cm[NCH][K], cssm[NCH];
#pragma unroll
                for (int j = 0; j < K; ++j) cm[0][j] = c[j];
#pragma unroll
                for (int h = 1; h < NCH; ++h) {
                    double cs[K];
                    S.spec_point(h - 1, cs);
#pragma unroll
                    for (int j = 0; j < K; ++j) cm[h][j] = cs[j];
                }
                css_pass_multi<P, Q, I, NCH, kRoundsPfF>(row, n, cm, cssm);
                if (valid) {
#pragma unroll
                    for (int h = 0; h < NCH; ++h) out[h] = css_to_loglik(cssm[h], n);
                }
            };
            const int nch = 1 + NS - (t - 1);         // list 1: NS predictions, ..., list NS + 1: none
            if constexpr (NS >= 2) {
                if (nch == 3) multi(IC<3>{});
                else if (nch == 2) multi(IC<2>{});
                else multi(IC<1>{});
            } else if constexpr (NS == 1) {
                if (nch == 2) multi(IC<2>{});
                else multi(IC<1>{});
            } else {
                multi(IC<1>{});
            }
            if (nch > 1) wave_m += lane == 0; else wave_f += lane == 0;
            lane_f += valid;
            chains += valid ? (unsigned long long)nch : 0ull;
        }
    }
    atomicAdd(&ctl[1], lane_f);
    atomicAdd(&ctl[2], lane_g);
    atomicAdd(&ctl[9], chains);
    if (lane == 0) {
        atomicAdd(&ctl[3], wave_f);
        atomicAdd(&ctl[4], wave_g);
        atomicAdd(&ctl[8], wave_m);
    }
}

// ---- each served series takes its response and posts its next request ------------------------------------------
// Grid-stride over the round's entries (the lists back to back); marks each series' next list. A series leaves the
// rounds when it finishes (its result is written) or, in a hand-off round (few series left, or the last round), for
// the tail list that k_cg_fit resumes from.
template <int P, int Q, int I>
__global__ __launch_bounds__(64) void k_rounds_advance(int r, int last, unsigned tail_at, int64_t N,
                                                       unsigned char *rec, const double *__restrict__ resp,
                                                       const int32_t *__restrict__ lists, const unsigned *__restrict__ rc,
                                                       uint8_t *__restrict__ mark, double *__restrict__ coef_out, double *__restrict__ ll_out,
                                                       int32_t *__restrict__ status_out,
                                                       int32_t *__restrict__ n_eval_out,
                                                       int32_t *__restrict__ n_grad_out, uint8_t *__restrict__ flags_out,
                                                       unsigned long long *__restrict__ ctl) {
    constexpr int K = I + P + Q;
    constexpr int NS = spec_ns<K>();
    constexpr int RW = rounds_resp_words<K>();
    using Lane = RoundLane<K>;
    const int lane = lane_id();
    const unsigned *rcr = rc + (size_t)r * kRcStride;
    const int32_t *lr = lists + (size_t)(r & 1) * kRoundLists * N;
    unsigned cnt[kRoundLists], start[kRoundLists + 1];
    start[0] = 0;
#pragma unroll
    for (int t = 0; t < kRoundLists; ++t) {
        cnt[t] = rcr[t];
        start[t + 1] = start[t] + cnt[t];
    }
    const unsigned total = start[kRoundLists];
    const bool handoff = last || total <= tail_at;
    unsigned long long evals = 0, grads = 0, hits = 0, done = 0;
    for (unsigned base = blockIdx.x * 64u; base < total; base += gridDim.x * 64u) {
        const unsigned idx = base + (unsigned)lane;
        const bool valid = idx < total;
        int t = 0;
#pragma unroll
        for (int u = 1; u < kRoundLists; ++u)
            if (idx >= start[u]) t = u;
        if (!valid) break;                               // the last, partial iteration (no wave-wide calls below)
        const int64_t sid = lr[(size_t)t * N + (idx - start[t])];
        int next;                                        // list of the next request, kRoundLists = done / dropped
        {
            Lane S = *rec_at<K>(rec, sid);
            const double *in = resp + sid * RW;
            double g[K];
            if (t == 0) {
#pragma unroll
                for (int j = 0; j < K; ++j) g[j] = in[1 + NS + j];
            } else {
#pragma unroll
                for (int j = 0; j < K; ++j) g[j] = 0.0;
                const int nsp = NS - (t - 1);
#pragma unroll
                for (int h = 1; h <= NS; ++h)
                    if (h <= nsp) S.spec_store(h - 1, in[h]);
            }
            S.req = REQ_NONE;
            S.step(in[0], g);
            if (S.done()) {
                double pt[K];
#pragma unroll
                for (int j = 0; j < K; ++j) pt[j] = S.point[j];
                write_fit<K>(sid, S.status, pt, S.prev_obj, S.n_eval, S.n_grad,
                             S.status == ARIMA_ST_OK ? model_flags<P, Q, I>(pt) : (uint8_t)0, coef_out, ll_out,
                             status_out, n_eval_out, n_grad_out, flags_out);
                evals += S.n_eval;
                grads += S.n_grad;
                hits += S.spec_hits;
                done++;
                next = kRoundLists;
            } else if (S.req == REQ_NONE) {               // invariant broken: drop the series, report a fault
                record_fault(ctl, FAULT_NO_REQUEST, (unsigned long long)r, (unsigned long long)sid, S.pc,
                             ((unsigned long long)S.status << 16) | S.n_eval, 0ull);
                next = kRoundLists;
            } else {
                *rec_at<K>(rec, sid) = S;
                next = S.req == REQ_G ? 0 : 1 + NS - (int)S.rq_nspec;
            }
        }
        mark[sid] = next == kRoundLists ? kMarkNone : (handoff ? kMarkTail : (uint8_t)next);
    }
    atomicAdd(&ctl[5], evals);
    atomicAdd(&ctl[6], grads);
    atomicAdd(&ctl[7], hits);
    atomicAdd(&ctl[32], done);
}

}  // namespace sts
