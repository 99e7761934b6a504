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

#include <algorithm>
#include <utility>

#include "arima_device.hpp"
#include "arima_launch.hpp"
#include <type_traits>

namespace sts {

template <int V>
using IC = std::integral_constant<int, V>;

// =======================================================================================================
// Hannan-Rissanen init (ARIMA.scala:216-242)
// =======================================================================================================
// F: the row generators difference the caller's raw row on the fly (dd = 1, fused differencing); F = false (dd = 0)
// streams differenced rows with no differencing logic. At high orders the fused generators cost ~110 registers
// (k_hr_init<5,5,1>: 399 in round 5, 512 + scratch with the runtime dd; C4 0.92 -> 0.77 M series/s,
// profiles/r06/p_c4fuse), so the runtime fuses only where that pays (fuse_pays, arima_launch.hpp)
template <int P, int Q, int I, bool F>
__global__ __launch_bounds__(256) void k_hr_init(const double *__restrict__ y, int64_t ld, int n, int64_t N,
                                                 double *__restrict__ init_out, int32_t *__restrict__ status_out,
                                                 int dd, FitPrep prep) {
    constexpr int K = I + P + Q;
    constexpr int KA = K > 0 ? K : 1;
    constexpr int M = P > Q ? P : Q;
    constexpr int m = M + 1;
    fit_prep(prep);                          // the fit kernel's counters and ring for the launch after this one
    // grid-stride over series: a grid smaller than N / 256 blocks bounds the rows in flight (their 2(C_A + C_B)
    // passes then re-read from the caches instead of HBM)
    for (int64_t sid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; sid < N;
         sid += (int64_t)gridDim.x * blockDim.x) {
    const double *row = y + sid * ld;
    int st = hr_shape_status(n, P, Q, I);
    double beta[KA];
#pragma unroll
    for (int j = 0; j < KA; ++j) beta[j] = __builtin_nan("");
    if (st == ARIMA_ST_OK) {
        double ab[1 + m];
        ARGen<m, 1, F> genA;
        genA.y = row;
        genA.dd = F ? dd : 0;
        st = stream_ols<1 + m>(genA, row, n, n - m, ab);           // Autoregression.fitModel(y, m)  :225
        if (st == ARIMA_ST_OK) {
            HRGen<P, Q, I, F> genB;
            genB.y = row;
            genB.dd = F ? dd : 0;
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
}

// =======================================================================================================
// AR-only shortcut of fitModel (ARIMA.scala:90-96): Autoregression.fitModel(diffed, p, !includeIntercept)
// =======================================================================================================
template <int P, int I>
__global__ __launch_bounds__(256) void k_ar_fit(const double *__restrict__ y, int64_t ld, int n, int64_t N,
                                                double *__restrict__ coef_out, double *__restrict__ ll_out,
                                                int32_t *__restrict__ status_out, int32_t *__restrict__ n_eval_out,
                                                int32_t *__restrict__ n_grad_out, uint8_t *__restrict__ flags_out,
                                                int dd) {
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
        gen.dd = dd;
        st = stream_ols<K>(gen, row, n, n - P, b);
        if (st == ARIMA_ST_OK) {
#pragma unroll
            for (int j = 0; j < K; ++j) beta[j] = b[j];
            double css, g[K];
            css_pass<P, 0, I, false, false, true>(row, n, beta, css, g, dd);
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
// Persistent CSS-CGD fit kernel (ARIMA.scala:174-200 over a batch)
//
// One 256-lane workgroup (4 waves, one per SIMD) per CU. Each wave owns SPW > 64 optimizer SLOTS in LDS (one
// series each: CGLane state + series id). A wave iteration picks up to 64 slots that posted the SAME kind of
// request (all objective F, or all gradient G), assigns them to its lanes, runs one pass over each assigned
// slot's series (a G pass also yields the objective; an F pass evaluates the request's predicted points as extra
// chains over the same streamed bytes), and lets each lane advance its slot's state machine with the response.
// Finished slots are refilled from a device work counter (wave-aggregated atomics). Oversubscribing the lanes
// (SPW/64 slots per lane) keeps the passes homogeneous and full: gradient passes cost several objective passes,
// and a mixed pass would make objective lanes wait for them.
// =======================================================================================================
template <int K>
__device__ __forceinline__ void write_fit(int64_t sid, int status, const double (&coef)[K], double ll, int n_eval,
                                          int n_grad, uint8_t flags, double *coef_out, double *ll_out,
                                          int32_t *status_out, int32_t *n_eval_out, int32_t *n_grad_out,
                                          uint8_t *flags_out, int path = 1) {
    const bool ok = status == ARIMA_ST_OK;
#pragma unroll
    for (int j = 0; j < K; ++j) coef_out[sid * K + j] = ok ? coef[j] : __builtin_nan("");
    ll_out[sid] = ok ? ll : __builtin_nan("");
    status_out[sid] = status;
    if (n_eval_out) n_eval_out[sid] = n_eval;
    if (n_grad_out) n_grad_out[sid] = n_grad;
    if (flags_out) flags_out[sid] = ok ? flags : 0;
#ifdef STS_TIMING
    // diagnostics build only: the finish time (100 MHz real-time counter) replaces the LL, flags = path taken
    ll_out[sid] = (double)__builtin_amdgcn_s_memrealtime();
    if (flags_out) flags_out[sid] = (uint8_t)path;
#endif
}

// speculation policy per parameter count (tests/sim/cglane_sim.cpp measures it: 2 predictions per request and a
// 4-entry line-search cache remove the bracket's value-independent passes and Brent's first two)
template <int K>
constexpr int spec_ns() { return 2; }
template <int K>
constexpr int spec_nc() { return 4; }

// One optimizer slot in LDS, padded to an odd number of 8-byte words so that 64 lanes reading the same field of
// 64 different slots with ds_read_b64 spread over the banks (MI355X_MICROARCH.md LDS table).
template <int K>
struct FitSlotCore {
    CGLane<K, spec_ns<K>(), spec_nc<K>()> s;
    int64_t sid;                    // series of the slot, -1 = empty
#ifdef STS_TIMING
    double t_start, t_donate;       // diagnostics build only: pick-up and hand-off times (100 MHz counter)
#endif
};

// diagnostics build only: coef[0] / coef[1] of a finished series = its pick-up / hand-off time
template <int K>
__device__ __forceinline__ void timing_stamp(const FitSlotCore<K> &S, double *coef_out) {
#ifdef STS_TIMING
    if constexpr (K >= 2) {
        coef_out[S.sid * K + 0] = S.t_start;
        coef_out[S.sid * K + 1] = S.t_donate;
    }
#endif
}
template <int K>
struct alignas(8) FitSlot {
    static constexpr int kWords = (int)((sizeof(FitSlotCore<K>) + 7) / 8);
    static constexpr int kPadWords = (kWords % 2 == 0) ? 1 : 2;
    FitSlotCore<K> c;
    double pad[kPadWords];
};

constexpr int kFitWaves = kFitBlockWaves;    // waves per workgroup (arima_launch.hpp)
constexpr bool kFRide = true;                // objective requests fill the idle lanes of gradient passes
constexpr int kOldEvals = 128;               // evaluations after which a series is served with priority
constexpr bool kNchChoice = true;            // objective pass width chosen by evaluations per cost
constexpr int kChainOverhead16 = 6;          // per-step streaming cost of a pass, in 1/16 chains

constexpr int kFitLdsBudget = 160 * 1024 - 1024;
// slots per wave: as many as the LDS holds, at most 2 per lane, a multiple of 8 (at least 64 unless more than
// one wave per SIMD shares the LDS)
template <int K>
constexpr int fit_slots_per_wave() {
    constexpr int fit = kFitLdsBudget / (kFitWavesPerCU * (int)sizeof(FitSlot<K>));
    constexpr int cap = fit > 128 ? 128 : fit;
    return (cap / 8) * 8;
}

// ---- express path: one long-running series per wave, its row in LDS -------------------------------------
// The launch's critical path is its slowest series (a few hundred of 1M series need 10-60x the median number of
// passes). In the lane-per-series waves a pass costs the whole wave's instruction stream (~30-60 instructions per
// time step), so such a series advances by one pass per wave pass. Express workgroups (the last blocks of the
// grid) instead give a long-running series a whole wave: the row is staged once into LDS, objective passes run
// the request's point and its predicted points on separate lanes, and gradient passes split dEdTheta's columns
// over lanes — a pass then costs about one chain of instructions. Hand-off: an idle express wave takes a ticket
// (ctl[20]); a bulk wave that sees an unserved ticket claims the next fill index (ctl[21], by compare-and-swap and
// only while it is below the ticket count), donates its oldest slot with >= kDonateEvals evaluations into that ring
// entry and publishes it (release, then the entry's ready word = index + 1); the express wave polls its entry's
// ready word (acquire). Express waves exit once every bulk wave has
// finished (ctl[22]) and no fill is left for their ticket, so they never hold up the launch.
// Ring: a fill index is only claimed while a ticket is waiting for it (fill < tickets, CAS below) and is never
// reused within a launch (fills stop at kExpressRing; a launch hands off a few thousand series at most in practice):
// a reused entry's lines can survive, stale, in the reading XCD's L2 from the previous round (observed on MI355X:
// an entry's tag read stale for 20 s while its ready word had moved on).
constexpr int kExpressRing = kExpressRingEntries;
constexpr int kExpressEntryBytes = 512;      // ring stride reserved per entry (>= sizeof(FitSlotCore<K>) for K <= 11)
constexpr int kExpressGroups = 1;            // series per express wave (2 and 4 measured slower)
constexpr int kDonateEvals = 256;            // a slot is donated only after this many evaluations ...
constexpr int kDonateEvalsDrained = 32;      // ... or this many once the batch's work counter has run out

template <int K>
constexpr int express_state_bytes() { return (int)((sizeof(FitSlotCore<K>) + 15) / 16 * 16); }

// longest differenced series an express wave can stage next to its state and exchange area (per-wave LDS share)
template <int K>
constexpr int express_max_n(int lds_per_wave) { return (lds_per_wave - express_state_bytes<K>() - 16 * 8) / 8 - 1; }

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Ring entry = the slot's state words + a tag word (the fill index + 1) in the entry's last 8 bytes. Entry words
// move with agent-scope atomic stores / loads (coherent across the XCDs' L2s whatever the fences do); the reader
// accepts an entry only when both its ready word and its tag carry its ticket.
constexpr int kExpressTagWord = kExpressEntryBytes / 8 - 1;

// ring entries this launch may fill: ctl[19] when the host set it (option "express_ring", tests reach the cap with a
// small ring), else the whole ring. Tickets beyond it are never filled (their groups retire); their series stay on
// the bulk path, so reaching the cap changes where a series is fitted, never its result.
// With the drain merge on (ctl[44] > 0) the ring's upper three quarters are the merge pool, so hand-offs stop at the
// lower quarter (8 192).
constexpr int kMergeCap = kExpressRing / 4 * 3;   // merge pool entries per launch (never reused within it)
__device__ __forceinline__ unsigned long long express_ring_entries(const unsigned long long *ctl) {
    const unsigned long long r = ctl[19];
    const unsigned long long cap = ctl[44] ? (unsigned long long)(kExpressRing - kMergeCap) : (unsigned long long)kExpressRing;
    return (r == 0 || r > cap) ? cap : r;
}

// Every word shared between workgroups of a launch is accessed as a GLOBAL (address space 1) agent-scope access,
// never flat (a flat load can keep hitting this CU's stale L1 line; cdna_hip_programming.md Guideline 16).
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long *p) {
    return __hip_atomic_load((const gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned ld_agent(const unsigned *p) {
    return __hip_atomic_load((const gu32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store((gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned *p, unsigned v) {
    __hip_atomic_store((gu32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// memory-side read (an atomic RMW that changes nothing): never served by a possibly stale cache line
__device__ __forceinline__ unsigned long long rd_fresh(const unsigned long long *p) {
    return __hip_atomic_fetch_or((gu64 *)p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned rd_fresh(const unsigned *p) {
    return __hip_atomic_fetch_or((gu32 *)p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long add_agent(unsigned long long *p, unsigned long long v) {
    return __hip_atomic_fetch_add((gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// returns the value found (== expected on success)
__device__ __forceinline__ unsigned long long cas_agent(unsigned long long *p, unsigned long long expected,
                                                        unsigned long long desired) {
    __hip_atomic_compare_exchange_strong((gu64 *)p, &expected, desired, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    return expected;
}
// agent acquire whose L1 invalidate has completed before any later load issues (the fence alone is asynchronous)
__device__ __forceinline__ void acquire_agent() {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int K>
__device__ __forceinline__ void publish_core(unsigned long long *dst, const FitSlotCore<K> *src, int lane,
                                             unsigned long long tag) {
    static_assert(sizeof(FitSlotCore<K>) % 8 == 0, "8-byte words");
    static_assert(sizeof(FitSlotCore<K>) / 8 <= kExpressTagWord, "entry + tag");
    constexpr int W = (int)(sizeof(FitSlotCore<K>) / 8);
    const unsigned long long *s = reinterpret_cast<const unsigned long long *>(src);
    for (int w = lane; w < W; w += 64) st_agent(&dst[w], s[w]);
    if (lane == 0) st_agent(&dst[kExpressTagWord], tag);
}

// Express wave: up to XG long series at once, one per group of 64/XG lanes (XG from the row length: each group
// needs its state, its row and an exchange area in the wave's LDS share). Each group holds either a series or an
// outstanding ticket. Per iteration: groups poll their ticket's ring entry (non-blocking) and load what arrived;
// then one objective pass serves every group that wants F (lane l of a group evaluates chain l: the request's
// point, then its predicted points) and one gradient pass every group that wants G (lane l carries dEdTheta's
// column l); lane 0 of each group advances its state machine. A group whose ticket can no longer be filled
// (every bulk wave done and the fills below the ticket) retires; the wave exits when all its groups retired.
template <int K>
constexpr int express_group_bytes(int n) { return express_state_bytes<K>() + ((n + 1) & ~1) * 8 + 16 * 8; }

// Hand-off watchdog: a persistent kernel must never spin forever. A waiting group that sees none of the launch's
// progress counters move for kWatchdogTicks (100 MHz real-time counter) gives up, and a fitting group whose state
// posts no request without being finished is dropped; either records the first fault in ctl[26..31] (the host
// reports it as a device error) and the wave drains normally.
constexpr unsigned long long kWatchdogTicks = 2000000000ull;    // 20 s without any progress of the launch
enum : unsigned long long { FAULT_HANDOFF_STALL = 1, FAULT_NO_REQUEST = 2, FAULT_MERGE_STALL = 3 };

__device__ __forceinline__ void record_fault(unsigned long long *ctl, unsigned long long code, unsigned long long a,
                                             unsigned long long b, unsigned long long c, unsigned long long d,
                                             unsigned long long e) {
    if (cas_agent(&ctl[26], 0ull, code) == 0ull) {
        st_agent(&ctl[27], a);
        st_agent(&ctl[28], b);
        st_agent(&ctl[29], c);
        st_agent(&ctl[30], d);
        st_agent(&ctl[31], e);
    }
}


constexpr bool kPit = true;                  // express objective passes parallel in time (css_pit_lds)
constexpr int kPitGMaxK = 12;                // gradient passes parallel in time (in column chunks of 6) for K <= this

template <int P, int Q, int I, bool SMEAR, int PIT_BMAX = 16, bool PIT_G = true>
__device__ void fit_express(unsigned char *lds, int lds_bytes, const double *__restrict__ y, int64_t ld, int n,
                            double *__restrict__ coef_out, double *__restrict__ ll_out,
                            int32_t *__restrict__ status_out, int32_t *__restrict__ n_eval_out,
                            int32_t *__restrict__ n_grad_out, uint8_t *__restrict__ flags_out,
                            unsigned long long *__restrict__ ctl, unsigned char *__restrict__ xq,
                            unsigned *__restrict__ xready, int64_t N, int lane, int dd) {
    constexpr int K = I + P + Q;
    constexpr int NS = spec_ns<K>();
    const int gbytes = express_group_bytes<K>(n);
    int XG = lds_bytes / gbytes;
    XG = XG >= kExpressGroups ? kExpressGroups : (XG >= 2 ? 2 : 1);
    const int GL = 64 / XG;                                 // lanes per group
    const int grp = lane / GL, gl = lane % GL;
    const bool glead = gl == 0;
    unsigned char *gbase = lds + grp * gbytes;
    FitSlotCore<K> &ES = *reinterpret_cast<FitSlotCore<K> *>(gbase);
    double *row = reinterpret_cast<double *>(gbase + express_state_bytes<K>());
    double *xch = row + ((n + 1) & ~1);                     // K + NS + 1 doubles
    unsigned long long served = 0, pf = 0, pg = 0, evals = 0, grads = 0, hits = 0, done = 0, pf_pit = 0, pg_pit = 0,
                       pit_sw = 0;
    // group state: 0 = waiting on ticket, 1 = fitting, 2 = retired (wave-uniform per group after each shfl)
    int gstate = 0;
    unsigned long long ticket = 0;
    unsigned long long wd_sig = 0, wd_t = 0;                // watchdog (group leaders)
    unsigned wd_polls = 0;
    unsigned long long tk_time = 0, tk_polls = 0;          // fault diagnostics: this ticket's age and polls,
    unsigned tk_rfirst = 0, tk_rmax = 0;                    // first / largest ready word seen
    if (glead) {
        ticket = add_agent(&ctl[20], 1ull);
        tk_time = __builtin_amdgcn_s_memrealtime();
    }
    ticket = __shfl(ticket, grp * GL);
    const unsigned long long xring = express_ring_entries(ctl);
    for (;;) {
        // ---- groups waiting on a ticket: poll (group leader), then load the entry (whole group) ----
        int arrived = 0;
        if (gstate == 0 && glead) {
            const unsigned e = (unsigned)(ticket % xring);
            const unsigned long long *ent = reinterpret_cast<const unsigned long long *>(xq + (size_t)e * kExpressEntryBytes);
            // poll the ready word; every 32nd poll reads it at the memory side
            unsigned r = (tk_polls & 31u) == 31u ? rd_fresh(&xready[e]) : ld_agent(&xready[e]);
            if (tk_polls++ == 0) tk_rfirst = r;
            tk_rmax = r > tk_rmax ? r : tk_rmax;
            if (ticket >= xring) {
                arrived = 2;                                // beyond the ring: never filled
            } else if (r == (unsigned)(ticket + 1)) {
                arrived = rd_fresh(&ent[kExpressTagWord]) == ticket + 1 ? 1 : 0;
            } else {
                // every fill has happened once the work counter has run out and every bulk wave that started has
                // finished (a bulk wave starting later gets no series, so it cannot fill): no dependence on bulk
                // workgroups that are not resident yet, so concurrent launches cannot deadlock
                if (ld_agent(&ctl[0]) >= (unsigned long long)N) {
                    acquire_agent();
                    const unsigned long long bd = ld_agent(&ctl[22]);
                    const unsigned long long bs = ld_agent(&ctl[17]);
                    if (bd == bs) {
                        acquire_agent();
                        const unsigned long long fl = ld_agent(&ctl[21]);
                        r = rd_fresh(&xready[e]);
                        if (r == (unsigned)(ticket + 1)) arrived = rd_fresh(&ent[kExpressTagWord]) == ticket + 1 ? 1 : 0;
                        else arrived = ticket >= fl ? 2 : 0;
                    }
                }
            }
            if (arrived == 0 && (++wd_polls & 255u) == 0u) {
                const unsigned long long sig = ld_agent(&ctl[0]) + ld_agent(&ctl[17]) + ld_agent(&ctl[20]) +
                                               ld_agent(&ctl[21]) + ld_agent(&ctl[22]);
                const unsigned long long now = __builtin_amdgcn_s_memrealtime();
                if (sig != wd_sig || wd_t == 0) {
                    wd_sig = sig;
                    wd_t = now;
                } else if (now - wd_t > kWatchdogTicks) {
                    record_fault(ctl, FAULT_HANDOFF_STALL, ticket, ld_agent(&ctl[21]) | (ld_agent(&ctl[20]) << 32),
                                 tk_polls | (((now - tk_time) / 100000ull) << 32),
                                 (unsigned long long)tk_rmax | ((unsigned long long)tk_rfirst << 32),
                                 (unsigned long long)r | ((unsigned long long)e << 32));
                    arrived = 2;
                }
            }
            if (arrived == 1) acquire_agent();
        }
        arrived = __shfl(arrived, grp * GL);
        if (arrived == 2) gstate = 2;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (arrived == 1) {
            const unsigned e = (unsigned)(ticket % xring);
            const unsigned long long *src = reinterpret_cast<const unsigned long long *>(xq + (size_t)e * kExpressEntryBytes);
            constexpr int W = (int)(sizeof(FitSlotCore<K>) / 8);
            for (int w = gl; w < W; w += GL) reinterpret_cast<unsigned long long *>(&ES)[w] = rd_fresh(&src[w]);
        }
        wave_sync_lds();
        if (arrived == 1) {
            const double *srow = y + ES.sid * ld;
            for (int i = gl; i < n; i += GL) row[i] = drow_at(srow, dd, i);   // the differenced row (fused, dd = 1)
            gstate = 1;
            served += glead;
        }
        wave_sync_lds();
        if (__all(gstate == 2)) break;
        if (!__any(gstate == 1)) {                          // nothing to compute: back off
            __builtin_amdgcn_s_sleep(16);
            continue;
        }
        // ---- one pass for every group: the objective pass when all groups want F; otherwise the gradient pass,
        //      whose lanes in F groups evaluate their chain points (the pass also yields the objective) ----
        if (gstate == 1 && ES.s.req == REQ_NONE && !ES.s.done()) {     // invariant broken: drop, never spin
            if (glead)
                record_fault(ctl, FAULT_NO_REQUEST, ticket, (unsigned long long)ES.sid, ES.s.pc,
                             ((unsigned long long)ES.s.status << 16) | ES.s.n_eval, ld_agent(&ctl[21]));
            gstate = 2;
        }
        const int req = gstate == 1 ? (int)ES.s.req : REQ_NONE;
        const int nsp = req == REQ_F ? (int)ES.s.rq_nspec : 0;
        double c[K];
        if (req == REQ_F && gl >= 1 && gl <= nsp) ES.s.spec_point(gl - 1, c);
        else if (req != REQ_NONE) ES.s.request_point(c);
        else {
#pragma unroll
            for (int j = 0; j < K; ++j) c[j] = 0.0;
        }
        const double *prow = gstate == 1 ? row : reinterpret_cast<double *>(lds + express_state_bytes<K>());
        double cssv = 0.0, gj = 0.0;
        // one series on the whole wave: objective passes parallel in time (every lane evaluates every chain)
        constexpr int M = (P > Q ? P : Q);
        const bool pit = kPit && XG == 1 && req == REQ_F && n - M <= 64 * PIT_BMAX;
        if (pit) {
            double cm[NS + 1][K];
            ES.s.request_point(cm[0]);
#pragma unroll
            for (int h = 1; h <= NS; ++h) {
                if (h <= nsp) {
                    ES.s.spec_point(h - 1, cm[h]);
                } else {
#pragma unroll
                    for (int j = 0; j < K; ++j) cm[h][j] = cm[0][j];
                }
            }
            auto run = [&](auto NCHc, auto BMc) {
                constexpr int NCH = decltype(NCHc)::value, BM = decltype(BMc)::value;
                double cc[NCH][K], cs[NCH];
#pragma unroll
                for (int h = 0; h < NCH; ++h)
#pragma unroll
                    for (int j = 0; j < K; ++j) cc[h][j] = cm[h][j];
                int sw = 0;
                css_pit_lds<P, Q, I, NCH, BM>(prow, n, cc, cs, lane, &sw);
                pit_sw += glead ? (unsigned long long)sw : 0ull;
#pragma unroll
                for (int h = 0; h < NCH; ++h)
                    if (gl == h) cssv = cs[h];
            };
            auto by_b = [&](auto NCHc) {
                if (PIT_BMAX > 16 && n - M > 64 * 16) run(NCHc, IC<(PIT_BMAX > 16 ? PIT_BMAX : 16)>{});
                else run(NCHc, IC<16>{});
            };
            if constexpr (NS >= 2) {
                if (nsp >= 2) by_b(IC<3>{});
                else if (nsp == 1) by_b(IC<2>{});
                else by_b(IC<1>{});
            } else if constexpr (NS == 1) {
                if (nsp >= 1) by_b(IC<2>{});
                else by_b(IC<1>{});
            } else {
                by_b(IC<1>{});
            }
            pf_pit += glead;
        } else if (PIT_G && K <= kPitGMaxK && kPit && XG == 1 && req == REQ_G && n - M <= 64 * 16) {
            // the gradient pass parallel in time (every lane gets the whole gradient and css)
            double cg[K], gg[K], cs = 0.0;
            ES.s.request_point(cg);
            int sw = 0;
            if constexpr (K <= kPitGMaxK) grad_pit_lds<P, Q, I, SMEAR, 16>(prow, n, cg, cs, gg, lane, &sw);
            cssv = cs;
#pragma unroll
            for (int j = 0; j < K; ++j)
                if (gl == j) gj = gg[j];
            pg_pit += glead;
            pit_sw += glead ? (unsigned long long)sw : 0ull;
        } else if (__any(req == REQ_G)) {
            grad_column_lds<P, Q, I, SMEAR>(prow, n, c, gl < K ? gl : 0, cssv, gj);
        } else {
            cssv = css_row_lds<P, Q, I>(prow, n, c);
        }
        if (req == REQ_F && gl <= nsp) xch[gl] = css_to_loglik(cssv, n);
        if (req == REQ_G && gl < K) xch[gl] = gj;
        if (req == REQ_G && glead) xch[K] = css_to_loglik(cssv, n);
        wave_sync_lds();
        if (glead && req != REQ_NONE) {
            CGLane<K, NS, spec_nc<K>()> &L = ES.s;
            if (req == REQ_F) {
                for (int h = 1; h <= nsp && h <= NS; ++h) L.spec_store(h - 1, xch[h]);
                double g0[K];
#pragma unroll
                for (int j = 0; j < K; ++j) g0[j] = 0.0;
                L.req = REQ_NONE;
                L.advance(xch[0], g0);
                pf++;
            } else {
                double g[K];
#pragma unroll
                for (int j = 0; j < K; ++j) g[j] = xch[j];
                L.req = REQ_NONE;
                L.advance(xch[K], g);
                pg++;
            }
        }
        wave_sync_lds();
        // ---- finished series: write the result, take a new ticket ----
        const bool fin = gstate == 1 && ES.s.done();
        if (fin && glead) {
            double pt[K];
#pragma unroll
            for (int j = 0; j < K; ++j) pt[j] = ES.s.point[j];
            write_fit<K>(ES.sid, ES.s.status, pt, ES.s.prev_obj, ES.s.n_eval, ES.s.n_grad,
                         ES.s.status == ARIMA_ST_OK ? model_flags<P, Q, I>(pt) : (uint8_t)0, coef_out, ll_out,
                         status_out, n_eval_out, n_grad_out, flags_out, 2);
            timing_stamp<K>(ES, coef_out);
            evals += ES.s.n_eval;
            grads += ES.s.n_grad;
            hits += ES.s.spec_hits;
            done++;
            ticket = add_agent(&ctl[20], 1ull);
            tk_time = __builtin_amdgcn_s_memrealtime();
            tk_polls = 0;
            tk_rfirst = tk_rmax = 0;
        }
        if (fin) gstate = 0;
        ticket = __shfl(ticket, grp * GL);
        wave_sync_lds();
    }
    if (glead) {
        atomicAdd(&ctl[5], evals);
        atomicAdd(&ctl[6], grads);
        atomicAdd(&ctl[7], hits);
        atomicAdd(&ctl[32], done);
        atomicAdd(&ctl[23], served);
        atomicAdd(&ctl[24], pf);
        atomicAdd(&ctl[25], pg);
        atomicAdd(&ctl[33], pf_pit);
        atomicAdd(&ctl[34], pit_sw);
        atomicAdd(&ctl[35], pg_pit);
    }
}

template <int P, int Q, int I, bool SMEAR, int SPW>
__global__ __launch_bounds__(64 * kFitWaves) __attribute__((amdgpu_waves_per_eu(kFitWavesPerCU / 4, kFitWavesPerCU / 4))) void k_cg_fit(
    const double *__restrict__ y, int64_t ld, int n, int64_t N, const double *__restrict__ init,
    const int32_t *__restrict__ init_status, double *__restrict__ coef_out, double *__restrict__ ll_out,
    int32_t *__restrict__ status_out, int32_t *__restrict__ n_eval_out, int32_t *__restrict__ n_grad_out,
    uint8_t *__restrict__ flags_out, unsigned long long *__restrict__ ctl, unsigned char *__restrict__ xq,
    unsigned *__restrict__ xready, int n_bulk, int join_express, int dd) {
    // ctl[0] = work counter, ctl[1] = lane F passes, ctl[2] = lane G passes, ctl[3] = wave F passes (one chain),
    // ctl[4] = wave G passes, ctl[5] = objective evaluations, ctl[6] = gradient evaluations, ctl[7] = spec hits,
    // ctl[8] = wave F passes with speculative chains, ctl[9] = speculative chains evaluated,
    // ctl[17] = bulk waves started, ctl[18] = objective requests served by gradient passes, ctl[20] = express tickets, ctl[21] = express fills (donations),
    // ctl[22] = bulk waves finished,
    // ctl[23] = series finished on the express path, ctl[24] / ctl[25] = express F / G passes
    constexpr int K = I + P + Q;
    constexpr int NS = spec_ns<K>();
    constexpr int NJ = (SPW + 63) / 64;      // slot groups: lane l owns slots l, l + 64, ...
    static_assert(SPW >= (kFitWavesPerCU > 4 ? 32 : 64) && SPW <= 128, "slots per wave");
    static_assert(sizeof(FitSlotCore<K>) <= kExpressEntryBytes, "express ring entry");
    __shared__ FitSlot<K> slots[kFitWaves][SPW];
    __shared__ int assign[kFitWaves][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool has_express = n_bulk < (int)gridDim.x;
    if ((int)blockIdx.x >= n_bulk) {                      // express workgroup: this wave's share of the LDS
        fit_express<P, Q, I, SMEAR>(reinterpret_cast<unsigned char *>(&slots[wave][0]), (int)sizeof(slots[0]), y, ld,
                                    n, coef_out, ll_out, status_out, n_eval_out, n_grad_out, flags_out, ctl, xq,
                                    xready, N, lane, dd);
        return;
    }
    if (has_express && lane == 0) {                       // counted before this wave takes any series (release)
        add_agent(&ctl[17], 1ull);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // Drain merge (round 4; ctl[44] = merge_live > 0, set by the host): once the batch's work counter has run out,
    // a wave whose live slots dropped to merge_live or fewer hands them to the merge pool (the upper three quarters
    // of the express ring) and leaves; waves still running take pool entries into their free slots (up to 64 live). Few
    // waves then run nearly full passes instead of many nearly empty ones, and a leaving wave's SIMD (its whole
    // workgroup, once all four left) goes to the next fit sharing the GPU. ctl[40] = active waves (bits 0-23) |
    // entries reserved (bits 24-63), ctl[41] = entries claimed, ctl[42] = waves that handed over, ctl[43] = claims.
    // A wave reserves entries and leaves the active count in one CAS, and leaves without entries only by a CAS that
    // sees every reserved entry claimed -- so while entries are unclaimed some active wave remains to take them.
    // Only where a series is fitted changes, never its result.
    const int merge_live = (int)ctl[44];
    // objective-pass width model: per-step streaming cost of a pass in 1/16 chains (ctl[47], option "chain_overhead";
    // 0 = kChainOverhead16). A larger value prices bytes higher and so prefers wider passes (more chains per row read)
    const int chain_ovh = ctl[47] ? (int)ctl[47] : kChainOverhead16;
    unsigned char *mpool = xq + (size_t)(kExpressRing - kMergeCap) * kExpressEntryBytes;
    unsigned *mready = xready + (kExpressRing - kMergeCap);
    unsigned long long merge_head = 0;     // entries claimed, as last seen (a lower bound)
    if (merge_live > 0 && lane == 0) add_agent(&ctl[40], 1ull);
    // donation thresholds: ctl[45] / ctl[46] when the host set them (options "donate_evals" / "donate_evals_drained")
    const int don_evals = ctl[45] ? (int)ctl[45] : kDonateEvals;
    const int don_drained = ctl[46] ? (int)ctl[46] : kDonateEvalsDrained;
    FitSlot<K> *ws = slots[wave];
    const unsigned long long xring = express_ring_entries(ctl);
    unsigned long long lane_f = 0, lane_g = 0, wave_f = 0, wave_g = 0, wave_m = 0, evals = 0, grads = 0, hits = 0,
                       chains = 0, rides = 0, done = 0, wave_chains = 0, low_passes = 0;
    unsigned round_no = 0;
    bool drained = false;                  // the batch's work counter has run out (this wave saw it)
    const bool lane0 = lane == 0;
#ifdef STS_TIMING
    // diagnostics build only: shader-clock cycles per phase, summed over waves (ctl[10..13]), the kernel span
    // (ctl[14] = max end, ctl[15] = min start) and the per-wave time after the batch drained (ctl[16])
    unsigned long long tm_f = 0, tm_g = 0, tm_adv = 0, tm_sel = 0, tm_drain = 0, tm_step = 0, tm_refill = 0;
    const unsigned long long tm_start = __builtin_amdgcn_s_memtime();
    auto now = [] { return __builtin_amdgcn_s_memtime(); };
#endif

    // Give the slots of the lanes with need = true a new series (or mark them empty once the batch is drained).
    // Wave-uniform control flow: every lane calls it. Series whose Hannan-Rissanen init failed are reported
    // here and skipped.
    auto refill = [&](int slot, bool need) {
        for (;;) {
            const unsigned long long m = __ballot(need);
            if (m == 0ull) break;
            const int leader = __ffsll((long long)m) - 1;
            unsigned long long base = 0;
            if (lane == leader) base = add_agent(&ctl[0], (unsigned long long)__popcll(m));
            base = __shfl(base, leader);
            if (need) {
                const int rank = __popcll(m & ((1ull << lane) - 1ull));
                const int64_t sid = (int64_t)(base + (unsigned long long)rank);
                FitSlotCore<K> &S = ws[slot].c;
                if (sid >= N) {
                    drained = true;
#ifdef STS_TIMING
                    if (tm_drain == 0) tm_drain = __builtin_amdgcn_s_memtime();
#endif
                    S.sid = -1;
                    S.s.req = REQ_NONE;
                    need = false;
                } else {
                    const int st0 = init_status ? init_status[sid] : ARIMA_ST_OK;
                    if (st0 != ARIMA_ST_OK) {
                        double nanc[K];
#pragma unroll
                        for (int j = 0; j < K; ++j) nanc[j] = __builtin_nan("");
                        write_fit<K>(sid, st0, nanc, 0.0, 0, 0, 0, coef_out, ll_out, status_out, n_eval_out,
                                     n_grad_out, flags_out);
                        done++;
                    } else {
                        double x0[K];
#pragma unroll
                        for (int j = 0; j < K; ++j) x0[j] = init[sid * K + j];
                        S.sid = sid;
#ifdef STS_TIMING
                        S.t_start = (double)__builtin_amdgcn_s_memrealtime();
                        S.t_donate = 0.0;
#endif
                        S.s.start_posted(x0);           // posts the first request: G at the initial point
                        need = false;
                    }
                }
            }
        }
    };

#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int slot = lane + 64 * j;
        refill(slot < SPW ? slot : 0, slot < SPW);
    }

    for (;;) {
#ifdef STS_TIMING
        const unsigned long long t_a = now();
#endif
        // ---- pick the pass: all-G or all-F, up to 64 slots ----
        // Long-running series (>= kOldEvals evaluations) set the critical path of the launch, so their requests
        // choose the pass type and are served first; the other slots are taken in a rotating order (no slot
        // starves while more than 64 requests of its type are pending).
        unsigned long long mF[NJ], mG[NJ], mO[NJ], mP1[NJ], mP2[NJ];
        int nF = 0, nG = 0, nOF = 0, nOG = 0, nP1 = 0, nP2 = 0;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int slot = lane + 64 * j;
            int r = REQ_NONE, nsp_j = 0;
            bool old = false;
            if (slot < SPW && ws[slot].c.sid >= 0) {
                r = ws[slot].c.s.req;
                old = ws[slot].c.s.n_eval >= kOldEvals;
                nsp_j = ws[slot].c.s.rq_nspec;
            }
            mF[j] = __ballot(r == REQ_F);
            mG[j] = __ballot(r == REQ_G);
            mO[j] = __ballot(old);
            mP1[j] = __ballot(r == REQ_F && nsp_j >= 1);
            mP2[j] = __ballot(r == REQ_F && nsp_j >= 2);
            nF += __popcll(mF[j]);
            nG += __popcll(mG[j]);
            nOF += __popcll(mF[j] & mO[j]);
            nOG += __popcll(mG[j] & mO[j]);
            nP1 += __popcll(mP1[j]);
            nP2 += __popcll(mP2[j]);
        }
        if (merge_live > 0 && __any(drained)) {
            const int live = nF + nG;
            int occ = 0;                          // occupied slots (live ones, with a request posted, in practice)
#pragma unroll
            for (int j = 0; j < NJ; ++j) occ += __popcll(__ballot(lane + 64 * j < SPW && ws[lane + 64 * j].c.sid >= 0));
            constexpr int kRoom = SPW < 64 ? SPW : 64;
            int act = 0;                          // 1 = handed over, 2 = claimed entries, 3 = left (pool empty)
            unsigned long long mbase = 0, mcnt = 0;
            if (lane0) {
                unsigned long long w = rd_fresh(&ctl[40]);
                bool offer = live > 0 && live <= merge_live;
                for (;;) {
                    const unsigned long long active = w & 0xffffffull, tail = w >> 24;
                    if (offer) {
                        if (active > 1 && tail + (unsigned long long)live <= (unsigned long long)kMergeCap) {
                            const unsigned long long o = cas_agent(&ctl[40], w, ((tail + live) << 24) | (active - 1));
                            if (o == w) {
                                act = 1;
                                mbase = tail;
                                break;
                            }
                            w = o;
                            continue;
                        }
                        offer = false;            // nobody left to take them, or the pool is full: keep fitting
                    }
                    if (occ < kRoom && tail > merge_head) {
                        unsigned long long head = rd_fresh(&ctl[41]);
                        while (head < tail) {
                            const unsigned long long c = tail - head < (unsigned long long)(kRoom - occ)
                                                             ? tail - head : (unsigned long long)(kRoom - occ);
                            const unsigned long long o = cas_agent(&ctl[41], head, head + c);
                            if (o == head) {
                                act = 2;
                                mbase = head;
                                mcnt = c;
                                break;
                            }
                            head = o;
                        }
                        merge_head = act == 2 ? mbase + mcnt : head;
                        if (act == 2) break;
                    }
                    if (live > 0) break;
                    // nothing live and every reserved entry claimed: leave (fails if an entry was reserved meanwhile)
                    const unsigned long long o = cas_agent(&ctl[40], w, w - 1ull);
                    if (o == w) {
                        act = 3;
                        break;
                    }
                    w = o;
                }
            }
            act = __shfl(act, 0);
            if (act == 1) {                       // every live slot into entries mbase.. in slot order
                mbase = __shfl(mbase, 0);
                int rk = 0;
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const unsigned long long m = mF[j] | mG[j];
                    const int slot = lane + 64 * j;
                    if ((m >> lane) & 1ull) {
                        const unsigned long long e = mbase + (unsigned long long)(rk + __popcll(m & ((1ull << lane) - 1ull)));
                        constexpr int W = (int)(sizeof(FitSlotCore<K>) / 8);
                        unsigned long long *dst = reinterpret_cast<unsigned long long *>(mpool + (size_t)e * kExpressEntryBytes);
                        const unsigned long long *src = reinterpret_cast<const unsigned long long *>(&ws[slot].c);
                        for (int w = 0; w < W; ++w) st_agent(&dst[w], src[w]);
                        st_agent(&dst[kExpressTagWord], e + 1ull);
                    }
                    rk += __popcll(m);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the entries before their ready words
                rk = 0;
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const unsigned long long m = mF[j] | mG[j];
                    const int slot = lane + 64 * j;
                    if ((m >> lane) & 1ull) {
                        const unsigned long long e = mbase + (unsigned long long)(rk + __popcll(m & ((1ull << lane) - 1ull)));
                        st_agent(&mready[e], (unsigned)(e + 1ull));
                        ws[slot].c.sid = -1;
                        ws[slot].c.s.req = REQ_NONE;
                    }
                    rk += __popcll(m);
                }
                if (lane0) add_agent(&ctl[42], 1ull);
                break;
            }
            if (act == 3) break;
            if (act == 2) {                       // entries mbase .. mbase + mcnt - 1 into the free slots, in order
                mbase = __shfl(mbase, 0);
                mcnt = __shfl(mcnt, 0);
                int rk = 0;
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int slot = lane + 64 * j;
                    const bool fr = slot < SPW && ws[slot].c.sid < 0;
                    const unsigned long long m = __ballot(fr);
                    const int r = rk + __popcll(m & ((1ull << lane) - 1ull));
                    if (fr && (unsigned long long)r < mcnt) {
                        const unsigned long long e = mbase + (unsigned long long)r;
                        const unsigned long long *src =
                            reinterpret_cast<const unsigned long long *>(mpool + (size_t)e * kExpressEntryBytes);
                        unsigned long long t0 = 0;
                        bool ok = true;
                        while (!(rd_fresh(&mready[e]) == (unsigned)(e + 1ull) && rd_fresh(&src[kExpressTagWord]) == e + 1ull)) {
                            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
                            if (t0 == 0) {
                                t0 = t;
                            } else if (t - t0 > kWatchdogTicks) {   // never spin forever: the series is reported lost
                                record_fault(ctl, FAULT_MERGE_STALL, e, ld_agent(&ctl[40]), ld_agent(&ctl[41]), 0, 0);
                                ok = false;
                                break;
                            }
                            __builtin_amdgcn_s_sleep(2);
                        }
                        if (ok) {
                            constexpr int W = (int)(sizeof(FitSlotCore<K>) / 8);
                            unsigned long long *dst = reinterpret_cast<unsigned long long *>(&ws[slot].c);
                            for (int w = 0; w < W; ++w) dst[w] = rd_fresh(&src[w]);
                        }
                    }
                    rk += __popcll(m);
                }
                if (lane0) add_agent(&ctl[43], 1ull);
                wave_sync_lds();
                continue;
            }
        }
        if (nF + nG == 0) break;                  // batch drained and every slot of this wave finished
        // (round 3: a cost-aware choice -- G when min(64, nG + nF) per gradient-pass cost beats min(64, nF) per
        // objective-pass cost -- measured at weights 2-4: C2 and C4 unchanged within noise, profiles/r03/o_gw)
        const bool doG = nOG != nOF ? nOG > nOF : (nG >= 64 || (nF < 64 && nG >= nF));
        // Objective pass width (round 4): an objective pass runs NCH chains on every lane, so a lane whose request
        // carries fewer predictions than NCH - 1 pays for chains it does not use. Choose NCH for the most objective
        // evaluations per unit of pass cost (cost ~ NCH + the per-step streaming share, kChainOverhead16 / 16 of a
        // chain), serving up to 64 requests, those that use all NCH chains first. Requests whose extra predictions
        // do not fit are served without them (a prediction only fills the value cache; results are unchanged).
        int nchc = NS + 1;
        if (kNchChoice && !doG) {
            const int n2 = nP2, n1 = nP1 - nP2, n0 = nF - nP1;
            int best = -1;
#pragma unroll
            for (int c = 1; c <= NS + 1; ++c) {
                int left = 64, u = 0, t;
                t = n2 < left ? n2 : left; u += t * (c < 3 ? c : 3); left -= t;
                t = n1 < left ? n1 : left; u += t * (c < 2 ? c : 2); left -= t;
                t = n0 < left ? n0 : left; u += t; left -= t;
                const int score = u * 4096 / (chain_ovh + 16 * c);
                if (score >= best) { best = score; nchc = c; }
            }
        }
        const int rot = (int)(round_no * 37u) & 63;
        round_no++;
        // A gradient pass also yields the objective, so its lanes left over after the G requests serve objective
        // requests (tiers 2-3: the request's own point; its predicted points wait for an objective pass). An
        // objective pass serves long-running requests first, then those that use all nchc chains, then the rest.
        int base = 0;
#pragma unroll
        for (int tier = 0; tier < 4; ++tier) {
            if (tier >= 2 && ((doG && !kFRide) || (!doG && !kNchChoice) || base >= 64)) break;
            if (tier == 3 && !doG) break;
#pragma unroll
            for (int jj = 0; jj < NJ; ++jj) {
                const int j = (jj + (int)round_no) % NJ;
                // select the slot group's masks without a dynamically indexed register array (that would live in
                // scratch memory: 4 scratch loads per pass selection)
                unsigned long long wG = mG[0], wF = mF[0], wO = mO[0], wP1 = mP1[0], wP2 = mP2[0];
#pragma unroll
                for (int i = 1; i < NJ; ++i) {
                    wG = (j == i) ? mG[i] : wG;
                    wF = (j == i) ? mF[i] : wF;
                    wO = (j == i) ? mO[i] : wO;
                    wP1 = (j == i) ? mP1[i] : wP1;
                    wP2 = (j == i) ? mP2[i] : wP2;
                }
                unsigned long long m;
                if (doG) {
                    m = (tier < 2 ? wG : wF) & ((tier & 1) == 0 ? wO : ~wO);
                } else if (!kNchChoice) {
                    m = wF & (tier == 0 ? wO : ~wO);
                } else {
                    const unsigned long long full = nchc >= 3 ? wP2 : (nchc == 2 ? wP1 : ~0ull);
                    m = wF & (tier == 0 ? wO : (tier == 1 ? (~wO & full) : (~wO & ~full)));
                }
                m = (m >> rot) | (rot ? (m << (64 - rot)) : 0ull);          // rotate: lane rot ranks first
                const int lr = (lane - rot) & 63;
                if ((m >> lr) & 1ull) {
                    const int rank = base + __popcll(m & ((1ull << lr) - 1ull));
                    if (rank < 64) assign[wave][rank] = lane + 64 * j;
                }
                base += __popcll(m);
            }
        }
        const int nsel = base < 64 ? base : 64;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const bool served = lane < nsel;
        const int my = served ? assign[wave][lane] : 0;
        FitSlotCore<K> &S = ws[my].c;
        // lanes without a slot stream a shared (L2-resident) row with dummy coefficients: uniform control flow
        const double *row = served ? y + S.sid * ld : y;
        double c[K], css, g[K];
        if (served) {
            S.s.request_point(c);
        } else {
#pragma unroll
            for (int j = 0; j < K; ++j) c[j] = 0.0;
        }
        double resp_f = 0.0;
#ifdef STS_TIMING
        const unsigned long long t_b = now();
        tm_sel += t_b - t_a;
#endif
        if (doG) {
            css_pass<P, Q, I, true, SMEAR, true>(row, n, c, css, g, dd);
            resp_f = css_to_loglik(css, n);
            wave_g += lane0;
            lane_g += served;
            rides += (served && S.s.req == REQ_F) ? 1ull : 0ull;
        } else {
            // chains = 1 + the most predictions any served lane posted, at most the chosen width (wave-uniform);
            // a lane evaluates its first nch - 1 predictions
            int nsp = served ? (int)S.s.rq_nspec : 0;
            nsp = nsp < nchc - 1 ? nsp : nchc - 1;
            int nch = 1;
#pragma unroll
            for (int h = 1; h <= NS; ++h)
                if (__ballot(nsp >= h) != 0ull) nch = h + 1;
            auto multi = [&](auto NCHc) {
                constexpr int NCH = decltype(NCHc)::value;
                double cm[NCH][K], cssm[NCH];
#pragma unroll
                for (int j = 0; j < K; ++j) cm[0][j] = c[j];
#pragma unroll
                for (int h = 1; h < NCH; ++h) {
                    if (h <= nsp) {
                        double cs[K];
                        S.s.spec_point(h - 1, cs);
#pragma unroll
                        for (int j = 0; j < K; ++j) cm[h][j] = cs[j];
                    } else {
#pragma unroll
                        for (int j = 0; j < K; ++j) cm[h][j] = c[j];
                    }
                }
                css_pass_multi<P, Q, I, NCH>(row, n, cm, cssm, dd);
                css = cssm[0];
                if (served) {
#pragma unroll
                    for (int h = 1; h < NCH; ++h)
                        if (h <= nsp) S.s.spec_store(h - 1, css_to_loglik(cssm[h], n));
                }
            };
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
            resp_f = css_to_loglik(css, n);
            if (nch > 1) wave_m += lane0; else wave_f += lane0;
            lane_f += served;
            chains += served ? (unsigned long long)(1 + nsp) : 0ull;
            wave_chains += lane0 ? (unsigned long long)(64 * nch) : 0ull;
        }
        low_passes += (lane0 && nsel < 32) ? 1ull : 0ull;
        // ---- each lane advances its slot with the response; finished slots are written out and refilled ----
#ifdef STS_TIMING
        const unsigned long long t_c = now();
        if (doG) tm_g += t_c - t_b; else tm_f += t_c - t_b;
#endif
        bool need = false;
        if (served) {
            CGLane<K, NS, spec_nc<K>()> &L = S.s;
            L.req = REQ_NONE;
            L.advance(resp_f, g);
            if (L.done()) {
                double pt[K];
#pragma unroll
                for (int j = 0; j < K; ++j) pt[j] = L.point[j];
                write_fit<K>(S.sid, L.status, pt, L.prev_obj, L.n_eval, L.n_grad,
                             L.status == ARIMA_ST_OK ? model_flags<P, Q, I>(pt) : (uint8_t)0, coef_out, ll_out,
                             status_out, n_eval_out, n_grad_out, flags_out);
                timing_stamp<K>(S, coef_out);
                evals += L.n_eval;
                grads += L.n_grad;
                hits += L.spec_hits;
                done++;
                need = true;
            }
        }
#ifdef STS_TIMING
        const unsigned long long t_s = now();
        tm_step += t_s - t_c;
#endif
        refill(my, need);
#ifdef STS_TIMING
        tm_refill += now() - t_s;
#endif
        if (has_express) {
            // an express wave is waiting: hand it this wave's oldest slot (the likely critical path)
            unsigned long long wants = 0, filled = 0, fault = 0;
            if (lane0) {
                wants = ld_agent(&ctl[20]);
                filled = ld_agent(&ctl[21]);
                fault = ld_agent(&ctl[26]);
            }
            wants = __shfl(wants, 0);
            filled = __shfl(filled, 0);
            fault = __shfl(fault, 0);
            // no donation once a fault is recorded (a retired ticket holder would never write it back)
            if (wants > filled && filled < xring && fault == 0) {
                const int donate_min = __any(drained) ? don_drained : don_evals;
                unsigned long long key = 0;
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int slot = lane + 64 * j;
                    if (slot < SPW && ws[slot].c.sid >= 0 && ws[slot].c.s.req != REQ_NONE &&
                        ws[slot].c.s.n_eval >= donate_min) {
                        const unsigned long long kk = ((unsigned long long)ws[slot].c.s.n_eval << 16) | (unsigned)(slot + 1);
                        key = kk > key ? kk : key;
                    }
                }
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
                    const unsigned long long o = __shfl_xor(key, off);
                    key = o > key ? o : key;
                }
                // claim a fill index that a waiting ticket will read: never beyond the tickets (an unbounded
                // fill could overwrite a ring entry before its ticket holder has read it)
                unsigned long long jx = 0;
                int claimed = 0;
                if (lane0 && key) {
                    unsigned long long f = filled;
                    while (f < wants && f < xring) {
                        const unsigned long long prev = cas_agent(&ctl[21], f, f + 1ull);
                        if (prev == f) {
                            jx = f;
                            claimed = 1;
                            break;
                        }
                        f = prev;
                        wants = ld_agent(&ctl[20]);
                    }
                }
                claimed = __shfl(claimed, 0);
                jx = __shfl(jx, 0);
                if (claimed) {
                    const int bs = (int)(key & 0xffffull) - 1;
                    const unsigned e = (unsigned)(jx % xring);
#ifdef STS_TIMING
                    if (lane == (bs & 63)) ws[bs].c.t_donate = (double)__builtin_amdgcn_s_memrealtime();
                    wave_sync_lds();
#endif
                    publish_core<K>(reinterpret_cast<unsigned long long *>(xq + (size_t)e * kExpressEntryBytes), &ws[bs].c,
                                    lane, jx + 1);
                    // the entry went out write-through (sc1): drain this wave's stores, then the flag (no L2
                    // write-back needed; cdna_hip_programming.md Guideline 16, R1)
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (lane0) st_agent(&xready[e], (unsigned)(jx + 1));
                    if (lane == (bs & 63)) {
                        ws[bs].c.sid = -1;
                        ws[bs].c.s.req = REQ_NONE;
                    }
                    wave_sync_lds();
                    refill(bs, lane == (bs & 63));
                }
            }
        }
#ifdef STS_TIMING
        tm_adv += now() - t_c;
#endif
    }
    if (has_express) {
        if (lane0) {                                        // this bulk wave will fill no more express entries
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            add_agent(&ctl[22], 1ull);
        }
        // its slots are all finished: unless the launch shares the GPU with other fits (join_express = 0: the
        // workgroup should exit and make room), the wave serves the remaining long series on the express path,
        // in the LDS share its slots used
        if (join_express) {
            wave_sync_lds();
            fit_express<P, Q, I, SMEAR>(reinterpret_cast<unsigned char *>(&slots[wave][0]), (int)sizeof(slots[0]), y,
                                        ld, n, coef_out, ll_out, status_out, n_eval_out, n_grad_out, flags_out, ctl,
                                        xq, xready, N, lane, dd);
        }
    }
#ifdef STS_TIMING
    if (lane0) {
        const unsigned long long tm_end = now();
        atomicAdd(&ctl[10], tm_f);
        atomicAdd(&ctl[11], tm_g);
        atomicAdd(&ctl[12], tm_adv);
        atomicAdd(&ctl[13], tm_sel);
        atomicMax(&ctl[14], tm_end);
        atomicMin(&ctl[15], tm_start);
        atomicAdd(&ctl[16], tm_drain ? tm_end - tm_drain : 0ull);
        atomicAdd(&ctl[38], tm_step);              // (part of tm_adv) the served slots' optimizer steps
        atomicAdd(&ctl[39], tm_refill);            // (part of tm_adv) refills from the work counter
    }
#endif
    atomicAdd(&ctl[1], lane_f);
    atomicAdd(&ctl[2], lane_g);
    if (lane0) {
        atomicAdd(&ctl[3], wave_f);
        atomicAdd(&ctl[4], wave_g);
        atomicAdd(&ctl[8], wave_m);
    }
    atomicAdd(&ctl[5], evals);
    atomicAdd(&ctl[6], grads);
    atomicAdd(&ctl[7], hits);
    atomicAdd(&ctl[9], chains);
    atomicAdd(&ctl[18], rides);
    atomicAdd(&ctl[32], done);
    if (lane0) {
        atomicAdd(&ctl[36], wave_chains);       // chains the objective passes computed (64 lanes x NCH each)
        atomicAdd(&ctl[37], low_passes);        // wave passes that served fewer than 32 lanes
    }
}

}  // namespace sts

namespace sts {

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
#ifdef STS_DEV
// dev build (make dev): only q = STS_DEV_Q and the default Breeze reading (smear) -- fast kernel experiments
template <class Fn>
int with_order(int v, Fn &&fn) {
    return v == STS_DEV_Q ? fn(IC<STS_DEV_Q>{}) : ARIMA_E_UNSUPPORTED;
}
template <class Fn>
int with_smear(int v, Fn &&fn) {
    return v ? fn(IC<1>{}) : ARIMA_E_UNSUPPORTED;
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

// one fusion variant of k_hr_init for AR order P (instantiated per (P, F) in arima_hr_p<P>_f<F>.hip: the build runs them
// in parallel)
template <int P, bool F>
int launch_hr_init_PF(const double *y, int64_t ld, int n, int64_t N, int q, int I, double *init_out,
                      int32_t *status_out, hipStream_t s, int hr_grid, int dd, const FitPrep &prep) {
    return with_order(q, [&](auto Qc) {
        return with_bool(I, [&](auto Ic) {
            constexpr int Q = decltype(Qc)::value, II = decltype(Ic)::value;
            const int block = hr_grid > 0 ? 64 : 256;
            const unsigned grid =
                hr_grid > 0 ? std::min<unsigned>(grid_for(N, 64), (unsigned)hr_grid) : grid_for(N, 256);
            hipLaunchKernelGGL((k_hr_init<P, Q, II, F>), dim3(grid), dim3(block), 0, s, y, ld, n, N, init_out,
                               status_out, F ? dd : 0, prep);
            STS_CHECK_LAUNCH();
            return ARIMA_OK;
        });
    });
}

template <int P>
int launch_hr_init_P(const double *y, int64_t ld, int n, int64_t N, int q, int I, double *init_out,
                     int32_t *status_out, hipStream_t s, int hr_grid, int dd, const FitPrep &prep) {
    return dd ? launch_hr_init_PF<P, true>(y, ld, n, N, q, I, init_out, status_out, s, hr_grid, dd, prep)
              : launch_hr_init_PF<P, false>(y, ld, n, N, q, I, init_out, status_out, s, hr_grid, 0, prep);
}

template <int P>
int launch_ar_fit_P(const double *y, int64_t ld, int n, int64_t N, int I, double *coef_out, double *ll_out,
                    int32_t *status_out, int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out,
                    hipStream_t s, int dd) {
    if constexpr (P == 0) {
        return ARIMA_E_INVALID_ARG;
    } else {
        return with_bool(I, [&](auto Ic) {
            constexpr int II = decltype(Ic)::value;
            hipLaunchKernelGGL((k_ar_fit<P, II>), dim3(grid_for(N, 256)), dim3(256), 0, s, y, ld, n, N, coef_out,
                               ll_out, status_out, n_eval_out, n_grad_out, flags_out, dd);
            STS_CHECK_LAUNCH();
            return ARIMA_OK;
        });
    }
}

// k_cg_fit launcher for one AR order and Breeze reading (each instantiated in its own translation unit,
// arima_cg_p<P>_s<S>.hip, so the build parallelises over the heaviest kernel).
template <int P, bool S>
int launch_cg_fit_PS(const double *y, int64_t ld, int n, int64_t N, int q, int I, const double *init,
                     const int32_t *init_status, double *coef_out, double *ll_out, int32_t *status_out,
                     int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out, unsigned long long *ctl,
                     int grid_blocks, int express_blocks, unsigned char *xq, unsigned *xready, int join_express,
                     hipStream_t s, int dd) {
    return with_order(q, [&](auto Qc) {
        return with_bool(I, [&](auto Ic) {
            constexpr int Q = decltype(Qc)::value, II = decltype(Ic)::value;
            constexpr int K = P + Q + II;
            if constexpr (K == 0) {
                return ARIMA_E_INVALID_ARG;
            } else {
                constexpr int SPW = fit_slots_per_wave<K>();
                // express blocks only when the row fits next to the state in one wave's LDS share
                const int lds_per_wave = SPW * (int)sizeof(FitSlot<K>);
                if (n > express_max_n<K>(lds_per_wave)) express_blocks = 0;
                hipLaunchKernelGGL((k_cg_fit<P, Q, II, S, SPW>), dim3(grid_blocks + express_blocks),
                                   dim3(64 * kFitWaves), 0, s, y, ld, n, N, init, init_status, coef_out, ll_out,
                                   status_out, n_eval_out, n_grad_out, flags_out, ctl, xq, xready, grid_blocks,
                                   join_express, dd);
                STS_CHECK_LAUNCH();
                return ARIMA_OK;
            }
        });
    });
}

template <int P>
int launch_cg_fit_P(const double *y, int64_t ld, int n, int64_t N, int q, int I, int smear, const double *init,
                    const int32_t *init_status, double *coef_out, double *ll_out, int32_t *status_out,
                    int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out, unsigned long long *ctl,
                    int grid_blocks, int express_blocks, unsigned char *xq, unsigned *xready, int join_express,
                    hipStream_t s, int dd) {
    return with_smear(smear, [&](auto Sc) {
        return launch_cg_fit_PS<P, (decltype(Sc)::value != 0)>(y, ld, n, N, q, I, init, init_status, coef_out, ll_out,
                                                               status_out, n_eval_out, n_grad_out, flags_out, ctl,
                                                               grid_blocks, express_blocks, xq, xready, join_express,
                                                               s, dd);
    });
}

// series one workgroup keeps in flight (blocks of the grid are sized from it)
template <int P>
int cg_fit_series_per_block_P(int q, int I) {
    return with_order(q, [&](auto Qc) {
        return with_bool(I, [&](auto Ic) {
            constexpr int Q = decltype(Qc)::value, II = decltype(Ic)::value;
            if constexpr (P + Q + II == 0) return 0;
            else return kFitWaves * fit_slots_per_wave<P + Q + II>();
        });
    });
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

#define STS_DECLARE_CG(PP, SS, EXT)                                                                             \
    EXT template int launch_cg_fit_PS<PP, SS>(const double *, int64_t, int, int64_t, int, int, const double *,    \
                                              const int32_t *, double *, double *, int32_t *, int32_t *,        \
                                              int32_t *, uint8_t *, unsigned long long *, int, int,             \
                                              unsigned char *, unsigned *, int, hipStream_t, int);

#define STS_DECLARE_HR(PP, FF, EXT)                                                                             \
    EXT template int launch_hr_init_PF<PP, FF>(const double *, int64_t, int, int64_t, int, int, double *,         \
                                               int32_t *, hipStream_t, int, int, const FitPrep &);

#define STS_DECLARE_P(PP, EXT)                                                                                  \
    STS_DECLARE_CG(PP, false, extern)                                                                           \
    STS_DECLARE_CG(PP, true, extern)                                                                            \
    STS_DECLARE_HR(PP, false, extern)                                                                           \
    STS_DECLARE_HR(PP, true, extern)                                                                            \
    EXT template int launch_hr_init_P<PP>(const double *, int64_t, int, int64_t, int, int, double *, int32_t *,  \
                                          hipStream_t, int, int, const FitPrep &);                              \
    EXT template int launch_ar_fit_P<PP>(const double *, int64_t, int, int64_t, int, double *, double *,         \
                                         int32_t *, int32_t *, int32_t *, uint8_t *, hipStream_t, int);         \
    EXT template int launch_cg_fit_P<PP>(const double *, int64_t, int, int64_t, int, int, int, const double *,   \
                                         const int32_t *, double *, double *, int32_t *, int32_t *, int32_t *,  \
                                         uint8_t *, unsigned long long *, int, int, unsigned char *, unsigned *, \
                                         int, hipStream_t, int);                                                \
    EXT template int cg_fit_series_per_block_P<PP>(int, int);                                                   \
    EXT template int launch_css_loglik_P<PP>(const double *, int64_t, int, int64_t, int, int, const double *,    \
                                             double *, hipStream_t);                                            \
    EXT template int launch_css_grad_P<PP>(const double *, int64_t, int, int64_t, int, int, int, const double *, \
                                           double *, hipStream_t);                                              \
    EXT template int launch_model_flags_P<PP>(const double *, int64_t, int, int, uint8_t *, hipStream_t);

}  // namespace sts
