#pragma once
// arima_fit_global.hpp — k_cg_fit_g: the persistent CSS-CGD fit kernel with its optimizer slots in HBM/L2
// (included by arima_kernels_impl.hpp after k_cg_fit, whose pass selection, speculation, refill and express hand-off
// it follows; DESIGN.md 4 "two waves per SIMD").
//
// Why: the CSS recursion is a chain of dependent fp64 ops (e_t needs e_{t-1} through mul -> add -> add -> sub, each
// rounded as the reference rounds it) and a dependent fp64 op on gfx950 waits ~20 cycles at one wave per SIMD
// (tools/ubench_fp64.hip: 20.0 cycles per wave-instruction for one chain, 10.75 SIMD-cycles with two waves,
// profiles/r03/c_pmc_c2/ubench_fp64.txt). k_cg_fit keeps ~104 optimizer slots per wave in LDS (376 B each), which
// pins it to one wave per SIMD; giving those slots less LDS costs lane utilisation (48 slots: 0.44 vs 0.68).
//
// Here a slot is a 384-B record in global memory (this wave's SPW records, L2/MALL-resident), and LDS keeps only a
// directory per slot (posted request type, evaluation count, series id) for the pass selection. A served lane reads
// its slot's request point before the pass, then copies the whole record into registers, advances the state
// machine there (CGLane::step, force-inlined) and writes it back: ~0.8 KB of extra traffic per lane-pass against the
// 8 KB row it streams. With <= 256 VGPRs and ~20 KB of LDS per wave, two waves share every SIMD.
#include "arima_device.hpp"

namespace sts {

#ifndef STS_FITG_SLOTS
#define STS_FITG_SLOTS 128
#endif
#ifndef STS_FITG_PREFETCH_F
#define STS_FITG_PREFETCH_F 2
#endif
#ifndef STS_FITG_PREFETCH_G
#define STS_FITG_PREFETCH_G 2
#endif
constexpr int kFitGWavesPerCU = 8;                   // two single-wave workgroups per SIMD
constexpr int kFitGSlots = STS_FITG_SLOTS;           // optimizer slots per wave (records in global memory)
constexpr int kFitGPrefetchF = STS_FITG_PREFETCH_F;  // chunks in flight per lane: the partner wave hides the rest
constexpr int kFitGPrefetchG = STS_FITG_PREFETCH_G;
constexpr int kFitGExpressLds = 18 * 1024;           // LDS of one wave for the express path (state + row)
constexpr int kFitGDirEmpty = 0xff;                  // directory: slot without a series

template <int K>
struct alignas(128) GSlot {
    FitSlotCore<K> c;
};

template <int K>
constexpr int fitg_slot_bytes() { return (int)sizeof(GSlot<K>); }
static_assert(kFitGSlots == kFitGSlotsPerWave, "arima_launch.hpp sizes the slot records from kFitGSlotsPerWave");

template <int P, int Q, int I, bool SMEAR, int SPW>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_cg_fit_g(
    const double *__restrict__ y, int64_t ld, int n, int64_t N, const double *__restrict__ init,
    const int32_t *__restrict__ init_status, double *__restrict__ coef_out, double *__restrict__ ll_out,
    int32_t *__restrict__ status_out, int32_t *__restrict__ n_eval_out, int32_t *__restrict__ n_grad_out,
    uint8_t *__restrict__ flags_out, unsigned long long *__restrict__ ctl, unsigned char *__restrict__ xq,
    unsigned *__restrict__ xready, int n_bulk, int join_express, unsigned char *__restrict__ slot_mem) {
    // ctl[] as k_cg_fit
    constexpr int K = I + P + Q;
    constexpr int NS = spec_ns<K>();
    constexpr int NJ = (SPW + 63) / 64;
    using Lane = CGLane<K, NS, spec_nc<K>()>;
    static_assert(SPW % 8 == 0 && SPW >= 64 && SPW <= 256, "slots per wave");
    static_assert(sizeof(FitSlotCore<K>) <= kExpressEntryBytes, "express ring entry");
    __shared__ uint8_t dreq[SPW];                 // posted request (REQ_F / REQ_G), REQ_NONE while advancing,
                                                  // kFitGDirEmpty: no series
    __shared__ uint16_t dnev[SPW];                // evaluations so far (priority, donation)
    __shared__ int64_t dsid[SPW];                 // series of the slot
    __shared__ int assign[64];
    __shared__ __attribute__((aligned(16))) unsigned char xlds[kFitGExpressLds];
    const int lane = threadIdx.x & 63;
    const bool lane0 = lane == 0;
    const bool has_express = n_bulk < (int)gridDim.x;
    if ((int)blockIdx.x >= n_bulk) {
        fit_express<P, Q, I, SMEAR>(xlds, (int)sizeof(xlds), y, ld, n, coef_out, ll_out, status_out, n_eval_out,
                                    n_grad_out, flags_out, ctl, xq, xready, N, lane);
        return;
    }
    if (has_express && lane0) {
        add_agent(&ctl[17], 1ull);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    static_assert(sizeof(GSlot<K>) <= kFitGSlotBytes, "slot record");
    GSlot<K> *gs = reinterpret_cast<GSlot<K> *>(slot_mem + (size_t)blockIdx.x * SPW * kFitGSlotBytes);
    const unsigned long long xring = express_ring_entries(ctl);
    unsigned long long lane_f = 0, lane_g = 0, wave_f = 0, wave_g = 0, wave_m = 0, evals = 0, grads = 0, hits = 0,
                       chains = 0, rides = 0;
    unsigned round_no = 0;
    bool drained = false;

    // a slot's record is written by whichever lane served it last: order this wave's global writes before its next
    // reads (single-wave workgroup; the L1 is the CU's own)
    auto sync_slots = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };

    // New series for the slots of the lanes with need = true (wave-uniform call): claim from the work counter,
    // report series whose Hannan-Rissanen init failed, post G at the initial point (what advance() does first).
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
                if (sid >= N) {
                    drained = true;
                    dreq[slot] = (uint8_t)kFitGDirEmpty;
                    dsid[slot] = -1;
                    need = false;
                } else {
                    const int st0 = init_status ? init_status[sid] : ARIMA_ST_OK;
                    if (st0 != ARIMA_ST_OK) {
                        double nanc[K];
#pragma unroll
                        for (int j = 0; j < K; ++j) nanc[j] = __builtin_nan("");
                        write_fit<K>(sid, st0, nanc, 0.0, 0, 0, 0, coef_out, ll_out, status_out, n_eval_out,
                                     n_grad_out, flags_out);
                    } else {
                        double x0[K];
#pragma unroll
                        for (int j = 0; j < K; ++j) x0[j] = init[sid * K + j];
                        FitSlotCore<K> &R = gs[slot].c;
                        R.s.start_posted(x0);
                        R.sid = sid;
#ifdef STS_TIMING
                        R.t_start = (double)__builtin_amdgcn_s_memrealtime();
                        R.t_donate = 0.0;
#endif
                        dreq[slot] = (uint8_t)REQ_G;
                        dnev[slot] = 0;
                        dsid[slot] = sid;
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
    sync_slots();

    for (;;) {
        // ---- pick the pass (k_cg_fit's rule): all-G or all-F, up to 64 slots, long-running slots first ----
        unsigned long long mF[NJ], mG[NJ], mO[NJ];
        int nF = 0, nG = 0, nOF = 0, nOG = 0;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int slot = lane + 64 * j;
            int r = REQ_NONE;
            bool old = false;
            if (slot < SPW) {
                const int dr = dreq[slot];
                r = dr == kFitGDirEmpty ? REQ_NONE : dr;
                old = r != REQ_NONE && dnev[slot] >= kOldEvals;
            }
            mF[j] = __ballot(r == REQ_F);
            mG[j] = __ballot(r == REQ_G);
            mO[j] = __ballot(old);
            nF += __popcll(mF[j]);
            nG += __popcll(mG[j]);
            nOF += __popcll(mF[j] & mO[j]);
            nOG += __popcll(mG[j] & mO[j]);
        }
        if (nF + nG == 0) break;
        const bool doG = nOG != nOF ? nOG > nOF : (nG >= 64 || (nF < 64 && nG >= nF));
        const int rot = (int)(round_no * 37u) & 63;
        round_no++;
        int base = 0;
#pragma unroll
        for (int tier = 0; tier < (kFRide ? 4 : 2); ++tier) {
            if (tier >= 2 && (!doG || base >= 64)) break;
#pragma unroll
            for (int jj = 0; jj < NJ; ++jj) {
                const int j = (jj + (int)round_no) % NJ;
                unsigned long long m = ((doG && tier < 2) ? mG[j] : mF[j]) & ((tier & 1) == 0 ? mO[j] : ~mO[j]);
                m = (m >> rot) | (rot ? (m << (64 - rot)) : 0ull);
                const int lr = (lane - rot) & 63;
                if ((m >> lr) & 1ull) {
                    const int rank = base + __popcll(m & ((1ull << lr) - 1ull));
                    if (rank < 64) assign[rank] = lane + 64 * j;
                }
                base += __popcll(m);
            }
        }
        const int nsel = base < 64 ? base : 64;
        wave_sync_lds();
        const bool served = lane < nsel;
        const int my = served ? assign[lane] : 0;
        const int myreq = served ? (int)dreq[my] : REQ_NONE;
        const int64_t sid = served ? dsid[my] : 0;
        const double *row = served ? y + sid * ld : y;
        // the request's point (and its predicted points) from the slot record
        double c[K], css, g[K];
        int nsp = 0;
        const Lane &GS = gs[my].c.s;
        if (served) {
            if (myreq == REQ_G) {
#pragma unroll
                for (int j = 0; j < K; ++j) c[j] = GS.point[j];
            } else {
                const double al = GS.ev_alpha;
#pragma unroll
                for (int j = 0; j < K; ++j) c[j] = GS.point[j] + al * GS.dir[j];
                if (!doG) nsp = GS.rq_nspec;
            }
        } else {
#pragma unroll
            for (int j = 0; j < K; ++j) c[j] = 0.0;
        }
        double resp_f = 0.0;
        double spv[NS > 0 ? NS : 1];
        if (doG) {
            css_pass<P, Q, I, true, SMEAR, kFitGPrefetchG>(row, n, c, css, g);
            resp_f = css_to_loglik(css, n);
            wave_g += lane0;
            lane_g += served;
            rides += (served && myreq == REQ_F) ? 1ull : 0ull;
        } else {
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
                        const double al = GS.rq_spec[h - 1];
#pragma unroll
                        for (int j = 0; j < K; ++j) cm[h][j] = GS.point[j] + al * GS.dir[j];
                    } else {
#pragma unroll
                        for (int j = 0; j < K; ++j) cm[h][j] = c[j];
                    }
                }
                css_pass_multi<P, Q, I, NCH, kFitGPrefetchF>(row, n, cm, cssm);
                css = cssm[0];
#pragma unroll
                for (int h = 1; h < NCH; ++h) spv[h - 1] = css_to_loglik(cssm[h], n);
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
        }
        // ---- each served lane advances its slot's state in registers and writes the record back ----
        bool need = false;
        if (served) {
            Lane S = GS;
            if (!doG) {
#pragma unroll
                for (int h = 1; h <= NS; ++h)
                    if (h <= nsp) S.spec_store(h - 1, spv[h - 1]);
            }
            S.req = REQ_NONE;
            S.step(resp_f, g);
            if (S.done()) {
                double pt[K];
#pragma unroll
                for (int j = 0; j < K; ++j) pt[j] = S.point[j];
                write_fit<K>(sid, S.status, pt, S.prev_obj, S.n_eval, S.n_grad,
                             S.status == ARIMA_ST_OK ? model_flags<P, Q, I>(pt) : (uint8_t)0, coef_out, ll_out,
                             status_out, n_eval_out, n_grad_out, flags_out);
#ifdef STS_TIMING
                if constexpr (K >= 2) {
                    coef_out[sid * K + 0] = gs[my].c.t_start;
                    coef_out[sid * K + 1] = gs[my].c.t_donate;
                }
#endif
                evals += S.n_eval;
                grads += S.n_grad;
                hits += S.spec_hits;
                need = true;
            } else {
                gs[my].c.s = S;
                dreq[my] = S.req;
                dnev[my] = S.n_eval;
            }
        }
        refill(my, need);
        if (has_express) {
            unsigned long long wants = 0, filled = 0, fault = 0;
            if (lane0) {
                wants = ld_agent(&ctl[20]);
                filled = ld_agent(&ctl[21]);
                fault = ld_agent(&ctl[26]);
            }
            wants = __shfl(wants, 0);
            filled = __shfl(filled, 0);
            fault = __shfl(fault, 0);
            if (wants > filled && filled < xring && fault == 0) {
                const int donate_min = __any(drained) ? kDonateEvalsDrained : kDonateEvals;
                unsigned long long key = 0;
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int slot = lane + 64 * j;
                    if (slot < SPW) {
                        const int dr = dreq[slot];
                        if (dr != kFitGDirEmpty && dr != REQ_NONE && dnev[slot] >= donate_min) {
                            const unsigned long long kk = ((unsigned long long)dnev[slot] << 16) | (unsigned)(slot + 1);
                            key = kk > key ? kk : key;
                        }
                    }
                }
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
                    const unsigned long long o = __shfl_xor(key, off);
                    key = o > key ? o : key;
                }
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
                    sync_slots();                           // the slot's latest record is visible to every lane
#ifdef STS_TIMING
                    if (lane == (bs & 63)) gs[bs].c.t_donate = (double)__builtin_amdgcn_s_memrealtime();
                    sync_slots();
#endif
                    publish_core<K>(reinterpret_cast<unsigned long long *>(xq + (size_t)e * kExpressEntryBytes),
                                    &gs[bs].c, lane, jx + 1);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (lane0) st_agent(&xready[e], (unsigned)(jx + 1));
                    if (lane == (bs & 63)) {
                        dreq[bs] = (uint8_t)kFitGDirEmpty;
                        dsid[bs] = -1;
                    }
                    wave_sync_lds();
                    refill(bs, lane == (bs & 63));
                }
            }
        }
        sync_slots();
    }
    if (has_express) {
        if (lane0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            add_agent(&ctl[22], 1ull);
        }
        if (join_express) {
            wave_sync_lds();
            fit_express<P, Q, I, SMEAR>(xlds, (int)sizeof(xlds), y, ld, n, coef_out, ll_out, status_out, n_eval_out,
                                        n_grad_out, flags_out, ctl, xq, xready, N, lane);
        }
    }
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
}

}  // namespace sts
