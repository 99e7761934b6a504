#pragma once
// arima_fit_reg.hpp — k_cg_fit_r: the persistent CSS-CGD fit kernel at TWO waves per SIMD (fit_kernel = 3).
// Included by arima_kernels_impl.hpp (uses its FitSlot, fit_express, write_fit, refill policy and counters).
//
// Why: k_cg_fit keeps every optimizer slot (CGLane + series id, 376 B at C2) in
// LDS, 104 slots per wave, which fills the CU's 160 KB at ONE wave per SIMD -- while the wave uses 144 of its 512
// registers. One wave cannot hide the fp64 dependency latency of the CSS recursion nor issue back to back
// (tools/ubench_fp64.hip: 6.75 SIMD-cycles per fp64 instruction at one wave, 4.28 at two). Here each lane owns one
// slot in REGISTERS (its "register slot", advanced by the force-inlined CGLane::step) and the wave keeps a reserve
// of SPL further slots in its eighth of the LDS. A pass of type X (all-objective or all-gradient, as in k_cg_fit)
// serves every lane whose register slot wants X; the other lanes SWAP their register slot with a reserve slot that
// wants X (one 376-B exchange through LDS), so passes stay full while 64 + SPL slots per wave (116 at C2, 232 per
// SIMD vs 104) keep requests of both types waiting. In a gradient pass, lanes left over after the G requests serve
// their own objective request as a rider (the pass yields the objective), as k_cg_fit does.
// Everything a slot computes is the same CGLane code on the same responses, so results and evaluation counts are
// bit-identical to k_cg_fit and the oracle; only which lane serves a slot, and when, changes.
//
// Express path, hand-off ring, watchdog and counters are k_cg_fit's (fit_express runs in the wave's LDS share, so
// only rows up to cg_fit_reg_max_n() doubles can take it: C2's 1023 can, C4's 4095 cannot -- the runtime then
// keeps k_cg_fit).

namespace sts {

#ifndef STS_REG_PREFETCH_F
#define STS_REG_PREFETCH_F 2
#endif
#ifndef STS_REG_PREFETCH_G
#define STS_REG_PREFETCH_G 2
#endif

// reserve slots per wave: the wave's eighth of the LDS less the hand-off staging slot and the pass assignment
#ifndef STS_REG_SPL_MAX
#define STS_REG_SPL_MAX 64
#endif
template <int K>
constexpr int reg_lds_slots() {
    constexpr int per_wave = kFitLdsBudget / kRegWavesPerCU;
    constexpr int avail = per_wave - 64 * 4 - (int)sizeof(FitSlot<K>);
    constexpr int nslots = avail / (int)sizeof(FitSlot<K>);
    constexpr int cap = nslots > STS_REG_SPL_MAX ? STS_REG_SPL_MAX : nslots;
    return (cap / 4) * 4;
}

template <int K, int SPL>
struct RegWaveLds {
    FitSlot<K> slots[SPL];       // reserve slots (lane l < SPL takes the census of slot l)
    FitSlot<K> stage;            // a register slot on its way into the express ring
    int assign[64];              // reserve slots of the pass type, in serving order
};

template <int K>
constexpr int reg_wave_lds_bytes() { return (int)sizeof(RegWaveLds<K, reg_lds_slots<K>()>); }

template <int P, int Q, int I, bool SMEAR, int SPL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_cg_fit_r(
    const double *__restrict__ y, int64_t ld, int n, int64_t N, const double *__restrict__ init,
    const int32_t *__restrict__ init_status, double *__restrict__ coef_out, double *__restrict__ ll_out,
    int32_t *__restrict__ status_out, int32_t *__restrict__ n_eval_out, int32_t *__restrict__ n_grad_out,
    uint8_t *__restrict__ flags_out, unsigned long long *__restrict__ ctl, unsigned char *__restrict__ xq,
    unsigned *__restrict__ xready, int n_bulk, int join_express, const int32_t *__restrict__ resume_list,
    const unsigned *__restrict__ resume_n, const unsigned char *__restrict__ resume_rec) {
    constexpr int K = I + P + Q;
    constexpr int NS = spec_ns<K>();
    constexpr int NC = spec_nc<K>();
    using Lane = CGLane<K, NS, NC>;
    static_assert(SPL >= 8 && SPL <= 64, "reserve slots per wave");
    static_assert(sizeof(FitSlotCore<K>) <= kExpressEntryBytes, "express ring entry");
    __shared__ RegWaveLds<K, SPL> W;
    const int lane = threadIdx.x & 63;
    const bool lane0 = lane == 0;
    const bool has_express = n_bulk < (int)gridDim.x;
    unsigned char *wlds = reinterpret_cast<unsigned char *>(&W);
    // (no resume mode: the rounds fit's tail runs on k_cg_fit; resume_list is always null here)
#ifndef STS_REG_EXP_NOX
    if ((int)blockIdx.x >= n_bulk) {
        fit_express<P, Q, I, SMEAR, 16, false>(wlds, (int)sizeof(W), y, ld, n, coef_out, ll_out, status_out, n_eval_out,
                                    n_grad_out, flags_out, ctl, xq, xready, N, lane);
        return;
    }
#endif
    if (has_express && lane0) {
        add_agent(&ctl[17], 1ull);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned long long xring = express_ring_entries(ctl);
    unsigned long long lane_f = 0, lane_g = 0, wave_f = 0, wave_g = 0, wave_m = 0, evals = 0, grads = 0, hits = 0,
                       chains = 0, rides = 0, done = 0;
    unsigned round_no = 0;
    bool drained = false;
#ifdef STS_TIMING
    unsigned long long tm_f = 0, tm_g = 0, tm_adv = 0, tm_sel = 0, tm_drain = 0;
    const unsigned long long tm_start = __builtin_amdgcn_s_memtime();
    auto now = [] { return __builtin_amdgcn_s_memtime(); };
#endif

    // the lane's register slot
    Lane R;
    int64_t rsid = -1;
    R.req = REQ_NONE;
    R.pc = PC_DONE;

    // next series from the work counter for every lane with need (wave-uniform call). to_reg: into the lane's
    // register slot; else into reserve slot `slot`. Series whose HR init failed are written out and skipped.
    auto refill = [&](bool need, bool to_reg, int slot) {
        for (;;) {
            const unsigned long long m = __ballot(need);
            if (m == 0ull) break;
            const int leader = __ffsll((long long)m) - 1;
            unsigned long long base = 0;
            if (lane == leader) base = add_agent(&ctl[0], (unsigned long long)__popcll(m));
            base = __shfl(base, leader);
            if (!need) continue;
            const int rank = __popcll(m & ((1ull << lane) - 1ull));
            const int64_t sid = (int64_t)(base + (unsigned long long)rank);
            if (sid >= N) {
                drained = true;
#ifdef STS_TIMING
                if (tm_drain == 0) tm_drain = __builtin_amdgcn_s_memtime();
#endif
                if (to_reg) {
                    rsid = -1;
                    R.req = REQ_NONE;
                } else {
                    W.slots[slot].c.sid = -1;
                    W.slots[slot].c.s.req = REQ_NONE;
                }
                need = false;
                continue;
            }
            Lane L;
            const int64_t lsid = sid;
            {
                const int st0 = init_status ? init_status[sid] : ARIMA_ST_OK;
                if (st0 != ARIMA_ST_OK) {
                    double nanc[K];
#pragma unroll
                    for (int j = 0; j < K; ++j) nanc[j] = __builtin_nan("");
                    write_fit<K>(sid, st0, nanc, 0.0, 0, 0, 0, coef_out, ll_out, status_out, n_eval_out, n_grad_out,
                                 flags_out);
                    done++;
                    continue;                           // still in need: take the next series
                }
                double x0[K];
#pragma unroll
                for (int j = 0; j < K; ++j) x0[j] = init[sid * K + j];
                L.start_posted(x0);                     // G at the initial point posted
            }
            if (to_reg) {
                R = L;
                rsid = lsid;
            } else {
                W.slots[slot].c.s = L;
                W.slots[slot].c.sid = lsid;
            }
            need = false;
        }
    };

    // every reserve slot and every register slot gets a series
    if (lane < SPL) W.slots[lane].c.sid = -1;
    refill(lane < SPL, false, lane < SPL ? lane : 0);
    refill(true, true, 0);
    wave_sync_lds();

    for (;;) {
#ifdef STS_TIMING
        const unsigned long long t_a = now();
#endif
        // ---- census: requests of the register slots and of the reserve slots ----
        const int rR = rsid >= 0 ? (int)R.req : REQ_NONE;
        const bool oR = rsid >= 0 && R.n_eval >= kOldEvals;
        int rL = REQ_NONE;
        bool oL = false;
        if (lane < SPL && W.slots[lane].c.sid >= 0) {
            rL = W.slots[lane].c.s.req;
            oL = W.slots[lane].c.s.n_eval >= kOldEvals;
        }
        const unsigned long long mRF = __ballot(rR == REQ_F), mRG = __ballot(rR == REQ_G), mRO = __ballot(oR);
        const unsigned long long mLF = __ballot(rL == REQ_F), mLG = __ballot(rL == REQ_G), mLO = __ballot(oL);
        const int nF = __popcll(mRF) + __popcll(mLF), nG = __popcll(mRG) + __popcll(mLG);
        if (nF + nG == 0) break;                      // batch drained and every slot of this wave finished
        const int nOF = __popcll(mRF & mRO) + __popcll(mLF & mLO), nOG = __popcll(mRG & mRO) + __popcll(mLG & mLO);
        // the pass type: k_cg_fit's rule (long-running requests decide, else the type that fills the pass)
        const bool doG = nOG != nOF ? nOG > nOF : (nG >= 64 || (nF < 64 && nG >= nF));
        const int X = doG ? REQ_G : REQ_F;
        const int rot = (int)(round_no * 37u) & 63;
        round_no++;
        // ---- reserve slots of type X in serving order (long-running first, rotating), then for a G pass the
        //      reserve objective requests that ride on lanes without a series of their own ----
        const unsigned long long mLX = doG ? mLG : mLF;
        const int lr = (lane - rot) & 63;
        auto rotl = [&](unsigned long long m) { return (m >> rot) | (rot ? (m << (64 - rot)) : 0ull); };
        int base = 0;
        // free lanes: register slot not of type X (another request, or no series)
        const unsigned long long mFree = ~(doG ? mRG : mRF);
        const int nFree = __popcll(mFree);
        const int nA = __popcll(mLX) < nFree ? __popcll(mLX) : nFree;     // reserve X slots that get a lane
#pragma unroll
        for (int tier = 0; tier < 2; ++tier) {
            unsigned long long m = rotl(mLX & (tier == 0 ? mLO : ~mLO));
            if ((m >> lr) & 1ull) {
                const int rank = base + __popcll(m & ((1ull << lr) - 1ull));
                if (rank < 64) W.assign[rank] = lane;
            }
            base += __popcll(m);
        }
        // lanes with no series left after the X matching take reserve F slots as riders of a G pass
        const unsigned long long mEmpty = __ballot(rsid < 0);
        const int frank = __popcll(mFree & ((1ull << lane) - 1ull));
        const bool takeA = ((mFree >> lane) & 1ull) && frank < nA;
        const unsigned long long mEmptyLeft = mEmpty & ~__ballot(takeA);
        int nB = 0;
        if (doG && kFRide && mEmptyLeft) {
            const int nEL = __popcll(mEmptyLeft);
            int b2 = nA;
#pragma unroll
            for (int tier = 0; tier < 2; ++tier) {
                unsigned long long m = rotl(mLF & (tier == 0 ? mLO : ~mLO));
                if ((m >> lr) & 1ull) {
                    const int rank = b2 + __popcll(m & ((1ull << lr) - 1ull));
                    if (rank < 64 && rank - nA < nEL) W.assign[rank] = lane;
                }
                b2 += __popcll(m);
            }
            nB = __popcll(mLF) < nEL ? __popcll(mLF) : nEL;
        }
        wave_sync_lds();
        // ---- swaps: a matched lane exchanges its register slot with its reserve slot ----
        int target = -1;
        if (takeA) target = W.assign[frank];
        else if (nB > 0 && ((mEmptyLeft >> lane) & 1ull)) {
            const int erank = __popcll(mEmptyLeft & ((1ull << lane) - 1ull));
            if (erank < nB) target = W.assign[nA + erank];
        }
#ifndef STS_REG_EXP_NOSWAP
        if (target >= 0) {
            FitSlotCore<K> in;
            __builtin_memcpy(&in, &W.slots[target].c, sizeof(in));
            W.slots[target].c.s = R;
            W.slots[target].c.sid = rsid;
            R = in.s;
            rsid = in.sid;
        }
#endif
        wave_sync_lds();
        // ---- the pass ----
        const bool served = rsid >= 0 && R.req != REQ_NONE && (doG || R.req == REQ_F);
        const double *row = served ? y + rsid * ld : y;
        double c[K], css, g[K];
        if (served) {
            R.request_point(c);
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
            css_pass<P, Q, I, true, SMEAR, STS_REG_PREFETCH_G>(row, n, c, css, g);
            resp_f = css_to_loglik(css, n);
            wave_g += lane0;
            lane_g += served;
            rides += (served && R.req == REQ_F) ? 1ull : 0ull;
        } else {
            const int nsp = served ? (int)R.rq_nspec : 0;
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
                        R.spec_point(h - 1, cs);
#pragma unroll
                        for (int j = 0; j < K; ++j) cm[h][j] = cs[j];
                    } else {
#pragma unroll
                        for (int j = 0; j < K; ++j) cm[h][j] = c[j];
                    }
                }
                css_pass_multi<P, Q, I, NCH, STS_REG_PREFETCH_F>(row, n, cm, cssm);
                css = cssm[0];
                if (served) {
#pragma unroll
                    for (int h = 1; h < NCH; ++h)
                        if (h <= nsp) R.spec_store(h - 1, css_to_loglik(cssm[h], n));
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
        }
#ifdef STS_TIMING
        const unsigned long long t_c = now();
        if (doG) tm_g += t_c - t_b; else tm_f += t_c - t_b;
#endif
        // ---- the served register slots advance (in registers); finished ones are written out and refilled ----
        bool need = false;
        if (served) {
            R.req = REQ_NONE;
#ifndef STS_REG_EXP_NOSTEP
            R.step(resp_f, g);
#endif
            if (R.done()) {
                double pt[K];
#pragma unroll
                for (int j = 0; j < K; ++j) pt[j] = R.point[j];
                write_fit<K>(rsid, R.status, pt, R.prev_obj, R.n_eval, R.n_grad,
                             R.status == ARIMA_ST_OK ? model_flags<P, Q, I>(pt) : (uint8_t)0, coef_out, ll_out,
                             status_out, n_eval_out, n_grad_out, flags_out);
                evals += R.n_eval;
                grads += R.n_grad;
                hits += R.spec_hits;
                done++;
                rsid = -1;
                need = true;
            }
        }
        refill(need, true, 0);
        if (has_express) {
            // an express wave is waiting: hand it this wave's oldest slot (register or reserve)
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
                unsigned long long key = 0;             // (n_eval << 16) | (1 + 64 * reserve + index)
                if (rsid >= 0 && R.req != REQ_NONE && R.n_eval >= donate_min)
                    key = ((unsigned long long)R.n_eval << 16) | (unsigned)(1 + lane);
                if (lane < SPL && W.slots[lane].c.sid >= 0 && W.slots[lane].c.s.req != REQ_NONE &&
                    W.slots[lane].c.s.n_eval >= donate_min) {
                    const unsigned long long kk = ((unsigned long long)W.slots[lane].c.s.n_eval << 16) |
                                                  (unsigned)(1 + 64 + lane);
                    key = kk > key ? kk : key;
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
                    const int who = (int)(key & 0xffffull) - 1;
                    const bool from_reserve = who >= 64;
                    const int idx = who & 63;
                    if (!from_reserve && lane == idx) {     // the register slot goes out through the staging slot
                        W.stage.c.s = R;
                        W.stage.c.sid = rsid;
                    }
                    wave_sync_lds();
                    const unsigned e = (unsigned)(jx % xring);
                    publish_core<K>(reinterpret_cast<unsigned long long *>(xq + (size_t)e * kExpressEntryBytes),
                                    from_reserve ? &W.slots[idx].c : &W.stage.c, lane, jx + 1);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (lane0) st_agent(&xready[e], (unsigned)(jx + 1));
                    if (lane == idx) {
                        if (from_reserve) {
                            W.slots[idx].c.sid = -1;
                            W.slots[idx].c.s.req = REQ_NONE;
                        } else {
                            rsid = -1;
                            R.req = REQ_NONE;
                        }
                    }
                    wave_sync_lds();
                    refill(lane == idx, !from_reserve, idx);
                }
            }
        }
        wave_sync_lds();
#ifdef STS_TIMING
        tm_adv += now() - t_c;
#endif
    }
    if (has_express) {
        if (lane0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            add_agent(&ctl[22], 1ull);
        }
        if (join_express) {
            wave_sync_lds();
#ifndef STS_REG_EXP_NOX
            fit_express<P, Q, I, SMEAR, 16, false>(wlds, (int)sizeof(W), y, ld, n, coef_out, ll_out, status_out, n_eval_out,
                                        n_grad_out, flags_out, ctl, xq, xready, N, lane);
#endif
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
}

}  // namespace sts
