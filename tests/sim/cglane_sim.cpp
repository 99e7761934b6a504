// cglane_sim.cpp — TEST INFRASTRUCTURE: runs the fit kernel's optimizer state machine (cg_lane.hpp, the exact
// code of k_cg_fit's slots) on the CPU, answering its requests with the CPU restatement's objective and gradient
// (oracle/arima_oracle.c). Used by tests/test_cglane_sim.py to check, without a GPU, that every speculation
// policy leaves the reference's evaluation accounting and results unchanged, and to count the passes a policy
// needs (the quantity the kernel's time follows). Built by tests/sim/Makefile into tests/sim/_build/.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../../spark-timeseries_amd/csrc/cg_lane.hpp"

extern "C" double orc_loglik_css_arma(const double *y, int n, int p, int q, int I, const double *coef);
extern "C" void orc_gradient_css_arma(const double *y, int n, int p, int q, int I, const double *coef, int smear,
                                      double *grad);

namespace {

template <int K, int NS, int NC>
void run_one(const double *y, int n, int p, int q, int I, int smear, const double *init, double *coef_out,
             double *ll_out, int32_t *status_out, int32_t *counts_out) {
    sts::CGLane<K, NS, NC> L;
    double x0[K];
    for (int i = 0; i < K; ++i) x0[i] = init[i];
    L.start(x0);
    double fr = 0.0, gr[K] = {};
    int passes_f = 0, passes_g = 0, chains = 0;
    for (int j = 6; j < 14; ++j) counts_out[j] = 0;
    for (;;) {
        L.advance(fr, gr);
        if (L.done()) break;
        double c[K];
        L.request_point(c);
        if (L.req == sts::REQ_G) {
            orc_gradient_css_arma(y, n, p, q, I, c, smear, gr);
            fr = orc_loglik_css_arma(y, n, p, q, I, c);
            passes_g++;
        } else {
            fr = orc_loglik_css_arma(y, n, p, q, I, c);
            int cls = 6;
            switch (L.pc) {
            case sts::PC_BR_FB: cls = 0; break;
            case sts::PC_BR_FC: cls = 1; break;
            case sts::PC_BR_SHIFT_EV: cls = 2; break;
            case sts::PC_BR_A1: cls = 3; break;
            case sts::PC_BR_C1: cls = 4; break;
            case sts::PC_BRENT_FU: cls = L.have_prev ? 6 : 5; break;
            default: cls = 7; break;
            }
            counts_out[6 + cls]++;
            if (std::getenv("SIM_TRACE")) {
                std::printf("F pc=%d alpha=%.17g spec:", (int)L.pc, L.ev_alpha);
                for (int h = 0; h < L.rq_nspec; ++h) std::printf(" %.17g", L.rq_spec[h]);
                if (L.pc == sts::PC_BRENT_FU)
                    std::printf("   [a=%.17g b=%.17g x=%.17g v=%.17g w=%.17g fx=%.17g fv=%.17g fw=%.17g be=%.3g bd=%.3g have_prev=%d]",
                                L.a, L.b, L.bx, L.bv, L.bw, L.fx, L.fv, L.fw, L.be, L.bd, (int)L.have_prev);
                std::printf("\n");
            }
            for (int h = 0; h < L.rq_nspec; ++h) {
                double cs[K];
                L.spec_point(h, cs);
                L.spec_store(h, orc_loglik_css_arma(y, n, p, q, I, cs));
            }
            chains += 1 + L.rq_nspec;
            passes_f++;
        }
        L.req = sts::REQ_NONE;
    }
    const bool ok = L.status == ARIMA_ST_OK;
    for (int i = 0; i < K; ++i) coef_out[i] = ok ? L.point[i] : NAN;
    *ll_out = ok ? L.prev_obj : NAN;
    *status_out = L.status;
    counts_out[0] = L.n_eval;
    counts_out[1] = L.n_grad;
    counts_out[2] = passes_f;
    counts_out[3] = passes_g;
    counts_out[4] = L.spec_hits;
    counts_out[5] = chains;
}

template <int K, int NS, int NC>
void run_batch(const double *y, int64_t N, int ld, int n, int p, int q, int I, int smear, const double *init,
               double *coef, double *ll, int32_t *st, int32_t *counts) {
#pragma omp parallel for schedule(dynamic, 8)
    for (int64_t i = 0; i < N; ++i)
        run_one<K, NS, NC>(y + i * ld, n, p, q, I, smear, init + i * K, coef + i * K, ll + i, st + i, counts + i * 14);
}

template <int K>
int dispatch_policy(int ns, int nc, const double *y, int64_t N, int ld, int n, int p, int q, int I, int smear,
                    const double *init, double *coef, double *ll, int32_t *st, int32_t *counts) {
#define POL(A, B)                                                                               \
    if (ns == A && nc == B) {                                                                  \
        run_batch<K, A, B>(y, N, ld, n, p, q, I, smear, init, coef, ll, st, counts);           \
        return 0;                                                                              \
    }
    POL(0, 0) POL(1, 1) POL(1, 2) POL(2, 2) POL(2, 4) POL(3, 3) POL(3, 4) POL(3, 6) POL(4, 4) POL(4, 8)
#undef POL
    return -1;
}

}  // namespace

// Evaluations per CG iteration of the NaN-absorbing state, counted by stepping the machine WITHOUT the fast-forward
// (a non-finite point, F(point) = NaN; every request answered with NaN), and the constant the kernel uses for it.
extern "C" int sim_nan_iter_evals(int dir_finite) {
    // advance() runs the absorbing state to MaxEval in one call, so E is found as the smallest evaluation budget
    // x (n_eval = MaxEval - x at the top of the loop) in which one whole iteration -- one gradient -- completes
    for (int x = 1; x <= 1000; ++x) {
        sts::CGLane<5, 2, 4, false> L;
        double x0[5] = {NAN, 0.1, 0.2, 0.3, 0.4};
        L.start(x0);
        L.pc = sts::PC_TOP;
        L.memo_obj = NAN;
        L.prev_obj = NAN;
        L.have_prev_obj = 1;
        for (int i = 0; i < 5; ++i) L.dir[i] = dir_finite ? 1.0 : NAN;
        L.n_eval = (uint16_t)(sts::kMaxEval - x);
        L.n_grad = 0;
        const double g[5] = {NAN, NAN, NAN, NAN, NAN};
        L.advance(NAN, g);
        if (!L.done() || L.status != ARIMA_ST_MAX_EVAL || L.n_eval != sts::kMaxEval) return -1;  // never a pass
        if (L.n_grad == 1) return x;
    }
    return -2;
}

extern "C" int sim_k_nan_iter_evals() { return sts::kNanIterEvals; }

// Fits N already-differenced series (row i at y + i * ld, length n) from the given initial points (N x K).
// counts (N x 14): n_eval, n_grad, F passes, G passes, speculative hits, objective chains evaluated, then F passes by resume point (FB, FC, SHIFT_EV, A1, C1, Brent u1, Brent later, other).
extern "C" int sim_fit_batch(const double *y, int64_t N, int ld, int n, int p, int q, int I, int smear,
                             const double *init, int ns, int nc, double *coef, double *ll, int32_t *status,
                             int32_t *counts) {
    const int K = I + p + q;
    switch (K) {
#define KC(KK) \
    case KK: return dispatch_policy<KK>(ns, nc, y, N, ld, n, p, q, I, smear, init, coef, ll, status, counts);
        KC(1) KC(2) KC(3) KC(4) KC(5) KC(6) KC(7) KC(8) KC(9) KC(10) KC(11)
#undef KC
    default: return -2;
    }
}
