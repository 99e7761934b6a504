// cg_lane.hpp — commons-math3 3.4.1 NonLinearConjugateGradientOptimizer(FLETCHER_REEVES,
// SimpleValueChecker(1e-7, 1e-7)) with LineSearch (BracketFinder + BrentOptimizer(1e-15, MIN_VALUE,
// SimpleUnivariateValueChecker(1e-8, 1e-8))), as one series' resumable state machine (ARIMA.scala:174-200;
// SURVEY.md Appendix A restates the commons algorithms).
//
// Portable C++ (host and device): the fit kernel keeps one CGLane per optimizer slot in LDS, and
// tests/sim/cglane_sim.cpp runs the same code on the CPU against the oracle's objective to check the evaluation
// accounting and to measure the speculation policy.
//
// The machine posts one request at a time (objective F or gradient G at a point); the kernel serves it with one
// pass over the series and calls advance() with the response. Requests that need no pass (every one of them
// still counted exactly as the reference counts it):
//   - F(point) at the top of each CG iteration: equals the line search's best value (same point, same ops)
//     or, on the first iteration, the objective fused into the G(x0) pass;
//   - the bracket's f(0) = F(point) when the direction is finite; Brent's f(mid) = the bracket's f at mid;
//   - any non-finite point: the CSS objective and gradient are NaN (every step multiplies every coefficient);
//   - a point whose value a speculative chain of an earlier pass of the same line search already computed.
//
// Speculation. Many line-search points do not depend on objective values, or depend on them only through a
// two-way branch, so an F request carries up to NS predicted alphas (predict()): BracketFinder's golden
// extension xC = xB + GOLD(xB - xA) and its grow-limit chain wLim = xB + 100 (xC - xB) while the objective keeps
// rising; the golden-section first step of BrentOptimizer for each bracket the pending evaluation can close
// (Brent's e = 0 at its first iteration); and Brent's second step, which is golden-section again for either
// outcome of the first (its parabola degenerates: v = w). The pass evaluates the predictions as extra chains
// over the same streamed bytes; their values go into a per-line-search cache keyed by the exact alpha bits. A
// hit is a point the reference evaluates with the same operations, so results and counts are unchanged.
#pragma once

#include <stdint.h>

#include "../../include/sparkts_arima.h"

#if defined(__HIPCC__) || defined(__HIP__)
#define STS_HD __host__ __device__
#define STS_FI __forceinline__
#else
#define STS_HD
#define STS_FI inline
#endif

namespace sts {

constexpr int kMaxEval = 10000;      // new MaxEval(10000)  ARIMA.scala:196
constexpr int kMaxIter = 10000;      // new MaxIter(10000)  ARIMA.scala:195
constexpr int kBracketMax = 500;     // commons BracketFinder() = BracketFinder(growLimit 100, maxEval 500)

STS_HD STS_FI long long dbits(double x) { return __builtin_bit_cast(long long, x); }
STS_HD STS_FI double dabs(double x) { return __builtin_fabs(x); }
STS_HD STS_FI bool finite(double v) { return __builtin_isfinite(v); }

enum : int { REQ_NONE = 0, REQ_F = 1, REQ_G = 2 };

enum : int {
    PC_START = 0, PC_G0, PC_TOP, PC_BR_FA, PC_BR_FB, PC_BR_FC, PC_BR_LOOP, PC_BR_A1, PC_BR_C1,
    PC_BR_SHIFT_EV, PC_BR_SHIFT, PC_BR_END, PC_BRENT_FX, PC_BRENT_LOOP, PC_BRENT_FU, PC_LS_DONE, PC_G,
    PC_EVAL, PC_DONE
};

// Precision.equals(x, y, 1)
STS_HD STS_FI bool prec_equals(double x, double y) {
    const long long xi = dbits(x), yi = dbits(y);
    bool eq;
    if (((xi ^ yi) & (long long)0x8000000000000000ull) == 0) {
        long long dd = xi - yi;
        eq = (dd < 0 ? -dd : dd) <= 1;
    } else {
        const long long NEG0 = (long long)0x8000000000000000ull;
        long long dplus, dminus;
        if (xi < yi) { dplus = yi; dminus = xi - NEG0; } else { dplus = xi; dminus = yi - NEG0; }
        eq = (dplus > 1) ? false : (dminus <= (1 - dplus));
    }
    return eq && !__builtin_isnan(x) && !__builtin_isnan(y);
}

// SimpleValueChecker.converged: |p-c| <= max(|p|,|c|)*rel || |p-c| <= abs, FastMath.max propagates NaN
STS_HD STS_FI bool value_converged(double p, double c, double rel, double abs_) {
    const double diff = dabs(p - c);
    const double ap = dabs(p), ac = dabs(c);
    double size;
    if (ap > ac) size = ap;
    else if (ap < ac) size = ac;
    else if (ap != ac) size = __builtin_nan("");
    else size = ap;
    return (diff <= size * rel) || (diff <= abs_);
}

constexpr double kGold = 1.618034, kEpsMin = 1e-21, kGrow = 100.0;   // BracketFinder
constexpr double kBrentAbs = 4.9e-324;                                // Double.MIN_VALUE

// BrentOptimizer.GOLDEN_SECTION = 0.5 * (3 - sqrt(5))
STS_HD STS_FI double brent_gs() { return 0.5 * (3 - __builtin_sqrt(5.0)); }

// Golden-section step of one BrentOptimizer iteration at (a, b, x) when the parabola is not taken (the first
// iteration, e = 0, and the second, v = w): the stopping test, then u. Returns false when Brent stops there.
STS_HD STS_FI bool brent_golden_u(double a, double b, double x, double &u) {
    const double m = 0.5 * (a + b);
    const double tol1 = 1e-15 * dabs(x) + kBrentAbs;
    const double tol2 = 2 * tol1;
    if (dabs(x - m) <= tol2 - 0.5 * (b - a)) return false;
    const double e = (x < m) ? b - x : a - x;
    const double d = brent_gs() * e;
    u = (dabs(d) < tol1) ? ((d >= 0) ? x + tol1 : x - tol1) : x + d;
    return true;
}

// Brent's first evaluation point for the bracket (A, B, C) that BracketFinder would hand to LineSearch
// (lo = A, mid = B, hi = C, then sorted); false when the SearchInterval is invalid or Brent stops at once.
STS_HD STS_FI bool brent_first_u(double A, double B, double C, double &u) {
    double lo = A, hi = C;
    if (lo > hi) { double t = lo; lo = hi; hi = t; }
    if (lo >= hi || B < lo || B > hi) return false;
    double a, b;
    if (lo < hi) { a = lo; b = hi; } else { a = hi; b = lo; }
    return brent_golden_u(a, b, B, u);
}

// Evaluations one CG iteration costs once the point is non-finite: every objective value is then NaN without a pass
// (PC_EVAL), so the iteration is value-independent -- the top-of-loop F(point), BracketFinder's f(0), f(1e-8) and
// f(xC) (`fC > fB` is false for NaN: the bracket closes at once on (0, 1e-8, xC)), Brent's f(mid) and its
// golden-section steps on [0, xC] (every comparison with NaN is false, so x stays at 1e-8 and the parabola is never
// taken) until the interval is below tolerance. tests/test_cglane_sim.py steps the machine to check the constant.
constexpr int kNanIterEvals = 77;

// The parameter count n = point.length of the optimizer: the conjugate-gradient restart period (`iter % n == 0`).
// KDim: the compile-time K of the order-specialised kernels (no storage); RuntimeDim: the runtime-order path
// (arima_generic.hip), whose lanes hold K = kGenMaxK padded coordinates of which the first kdim are the fit's --
// every other operation of the machine leaves zero padding exact (a dot product gains + 0.0 terms, a padded
// coordinate of a non-finite point is non-finite only when a real one is).
template <int K>
struct KDim {
    STS_HD STS_FI int dim() const { return K; }
};
struct RuntimeDim {
    int32_t kdim;
    STS_HD STS_FI int dim() const { return kdim; }
};

// NS: predicted alphas posted with one F request; NC: values cached per line search. FF: fast-forward the
// NaN-absorbing state in closed form (PC_TOP below); false only in the CPU simulator, to check kNanIterEvals.
template <int K, int NS_, int NC_, bool FF = true, class DimT = KDim<K>>
struct CGLane : DimT {
    static constexpr int NS = NS_;
    static constexpr int NC = NC_;
    static constexpr int NS1 = NS > 0 ? NS : 1;
    static constexpr int NC1 = NC > 0 ? NC : 1;
    // optimizer (NonLinearConjugateGradientOptimizer.doOptimize)
    double point[K], dir[K];
    double delta, memo_obj, prev_obj;
    // line search: BracketFinder and BrentOptimizer state (disjoint lifetimes)
    union {
        struct { double xA, xB, xC, fA, fB, fC, w, fW; };
        struct { double a, b, bx, bv, bw, bd, be, fx, fv, fw, u, prev_x, prev_f, cur_x, cur_f, best_x, best_f; };
    };
    double ev_alpha;                       // pending objective request: point + ev_alpha * dir
    double sp_alpha[NC1], sp_f[NC1];       // speculative values of the current line search
    double rq_spec[NS1];                   // predicted alphas of the posted request
    uint16_t n_eval, n_grad, iter, bcount, spec_hits;
    uint8_t pc, status, req, have_prev_obj, have_prev, sp_n, sp_next, rq_nspec;

    STS_HD STS_FI void start(const double (&init)[K]) {
#pragma unroll
        for (int i = 0; i < K; ++i) point[i] = init[i];
        pc = PC_START;
        status = ARIMA_ST_OK;
        n_eval = n_grad = iter = 0;
        have_prev_obj = 0;
        req = REQ_NONE;
        sp_n = sp_next = rq_nspec = 0;
        spec_hits = 0;
    }

    STS_HD STS_FI void fail(int st) {
        status = (uint8_t)st;
        pc = PC_DONE;
    }

    STS_HD STS_FI bool done() const { return pc == PC_DONE; }

    // coefficients of the posted request (the same expression PC_EVAL checks for finiteness)
    STS_HD STS_FI void request_point(double (&c)[K]) const {
        if (req == REQ_G) {
#pragma unroll
            for (int i = 0; i < K; ++i) c[i] = point[i];
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i) c[i] = point[i] + ev_alpha * dir[i];
        }
    }

    // coefficients of speculative chain h of the posted request (same expression as request_point)
    STS_HD STS_FI void spec_point(int h, double (&c)[K]) const {
        const double al = rq_spec[h];
#pragma unroll
        for (int i = 0; i < K; ++i) c[i] = point[i] + al * dir[i];
    }

    // value of speculative chain h of the served request (the objective at point + rq_spec[h] * dir)
    STS_HD STS_FI void spec_store(int h, double f) {
        if constexpr (NC > 0) {
            const int slot = sp_next;
            const double al = rq_spec[h];
#pragma unroll
            for (int s = 0; s < NC; ++s)            // static indices: the state can live in registers
                if (s == slot) {
                    sp_alpha[s] = al;
                    sp_f[s] = f;
                }
            sp_next = (uint8_t)(slot + 1 == NC ? 0 : slot + 1);
            if (sp_n < NC) sp_n++;
        }
    }

    // start() plus what advance() does at PC_START: post G at the initial point (a refill needs no advance call)
    STS_HD STS_FI void start_posted(const double (&init)[K]) {
        start(init);
        req = REQ_G;
        pc = PC_G0;
    }

  private:
    STS_HD STS_FI bool cached(double alpha) const {
        if constexpr (NC > 0) {
            const long long ab = dbits(alpha);
#pragma unroll
            for (int s = 0; s < NC; ++s)
                if (s < sp_n && dbits(sp_alpha[s]) == ab) return true;
        }
        return false;
    }

    STS_HD STS_FI void add_pred(int &cnt, double alpha) {
        if constexpr (NS > 0) {
            if (cnt >= NS || !finite(alpha) || dbits(alpha) == dbits(ev_alpha) || cached(alpha)) return;
#pragma unroll
            for (int h = 0; h < NS; ++h)
                if (h < cnt && dbits(rq_spec[h]) == dbits(alpha)) return;
#pragma unroll
            for (int h = 0; h < NS; ++h)
                if (h == cnt) rq_spec[h] = alpha;
            cnt++;
        }
    }

    // grow-limit chain from (bb, cc): wLim = bb + 100 (cc - bb), then (cc, wLim), ... (BracketFinder's
    // `(w - wLim) * (wLim - xC) >= 0` branch, taken while the objective keeps rising almost linearly)
    STS_HD STS_FI void add_chain(int &cnt, double bb, double cc) {
#pragma unroll
        for (int h = 0; h < NS; ++h) {
            const double nx = bb + kGrow * (cc - bb);
            add_pred(cnt, nx);
            bb = cc;
            cc = nx;
        }
    }

    STS_HD STS_FI void add_brent_u1(int &cnt, double A, double B, double C) {
        double uu;
        if (brent_first_u(A, B, C, uu)) add_pred(cnt, uu);
    }

    // predictions for the objective request resuming at `ret` (the state is the one at posting time)
    STS_HD STS_FI int predict(int ret) {
        int cnt = 0;
        if constexpr (NS > 0) {
            switch (ret) {
            case PC_BR_FB: {                        // f(xB): then xC (no swap: fA <= fB), then the wLim chain
                const double c0 = xB + kGold * (xB - xA);
                add_pred(cnt, c0);
                add_chain(cnt, xB, c0);
                break;
            }
            case PC_BR_FC:                          // f(xC): loop continues on the chain, or ends at (A, B, C)
                add_chain(cnt, xB, xC);
                add_brent_u1(cnt, xA, xB, xC);
                break;
            case PC_BR_SHIFT_EV:                    // f(w), then shift (A, B, C) <- (B, C, w)
                add_chain(cnt, xC, w);
                add_brent_u1(cnt, xB, xC, w);
                break;
            case PC_BR_A1:                          // w inside (B, C): fW > fC | fW < fB | golden extension
                add_brent_u1(cnt, xB, w, xC);
                add_brent_u1(cnt, xA, xB, w);
                add_pred(cnt, xC + kGold * (xC - xB));
                break;
            case PC_BR_C1: {                        // w beyond C: fW > fC -> golden extension w' from w (and the
                const double w2 = w + kGold * (w - xC);   // bracket (C, w, w') if f stops rising), else end at (B, C, w)
                add_pred(cnt, w2);
                add_brent_u1(cnt, xC, w, w2);
                add_brent_u1(cnt, xB, xC, w);
                break;
            }
            case PC_BRENT_FU:
                if (!have_prev) {                   // Brent's first u: its second step is golden for both outcomes
                    double uu;
                    {   // fu <= fx: x = u, the side of the old x becomes the bound
                        double aa = a, bbnd = b;
                        if (u < bx) bbnd = bx; else aa = bx;
                        if (brent_golden_u(aa, bbnd, u, uu)) add_pred(cnt, uu);
                    }
                    {   // fu > fx: x stays, u becomes the bound
                        double aa = a, bbnd = b;
                        if (u < bx) aa = u; else bbnd = u;
                        if (brent_golden_u(aa, bbnd, bx, uu)) add_pred(cnt, uu);
                    }
                }
                break;
            default:
                break;
            }
        }
        return cnt;
    }

  public:
    // Run the state machine until a request is posted (req != REQ_NONE) or the fit is finished. fr / gr are
    // the response to the request served last (objective; and the gradient for a G request).
    // out-of-line: the LDS-resident slots of the bulk kernel and the express path call it through a pointer
    STS_HD void advance(double fr, const double (&gr)[K]) { step(fr, gr); }

    // the state machine itself, force-inlined where the lane's state is a register-resident copy
    STS_HD STS_FI void step(double fr, const double (&gr)[K]) {
        const double GS = brent_gs();
        double ev_val = fr;                                   // objective value delivered to the resume point
        double grad[K];                                       // gradient delivered to PC_G0 / PC_G
#pragma unroll
        for (int i = 0; i < K; ++i) grad[i] = gr[i];
        // eval subroutine (LineSearch's objective): locals of this call, never live across a pass
        double ev_memo = 0.0;
        int ev_memo_ok = 0, ev_bracket = 0, ev_ret = PC_DONE;
        auto eval = [&](double alpha, int bracket, int memo_ok, double memo, int ret) {
            ev_alpha = alpha;
            ev_bracket = bracket;
            ev_memo_ok = memo_ok;
            ev_memo = memo;
            ev_ret = ret;
            pc = PC_EVAL;
        };
        for (;;) {
            switch (pc) {
            case PC_START:
                // r = computeObjectiveGradient(point)
                req = REQ_G;
                pc = PC_G0;
                return;
            case PC_G0: {
                n_grad++;
                double dl = 0.0;
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    dir[i] = grad[i];                     // steepestDescent = precondition(r) = r.clone()
                    dl = dl + grad[i] * dir[i];
                }
                delta = dl;
                memo_obj = ev_val;                        // F(point) fused into the gradient pass
                pc = PC_TOP;
                break;
            }
            case PC_TOP: {
                if constexpr (FF) {
                    // NaN-absorbing state: a non-finite coordinate makes every later evaluation
                    // NaN (point + alpha * dir is never finite), and with F(point) = NaN the convergence test is
                    // false, so the reference runs kNanIterEvals evaluations per iteration (one gradient each, at the
                    // end) until MaxEval. Jump there: the m iterations that still fit complete, the next one stops
                    // inside with MAX_EVAL at n_eval = kMaxEval (iter <= n_eval / 2, so MaxIter cannot come first).
                    // Failed fits report NaN coefficients, so the point itself no longer matters.
                    bool pfin = true;
#pragma unroll
                    for (int i = 0; i < K; ++i) pfin = pfin && finite(point[i]);
                    if (!pfin && __builtin_isnan(memo_obj)) {
                        const int m = (kMaxEval - (int)n_eval) / kNanIterEvals;
                        n_grad = (uint16_t)(n_grad + m);
                        iter = (uint16_t)(iter + m + 1);
                        n_eval = (uint16_t)kMaxEval;
                        fail(ARIMA_ST_MAX_EVAL);
                        return;
                    }
                }
                if (iter + 1 > kMaxIter) { fail(ARIMA_ST_MAX_ITER); return; }
                iter++;
                if (n_eval + 1 > kMaxEval) { fail(ARIMA_ST_MAX_EVAL); return; }
                n_eval++;
                const double objective = memo_obj;
                const bool conv = have_prev_obj && value_converged(prev_obj, objective, 1e-7, 1e-7);
                prev_obj = objective;
                have_prev_obj = 1;
                if (conv) { pc = PC_DONE; return; }   // status OK; point / prev_obj are the result
                // line.search(point, searchDirection)
                sp_n = sp_next = 0;
                bcount = 0;
                xA = 0.0;
                xB = 1e-8;
                bool dfin = true;
#pragma unroll
                for (int i = 0; i < K; ++i) dfin = dfin && finite(dir[i]);
                eval(xA, 1, dfin ? 1 : 0, objective, PC_BR_FA);
                break;
            }
            case PC_BR_FA:
                fA = ev_val;
                eval(xB, 1, 0, 0.0, PC_BR_FB);
                break;
            case PC_BR_FB: {
                fB = ev_val;
                if (fA > fB) {
                    double t = xA; xA = xB; xB = t;
                    t = fA; fA = fB; fB = t;
                }
                xC = xB + kGold * (xB - xA);
                eval(xC, 1, 0, 0.0, PC_BR_FC);
                break;
            }
            case PC_BR_FC:
                fC = ev_val;
                pc = PC_BR_LOOP;
                break;
            case PC_BR_LOOP: {
                if (!(fC > fB)) { pc = PC_BR_END; break; }
                const double tmp1 = (xB - xA) * (fB - fC);
                const double tmp2 = (xB - xC) * (fB - fA);
                const double val = tmp2 - tmp1;
                const double denom = dabs(val) < kEpsMin ? 2 * kEpsMin : val;
                w = xB - ((xB - xC) * tmp2 - (xB - xA) * tmp1) / (2 * denom);
                const double wLim = xB + kGrow * (xC - xB);
                if ((w - xC) * (xB - w) > 0) {
                    eval(w, 1, 0, 0.0, PC_BR_A1);
                } else if ((w - wLim) * (wLim - xC) >= 0) {
                    w = wLim;
                    eval(w, 1, 0, 0.0, PC_BR_SHIFT_EV);
                } else if ((w - wLim) * (xC - w) > 0) {
                    eval(w, 1, 0, 0.0, PC_BR_C1);
                } else {
                    w = xC + kGold * (xC - xB);
                    eval(w, 1, 0, 0.0, PC_BR_SHIFT_EV);
                }
                break;
            }
            case PC_BR_A1:
                fW = ev_val;
                if (fW > fC) {
                    xA = xB; xB = w; fA = fB; fB = fW;
                    pc = PC_BR_END;
                } else if (fW < fB) {
                    xC = w; fC = fW;
                    pc = PC_BR_END;
                } else {
                    w = xC + kGold * (xC - xB);
                    eval(w, 1, 0, 0.0, PC_BR_SHIFT_EV);
                }
                break;
            case PC_BR_C1:
                fW = ev_val;
                if (fW > fC) {
                    xB = xC; xC = w; w = xC + kGold * (xC - xB); fB = fC; fC = fW;
                    eval(w, 1, 0, 0.0, PC_BR_SHIFT_EV);
                } else {
                    pc = PC_BR_SHIFT;
                }
                break;
            case PC_BR_SHIFT_EV:
                fW = ev_val;
                pc = PC_BR_SHIFT;
                break;
            case PC_BR_SHIFT:
                xA = xB; fA = fB; xB = xC; fB = fC; xC = w; fC = fW;
                pc = PC_BR_LOOP;
                break;
            case PC_BR_END: {
                // bracket -> Brent (shared storage: read everything needed before writing)
                double lo = xA, hi = xC;
                const double mid = xB, fmid = fB;
                if (lo > hi) { double t = lo; lo = hi; hi = t; }
                if (lo >= hi || mid < lo || mid > hi) { fail(ARIMA_ST_BAD_INTERVAL); return; }  // SearchInterval
                if (lo < hi) { a = lo; b = hi; } else { a = hi; b = lo; }
                bx = bv = bw = mid;
                bd = be = 0.0;
                eval(mid, 0, 1, fmid, PC_BRENT_FX);                      // fx = f(mid) (memo: bracket fMid)
                break;
            }
            case PC_BRENT_FX:
                fx = -ev_val;
                fv = fw = fx;
                have_prev = 0;
                cur_x = bx; cur_f = -fx;
                best_x = cur_x; best_f = cur_f;
                pc = PC_BRENT_LOOP;
                break;
            case PC_BRENT_LOOP: {
                const double m = 0.5 * (a + b);
                const double tol1 = 1e-15 * dabs(bx) + kBrentAbs;
                const double tol2 = 2 * tol1;
                if (dabs(bx - m) <= tol2 - 0.5 * (b - a)) {
                    // return best(best, best(previous, current))
                    double ix = cur_x, iv = cur_f;
                    if (have_prev && prev_f >= cur_f) { ix = prev_x; iv = prev_f; }
                    if (!(best_f >= iv)) { best_x = ix; best_f = iv; }
                    pc = PC_LS_DONE;
                    break;
                }
                double p = 0, q = 0, r = 0;
                if (dabs(be) > tol1) {
                    r = (bx - bw) * (fx - fv);
                    q = (bx - bv) * (fx - fw);
                    p = (bx - bv) * q - (bx - bw) * r;
                    q = 2 * (q - r);
                    if (q > 0) p = -p; else q = -q;
                    r = be;
                    be = bd;
                    if (p > q * (a - bx) && p < q * (b - bx) && dabs(p) < dabs(0.5 * q * r)) {
                        bd = p / q;
                        u = bx + bd;
                        if (u - a < tol2 || b - u < tol2) bd = (bx <= m) ? tol1 : -tol1;
                    } else {
                        be = (bx < m) ? b - bx : a - bx;
                        bd = GS * be;
                    }
                } else {
                    be = (bx < m) ? b - bx : a - bx;
                    bd = GS * be;
                }
                if (dabs(bd) < tol1) u = (bd >= 0) ? bx + tol1 : bx - tol1;
                else u = bx + bd;
                eval(u, 0, 0, 0.0, PC_BRENT_FU);
                break;
            }
            case PC_BRENT_FU: {
                const double fu = -ev_val;
                prev_x = cur_x; prev_f = cur_f; have_prev = 1;
                cur_x = u; cur_f = ev_val;
                {
                    double ix = cur_x, iv = cur_f;
                    if (prev_f >= cur_f) { ix = prev_x; iv = prev_f; }
                    if (!(best_f >= iv)) { best_x = ix; best_f = iv; }
                }
                if (value_converged(prev_f, cur_f, 1e-8, 1e-8)) { pc = PC_LS_DONE; break; }
                if (fu <= fx) {
                    if (u < bx) b = bx; else a = bx;
                    bv = bw; fv = fw; bw = bx; fw = fx; bx = u; fx = fu;
                } else {
                    if (u < bx) a = u; else b = u;
                    if (fu <= fw || prec_equals(bw, bx)) { bv = bw; fv = fw; bw = u; fw = fu; }
                    else if (fu <= fv || prec_equals(bv, bx) || prec_equals(bv, bw)) { bv = u; fv = fu; }
                }
                pc = PC_BRENT_LOOP;
                break;
            }
            case PC_LS_DONE: {
                // point[i] += step * searchDirection[i]; r = computeObjectiveGradient(point)
                const double step = best_x;
                memo_obj = best_f;                    // F(point) == Brent's value at `step`
                bool pfin = true;
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    point[i] = point[i] + step * dir[i];
                    pfin = pfin && finite(point[i]);
                }
                if (!pfin) {                          // the gradient at a non-finite point is NaN: no pass
#pragma unroll
                    for (int i = 0; i < K; ++i) grad[i] = __builtin_nan("");
                    pc = PC_G;
                    break;
                }
                req = REQ_G;
                pc = PC_G;
                return;
            }
            case PC_G: {
                n_grad++;
                const double deltaOld = delta;
                double dl = 0.0;
#pragma unroll
                for (int i = 0; i < K; ++i) dl = dl + grad[i] * grad[i];
                delta = dl;
                const double beta = delta / deltaOld;       // FLETCHER_REEVES
                if (iter % this->dim() == 0 || beta < 0) {
#pragma unroll
                    for (int i = 0; i < K; ++i) dir[i] = grad[i];
                } else {
#pragma unroll
                    for (int i = 0; i < K; ++i) dir[i] = grad[i] + beta * dir[i];
                }
                pc = PC_TOP;
                break;
            }
            case PC_EVAL: {
                if (ev_bracket) {
                    if (bcount + 1 > kBracketMax) { fail(ARIMA_ST_BRACKET_MAX_EVAL); return; }
                    bcount++;
                }
                if (n_eval + 1 > kMaxEval) { fail(ARIMA_ST_MAX_EVAL); return; }
                n_eval++;
                if (ev_memo_ok) { ev_val = ev_memo; pc = ev_ret; break; }
                bool fin = true;
#pragma unroll
                for (int i = 0; i < K; ++i) fin = fin && finite(point[i] + ev_alpha * dir[i]);
                if (!fin) { ev_val = __builtin_nan(""); pc = ev_ret; break; }
                if constexpr (NC > 0) {
                    const long long ab = dbits(ev_alpha);
                    bool hit = false;
#pragma unroll
                    for (int s = 0; s < NC; ++s)
                        if (s < sp_n && dbits(sp_alpha[s]) == ab) { ev_val = sp_f[s]; hit = true; }
                    if (hit) { spec_hits++; pc = ev_ret; break; }
                }
                rq_nspec = (uint8_t)predict(ev_ret);
                req = REQ_F;
                pc = (uint8_t)ev_ret;                  // resume point once the response arrives
                return;
            }
            case PC_DONE:
            default:
                return;
            }
        }
    }
};

}  // namespace sts
