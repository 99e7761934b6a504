#pragma once
// arima_bobyqa_impl.hpp — css-bobyqa on the device (templates; kernels instantiated per dimension in
// arima_bobyqa_k<K>.hip, dispatched from arima_bobyqa.hip): ARIMA.fitWithCSSBOBYQA (ARIMA.scala:130-160) over a batch.
//
// The reference runs commons-math3 3.4.1's BOBYQAOptimizer (a Java translation of M.J.D. Powell's BOBYQA, 2009) with
// npt = 2k + 1, rhobeg = min(0.96, 0.2 * max|init|), rhoend = 1e-6 * rhobeg, unbounded, maximising
// logLikelihoodCSSARMA, MaxEval(10000). k_bobyqa_fit gives every series a lane that runs Powell's routines (PRELIM,
// BOBYQB, TRSBOX, ALTMOV, UPDATE, RESCUE) for that configuration in their published operation order -- with infinite
// bounds every bound test is inactive -- and evaluates the objective by streaming its own row (bq_css_ll: the CSS
// recursion of ARIMA.scala:430-445 / 581-618, css_pass's operations). The interpolation state (XPT, BMAT, ZMAT, the
// quadratic model: 2.9 KB at k = 5, 6 KB at k = 8) is a BqState<k>. RESCUE (bobyqb label 190) follows the oracle's
// bq_rescue (oracle/bobyqa_oracle.c). Two layouts, bit-identical: a lane per series (the state in private memory;
// lanes diverge, every series takes its own trust-region path) for large batches, and a wave per series (the state in
// LDS, the wave's lanes run one series' uniform code: no divergence, LDS instead of scratch latency) for small batches
// and autoFit's retries, whose time is set by their slowest series.
#include <algorithm>

#include "arima_device.hpp"
#include "arima_launch.hpp"

namespace sts {

#define BQ_KMAX 11
// row-major interpolation matrices with the dimension's own stride (every routine is templated on it, NN)
#define BQ_S (NN > 0 ? NN : 1)
#define XPT(k, j) xpt[(k) * BQ_S + (j)]
#define BMAT(i, j) bmat[(i) * BQ_S + (j)]
#define ZMAT(k, j) zmat[(k) * BQ_S + (j)]

// One fit's BOBYQA state for dimension NN (npt = 2 NN + 1 interpolation points, ndim = npt + NN): in the lane's
// private memory (k_bobyqa_fit: a lane per series) or in LDS (k_bobyqa_fit_wave: a wave per series).
template <int NN>
struct BqState {
    static constexpr int N1 = NN > 0 ? NN : 1, NPT = 2 * N1 + 1, NDIM = NPT + N1;
    double xbase[N1], xpt[NPT * N1], fval[NPT], xopt[N1], gopt[N1], hq[N1 * (N1 + 1) / 2], pq[NPT], bmat[NDIM * N1],
        zmat[NPT * N1], sl[N1], su[N1], xnew[N1], xalt[N1], d[N1], vlag[NDIM], w[3 * NDIM], x[N1], tw[5 * N1],
        par[2 * NDIM];                             // the wave layout's per-index temporaries
};

// for i in [0, count): f(i), independent bodies. Wave layout: lane i (i < count, strided by 64) runs body i, then
// the wave's LDS writes are complete before any lane reads them (one wave per workgroup: a cheap barrier). Lane
// layout: the serial loop. Each body runs the serial code's operations for its index in their order, so every
// value is the serial loop's bit for bit.
template <bool WAVE, class F>
__device__ __forceinline__ void bq_par(int count, F &&f) {
    if constexpr (WAVE) {
        for (int i = (int)(threadIdx.x & 63); i < count; i += 64) f(i);
        __syncthreads();
    } else {
        for (int i = 0; i < count; i++) f(i);
    }
}

template <bool WAVE>
__device__ __forceinline__ void bq_sync() {        // uniform LDS writes before other lanes read them
    if constexpr (WAVE) __syncthreads();
}

// logLikelihoodCSSARMA (ARIMA.scala:430-445, iterateARMA :581-618, updateMAErrors :544-554) at runtime orders
// p, q <= 5: the operations of css_pass in the same order (dest = 0 + I * c0, + AR lags, + MA terms; the ascending
// maTerms copy leaves [e_{t-1}, e_{t-2}, e_{t-2}, ...]; css folded left; Int -n/2)
__device__ double bq_css_ll(const double *__restrict__ row, int n, int p, int q, int I, const double *c) {
    if (p > 5 || q > 5) {                          // the runtime-order path's recursion (arima_device.hpp gen_css)
        double cg[BQ_KMAX];
        for (int j = 0; j < BQ_KMAX; ++j) cg[j] = (j < I + p + q) ? c[j] : 0.0;
        return css_to_loglik(gen_css(GRow{row, 0}, n, p, q, I, cg), n);
    }
    const int M = p > q ? p : q;
    double yl[5], ma[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        yl[j] = (j < p) ? row[M - 1 - j] : 0.0;
        ma[j] = 0.0;
    }
    double cc[11];
#pragma unroll
    for (int j = 0; j < 11; ++j) cc[j] = (j < I + p + q) ? c[j] : 0.0;
    double ar[5], mc[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        double a = 0.0, m = 0.0;
#pragma unroll
        for (int t = 0; t < 11; ++t) {
            a = (t == I + j) ? cc[t] : a;
            m = (t == I + p + j) ? cc[t] : m;
        }
        ar[j] = a;
        mc[j] = m;
    }
    const double c0 = cc[0];
    double css = 0.0;
    if (M < n) {
        stream_elems<2>(row, M, n, [&](double yi) {
            double dest = 0.0;
            dest = dest + (double)I * c0;
#pragma unroll
            for (int j = 0; j < 5; ++j)
                if (j < p) dest = dest + yl[j] * ar[j];
#pragma unroll
            for (int j = 0; j < 5; ++j)
                if (j < q) dest = dest + ma[j] * mc[j];
            const double err = yi - dest;
#pragma unroll
            for (int j = 4; j >= 1; --j)
                if (j < q) ma[j] = ma[0];
            if (q > 0) ma[0] = err;
            const double r = yi - dest;
            css = css + r * r;
#pragma unroll
            for (int j = 4; j >= 1; --j) yl[j] = yl[j - 1];
            yl[0] = yi;
        });
    }
    return css_to_loglik(css, n);
}

// The same log-likelihood through css_pass (the css-cgd fits' objective pass: compile-time orders, the lag windows
// in registers, no per-step moves), for the orders of dimension K = I + p + q; one lane, one chunk in flight
template <int P, int Q, int I>
__device__ __forceinline__ double bq_css_ll_t(const double *__restrict__ row, int n, const double *x) {
    constexpr int KA = I + P + Q > 0 ? I + P + Q : 1;
    double c[KA], g[KA], css;
#pragma unroll
    for (int j = 0; j < KA; ++j) c[j] = (j < I + P + Q) ? x[j] : 0.0;
    css_pass<P, Q, I, false, true, false, 1>(row, n, c, css, g);
    return css_to_loglik(css, n);
}

template <int K>
__device__ double bq_css_ll_k(const double *__restrict__ row, int n, int p, int q, int I, const double *x) {
#define BQ_CSS_CASE(P, Q, II)                                                                                         \
    case (P) * 12 + (Q) * 2 + (II):                                                                                   \
        if constexpr ((P) + (Q) + (II) == K) return bq_css_ll_t<P, Q, II>(row, n, x);                                 \
        break;
#define BQ_CSS_Q(P, Q) BQ_CSS_CASE(P, Q, 0) BQ_CSS_CASE(P, Q, 1)
#define BQ_CSS_P(P) BQ_CSS_Q(P, 0) BQ_CSS_Q(P, 1) BQ_CSS_Q(P, 2) BQ_CSS_Q(P, 3) BQ_CSS_Q(P, 4) BQ_CSS_Q(P, 5)
    switch (p * 12 + q * 2 + I) {
        BQ_CSS_P(0) BQ_CSS_P(1) BQ_CSS_P(2) BQ_CSS_P(3) BQ_CSS_P(4) BQ_CSS_P(5)
    default:
        break;
    }
#undef BQ_CSS_P
#undef BQ_CSS_Q
#undef BQ_CSS_CASE
    return bq_css_ll(row, n, p, q, I, x);          // unreachable for p, q <= 5 (the launchers' bounds)
}

struct BqObj {
    const double *y;
    int n, p, q, I;
    int n_eval, max_eval;
};

// BaseOptimizer.computeObjectiveValue: counts, throws (TooManyEvaluations) past MaxEval; f = -LL (MAXIMIZE)
template <int K>
__device__ __forceinline__ int bq_eval(BqObj *o, const double *x, double *f) {
    if (++o->n_eval > o->max_eval) return 0;
    *f = -bq_css_ll_k<K>(o->y, o->n, o->p, o->q, o->I, x);
    return 1;
}

/* commons FastMath.max / min (NaN-propagating; max(-0, +0) = +0, min(+0, -0) = -0) */
__device__ __forceinline__ double bq_jmax(double a, double b) {
    if (a > b) return a;
    if (a < b) return b;
    if (a != b) return __builtin_nan("");
    const unsigned long long bits = (unsigned long long)__double_as_longlong(a);
    return bits == 0x8000000000000000ull ? b : a;
}
__device__ __forceinline__ double bq_jmin(double a, double b) {
    if (a > b) return b;
    if (a < b) return a;
    if (a != b) return __builtin_nan("");
    const unsigned long long bits = (unsigned long long)__double_as_longlong(a);
    return bits == 0x8000000000000000ull ? a : b;
}

/* ---- TRSBOX (trust-region step of the quadratic model, bound tests inactive) ---------------------------- */
template <int NN, bool WAVE = false>
__device__ __forceinline__ void bq_trsbox(const double *xpt, const double *xopt, const double *gopt, const double *hq,
                      const double *pq, const double *sl, const double *su, double delta, double *xnew, double *d,
                      double *gnew, double *xbdi, double *s, double *hs, double *hred, double *dsq_out,
                      double *crvmin_out, double *par) {
    constexpr int n = NN, npt = 2 * NN + 1;
    int iterc = 0, nact = 0, itermax = 0, itcsav = 0, iact = 0, isav = 0, iu = 0;
    double beta = 0, stepsq = 0, gredsq = 0, delsq, qred, crvmin, resid, ds, shs, temp, blen, stplen, sdec, ggsav = 0;
    double dredsq = 0, dredg = 0, sredg = 0, angbd = 0, xsav = 0, dhs = 0, dhd = 0, redmax, redsav, rdprev = 0,
           rdnext = 0, angt = 0, sth, cth, rednew;
    for (int i = 0; i < n; i++) {
        xbdi[i] = 0.0;
        if (xopt[i] <= sl[i]) {
            if (gopt[i] >= 0.0) xbdi[i] = -1.0;
        } else if (xopt[i] >= su[i]) {
            if (gopt[i] <= 0.0) xbdi[i] = 1.0;
        }
        if (xbdi[i] != 0.0) nact++;
        d[i] = 0.0;
        gnew[i] = gopt[i];
    }
    delsq = delta * delta;
    qred = 0.0;
    crvmin = -1.0;
    int state = 20;
    for (;;) {
        switch (state) {
        case 20:
            beta = 0.0;
            /* fallthrough */
        case 30:
            stepsq = 0.0;
            for (int i = 0; i < n; i++) {
                if (xbdi[i] != 0.0) s[i] = 0.0;
                else if (beta == 0.0) s[i] = -gnew[i];
                else s[i] = beta * s[i] - gnew[i];
                stepsq = stepsq + s[i] * s[i];
            }
            if (stepsq == 0.0) { state = 190; break; }
            if (beta == 0.0) {
                gredsq = stepsq;
                itermax = iterc + n - nact;
            }
            if (gredsq * delsq <= 1.0e-4 * qred * qred) { state = 190; break; }
            state = 210;
            break;
        case 50:
            resid = delsq;
            ds = 0.0;
            shs = 0.0;
            for (int i = 0; i < n; i++) {
                if (xbdi[i] == 0.0) {
                    resid = resid - d[i] * d[i];
                    ds = ds + s[i] * d[i];
                    shs = shs + s[i] * hs[i];
                }
            }
            if (resid <= 0.0) { state = 90; break; }
            temp = sqrt(stepsq * resid + ds * ds);
            if (ds < 0.0) blen = (temp - ds) / stepsq;
            else blen = resid / (temp + ds);
            stplen = blen;
            if (shs > 0.0) stplen = bq_jmin(blen, gredsq / shs);
            iact = 0;
            for (int i = 0; i < n; i++) {
                if (s[i] != 0.0) {
                    const double xsum = xopt[i] + d[i];
                    if (s[i] > 0.0) temp = (su[i] - xsum) / s[i];
                    else temp = (sl[i] - xsum) / s[i];
                    if (temp < stplen) { stplen = temp; iact = i + 1; }
                }
            }
            sdec = 0.0;
            if (stplen > 0.0) {
                iterc++;
                temp = shs / stepsq;
                if (iact == 0 && temp > 0.0) {
                    crvmin = bq_jmin(crvmin, temp);
                    if (crvmin == -1.0) crvmin = temp;
                }
                ggsav = gredsq;
                gredsq = 0.0;
                for (int i = 0; i < n; i++) {
                    gnew[i] = gnew[i] + stplen * hs[i];
                    if (xbdi[i] == 0.0) gredsq = gredsq + gnew[i] * gnew[i];
                    d[i] = d[i] + stplen * s[i];
                }
                sdec = bq_jmax(stplen * (ggsav - 0.5 * stplen * shs), 0.0);
                qred = qred + sdec;
            }
            if (iact > 0) {
                nact++;
                xbdi[iact - 1] = 1.0;
                if (s[iact - 1] < 0.0) xbdi[iact - 1] = -1.0;
                delsq = delsq - d[iact - 1] * d[iact - 1];
                if (delsq <= 0.0) { state = 90; break; }
                state = 20;
                break;
            }
            if (stplen < blen) {
                if (iterc == itermax) { state = 190; break; }
                if (sdec <= 0.01 * qred) { state = 190; break; }
                beta = gredsq / ggsav;
                state = 30;
                break;
            }
            /* fallthrough */
        case 90:
            crvmin = 0.0;
            /* fallthrough */
        case 100:
            if (nact >= n - 1) { state = 190; break; }
            dredsq = 0.0;
            dredg = 0.0;
            gredsq = 0.0;
            for (int i = 0; i < n; i++) {
                if (xbdi[i] == 0.0) {
                    dredsq = dredsq + d[i] * d[i];
                    dredg = dredg + d[i] * gnew[i];
                    gredsq = gredsq + gnew[i] * gnew[i];
                    s[i] = d[i];
                } else {
                    s[i] = 0.0;
                }
            }
            itcsav = iterc;
            state = 210;
            break;
        case 120:
            iterc++;
            temp = gredsq * dredsq - dredg * dredg;
            if (temp <= 1.0e-4 * qred * qred) { state = 190; break; }
            temp = sqrt(temp);
            for (int i = 0; i < n; i++) {
                if (xbdi[i] == 0.0) s[i] = (dredg * d[i] - dredsq * gnew[i]) / temp;
                else s[i] = 0.0;
            }
            sredg = -temp;
            angbd = 1.0;
            iact = 0;
            {
                int back = 0;
                for (int i = 0; i < n; i++) {
                    if (xbdi[i] == 0.0) {
                        const double tempa = xopt[i] + d[i] - sl[i];
                        const double tempb = su[i] - xopt[i] - d[i];
                        if (tempa <= 0.0) { nact++; xbdi[i] = -1.0; back = 1; break; }
                        else if (tempb <= 0.0) { nact++; xbdi[i] = 1.0; back = 1; break; }
                        const double ssq = d[i] * d[i] + s[i] * s[i];
                        temp = ssq - (xopt[i] - sl[i]) * (xopt[i] - sl[i]);
                        if (temp > 0.0) {
                            temp = sqrt(temp) - s[i];
                            if (angbd * temp > tempa) { angbd = tempa / temp; iact = i + 1; xsav = -1.0; }
                        }
                        temp = ssq - (su[i] - xopt[i]) * (su[i] - xopt[i]);
                        if (temp > 0.0) {
                            temp = sqrt(temp) + s[i];
                            if (angbd * temp > tempb) { angbd = tempb / temp; iact = i + 1; xsav = 1.0; }
                        }
                    }
                }
                if (back) { state = 100; break; }
            }
            state = 210;
            break;
        case 150:
            shs = 0.0;
            dhs = 0.0;
            dhd = 0.0;
            for (int i = 0; i < n; i++) {
                if (xbdi[i] == 0.0) {
                    shs = shs + s[i] * hs[i];
                    dhs = dhs + d[i] * hs[i];
                    dhd = dhd + d[i] * hred[i];
                }
            }
            redmax = 0.0;
            isav = 0;
            redsav = 0.0;
            iu = (int)(17.0 * angbd + 3.1);
            for (int i = 1; i <= iu; i++) {
                angt = angbd * (double)i / (double)iu;
                sth = (angt + angt) / (1.0 + angt * angt);
                temp = shs + angt * (angt * dhd - dhs - dhs);
                rednew = sth * (angt * dredg - sredg - 0.5 * sth * temp);
                if (rednew > redmax) {
                    redmax = rednew;
                    isav = i;
                    rdprev = redsav;
                } else if (i == isav + 1) {
                    rdnext = rednew;
                }
                redsav = rednew;
            }
            if (isav == 0) { state = 190; break; }
            if (isav < iu) {
                temp = (rdnext - rdprev) / (redmax + redmax - rdprev - rdnext);
                angt = angbd * ((double)isav + 0.5 * temp) / (double)iu;
            }
            cth = (1.0 - angt * angt) / (1.0 + angt * angt);
            sth = (angt + angt) / (1.0 + angt * angt);
            temp = shs + angt * (angt * dhd - dhs - dhs);
            sdec = sth * (angt * dredg - sredg - 0.5 * sth * temp);
            if (sdec <= 0.0) { state = 190; break; }
            dredg = 0.0;
            gredsq = 0.0;
            for (int i = 0; i < n; i++) {
                gnew[i] = gnew[i] + (cth - 1.0) * hred[i] + sth * hs[i];
                if (xbdi[i] == 0.0) {
                    d[i] = cth * d[i] + sth * s[i];
                    dredg = dredg + d[i] * gnew[i];
                    gredsq = gredsq + gnew[i] * gnew[i];
                }
                hred[i] = cth * hred[i] + sth * hs[i];
            }
            qred = qred + sdec;
            if (iact > 0 && isav == iu) {
                nact++;
                xbdi[iact - 1] = xsav;
                state = 100;
                break;
            }
            if (sdec > 0.01 * qred) { state = 120; break; }
            state = 190;
            break;
        case 190: {
            double dsq = 0.0;
            for (int i = 0; i < n; i++) {
                xnew[i] = bq_jmax(bq_jmin(xopt[i] + d[i], su[i]), sl[i]);
                if (xbdi[i] == -1.0) xnew[i] = sl[i];
                if (xbdi[i] == 1.0) xnew[i] = su[i];
                d[i] = xnew[i] - xopt[i];
                dsq = dsq + d[i] * d[i];
            }
            *dsq_out = dsq;
            *crvmin_out = crvmin;
            return;
        }
        case 210: {
            /* HS = (second-derivative matrix of Q) * S */
            int ih = 0;
            for (int j = 0; j < n; j++) {
                hs[j] = 0.0;
                for (int i = 0; i <= j; i++) {
                    if (i < j) hs[j] = hs[j] + hq[ih] * s[i];
                    hs[i] = hs[i] + hq[ih] * s[j];
                    ih++;
                }
            }
            bq_sync<WAVE>();
            if constexpr (WAVE) {                // per-point scalars by lane k, then hs[i] folded over k by lane i
                bq_par<true>(npt, [&](int k) {
                    if (pq[k] != 0.0) {
                        double t = 0.0;
                        for (int j = 0; j < n; j++) t = t + XPT(k, j) * s[j];
                        par[k] = t * pq[k];
                    }
                });
                bq_par<true>(n, [&](int i) {
                    double h = hs[i];
                    for (int k = 0; k < npt; k++)
                        if (pq[k] != 0.0) h = h + par[k] * XPT(k, i);
                    hs[i] = h;
                });
            } else {
                for (int k = 0; k < npt; k++) {
                    if (pq[k] != 0.0) {
                        temp = 0.0;
                        for (int j = 0; j < n; j++) temp = temp + XPT(k, j) * s[j];
                        temp = temp * pq[k];
                        for (int i = 0; i < n; i++) hs[i] = hs[i] + temp * XPT(k, i);
                    }
                }
            }
            if (crvmin != 0.0) { state = 50; break; }
            if (iterc > itcsav) { state = 150; break; }
            for (int i = 0; i < n; i++) hred[i] = hs[i];
            state = 120;
            break;
        }
        default:
            return;
        }
    }
}

/* ---- ALTMOV (alternative positions of the KNEW-th point, bound tests inactive) --------------------------- */
template <int NN>
__device__ __forceinline__ void bq_altmov(const double *xpt, const double *xopt, const double *bmat, const double *zmat,
                      const double *sl, const double *su, int kopt, int knew, double adelt, double *xnew,
                      double *xalt, double *alpha_out, double *cauchy_out, double *glag, double *hcol, double *w) {
    constexpr int n = NN, npt = 2 * NN + 1;
    const int nptm = npt - n - 1;
    const double cnst = 1.0 + sqrt(2.0);
    double temp, alpha, ha, presav, step = 0, vlag, stpsav = 0, cauchy = 0, csave = 0, ggfree, wfixsq, wsqsav, gw,
                                    curv, scale, bigstp, tempa, tempb;
    int ksav = 0, ibdsav = 0, iflag;
    for (int k = 0; k < npt; k++) hcol[k] = 0.0;
    for (int j = 0; j < nptm; j++) {
        temp = ZMAT(knew, j);
        for (int k = 0; k < npt; k++) hcol[k] = hcol[k] + temp * ZMAT(k, j);
    }
    alpha = hcol[knew];
    ha = 0.5 * alpha;
    for (int i = 0; i < n; i++) glag[i] = BMAT(knew, i);
    for (int k = 0; k < npt; k++) {
        temp = 0.0;
        for (int j = 0; j < n; j++) temp = temp + XPT(k, j) * xopt[j];
        temp = hcol[k] * temp;
        for (int i = 0; i < n; i++) glag[i] = glag[i] + temp * XPT(k, i);
    }
    presav = 0.0;
    for (int k = 0; k < npt; k++) {
        if (k == kopt) continue;
        double dderiv = 0.0, distsq = 0.0;
        for (int i = 0; i < n; i++) {
            temp = XPT(k, i) - xopt[i];
            dderiv = dderiv + glag[i] * temp;
            distsq = distsq + temp * temp;
        }
        double subd = adelt / sqrt(distsq);
        double slbd = -subd;
        int ilbd = 0, iubd = 0, isbd;
        const double sumin = bq_jmin(1.0, subd);
        for (int i = 0; i < n; i++) {
            temp = XPT(k, i) - xopt[i];
            if (temp > 0.0) {
                if (slbd * temp < sl[i] - xopt[i]) { slbd = (sl[i] - xopt[i]) / temp; ilbd = -(i + 1); }
                if (subd * temp > su[i] - xopt[i]) { subd = bq_jmax(sumin, (su[i] - xopt[i]) / temp); iubd = i + 1; }
            } else if (temp < 0.0) {
                if (slbd * temp > su[i] - xopt[i]) { slbd = (su[i] - xopt[i]) / temp; ilbd = i + 1; }
                if (subd * temp < sl[i] - xopt[i]) { subd = bq_jmax(sumin, (sl[i] - xopt[i]) / temp); iubd = -(i + 1); }
            }
        }
        if (k == knew) {
            const double diff = dderiv - 1.0;
            step = slbd;
            vlag = slbd * (dderiv - slbd * diff);
            isbd = ilbd;
            temp = subd * (dderiv - subd * diff);
            if (fabs(temp) > fabs(vlag)) { step = subd; vlag = temp; isbd = iubd; }
            const double tempd = 0.5 * dderiv;
            tempa = tempd - diff * slbd;
            tempb = tempd - diff * subd;
            if (tempa * tempb < 0.0) {
                temp = tempd * tempd / diff;
                if (fabs(temp) > fabs(vlag)) { step = tempd / diff; vlag = temp; isbd = 0; }
            }
        } else {
            step = slbd;
            vlag = slbd * (1.0 - slbd);
            isbd = ilbd;
            temp = subd * (1.0 - subd);
            if (fabs(temp) > fabs(vlag)) { step = subd; vlag = temp; isbd = iubd; }
            if (subd > 0.5) {
                if (fabs(vlag) < 0.25) { step = 0.5; vlag = 0.25; isbd = 0; }
            }
            vlag = vlag * dderiv;
        }
        temp = step * (1.0 - step) * distsq;
        const double predsq = vlag * vlag * (vlag * vlag + ha * temp * temp);
        if (predsq > presav) { presav = predsq; ksav = k; stpsav = step; ibdsav = isbd; }
    }
    for (int i = 0; i < n; i++) {
        temp = xopt[i] + stpsav * (XPT(ksav, i) - xopt[i]);
        xnew[i] = bq_jmax(sl[i], bq_jmin(su[i], temp));
    }
    if (ibdsav < 0) xnew[-ibdsav - 1] = sl[-ibdsav - 1];
    if (ibdsav > 0) xnew[ibdsav - 1] = su[ibdsav - 1];
    bigstp = adelt + adelt;
    iflag = 0;
    for (;;) {
        wfixsq = 0.0;
        ggfree = 0.0;
        for (int i = 0; i < n; i++) {
            w[i] = 0.0;
            tempa = bq_jmin(xopt[i] - sl[i], glag[i]);
            tempb = bq_jmax(xopt[i] - su[i], glag[i]);
            if (tempa > 0.0 || tempb < 0.0) {
                w[i] = bigstp;
                ggfree = ggfree + glag[i] * glag[i];
            }
        }
        if (ggfree == 0.0) {
            cauchy = 0.0;
            break;
        }
        for (;;) {
            temp = adelt * adelt - wfixsq;
            if (temp > 0.0) {
                wsqsav = wfixsq;
                step = sqrt(temp / ggfree);
                ggfree = 0.0;
                for (int i = 0; i < n; i++) {
                    if (w[i] == bigstp) {
                        temp = xopt[i] - step * glag[i];
                        if (temp <= sl[i]) { w[i] = sl[i] - xopt[i]; wfixsq = wfixsq + w[i] * w[i]; }
                        else if (temp >= su[i]) { w[i] = su[i] - xopt[i]; wfixsq = wfixsq + w[i] * w[i]; }
                        else ggfree = ggfree + glag[i] * glag[i];
                    }
                }
                if (wfixsq > wsqsav && ggfree > 0.0) continue;
            }
            break;
        }
        gw = 0.0;
        for (int i = 0; i < n; i++) {
            if (w[i] == bigstp) {
                w[i] = -step * glag[i];
                xalt[i] = bq_jmax(sl[i], bq_jmin(su[i], xopt[i] + w[i]));
            } else if (w[i] == 0.0) {
                xalt[i] = xopt[i];
            } else if (glag[i] > 0.0) {
                xalt[i] = sl[i];
            } else {
                xalt[i] = su[i];
            }
            gw = gw + glag[i] * w[i];
        }
        curv = 0.0;
        for (int k = 0; k < npt; k++) {
            temp = 0.0;
            for (int j = 0; j < n; j++) temp = temp + XPT(k, j) * w[j];
            curv = curv + hcol[k] * temp * temp;
        }
        if (iflag == 1) curv = -curv;
        if (curv > -gw && curv < -cnst * gw) {
            scale = -gw / curv;
            for (int i = 0; i < n; i++) {
                temp = xopt[i] + scale * w[i];
                xalt[i] = bq_jmax(sl[i], bq_jmin(su[i], temp));
            }
            cauchy = (0.5 * gw * scale) * (0.5 * gw * scale);
        } else {
            cauchy = (gw + 0.5 * curv) * (gw + 0.5 * curv);
        }
        if (iflag == 0) {
            for (int i = 0; i < n; i++) {
                glag[i] = -glag[i];
                w[n + i] = xalt[i];
            }
            csave = cauchy;
            iflag = 1;
            continue;
        }
        if (csave > cauchy) {
            for (int i = 0; i < n; i++) xalt[i] = w[n + i];
            cauchy = csave;
        }
        break;
    }
    *alpha_out = alpha;
    *cauchy_out = cauchy;
}

/* ---- UPDATE (BMAT and ZMAT after moving the KNEW-th interpolation point) ---------------------------------- */
template <int NN, bool WAVE = false>
__device__ __forceinline__ void bq_update(double *bmat, double *zmat, double *vlag, double beta, double denom, int knew,
                      double *w, double *par) {
    constexpr int n = NN, npt = 2 * NN + 1;
    const int nptm = npt - n - 1;
    double ztest = 0.0, temp, tempa, tempb, alpha, tau;
    for (int k = 0; k < npt; k++)
        for (int j = 0; j < nptm; j++) ztest = bq_jmax(ztest, fabs(ZMAT(k, j)));
    ztest = 1.0e-20 * ztest;
    for (int j = 1; j < nptm; j++) {
        if (fabs(ZMAT(knew, j)) > ztest) {
            temp = sqrt(ZMAT(knew, 0) * ZMAT(knew, 0) + ZMAT(knew, j) * ZMAT(knew, j));
            tempa = ZMAT(knew, 0) / temp;
            tempb = ZMAT(knew, j) / temp;
            const double ta = tempa, tb = tempb;
            bq_par<WAVE>(npt, [&](int i) {
                const double t = ta * ZMAT(i, 0) + tb * ZMAT(i, j);
                ZMAT(i, j) = ta * ZMAT(i, j) - tb * ZMAT(i, 0);
                ZMAT(i, 0) = t;
            });
        }
        ZMAT(knew, j) = 0.0;
        bq_sync<WAVE>();
    }
    bq_par<WAVE>(npt, [&](int i) { w[i] = ZMAT(knew, 0) * ZMAT(i, 0); });
    alpha = w[knew];
    tau = vlag[knew];
    bq_sync<WAVE>();
    vlag[knew] = vlag[knew] - 1.0;
    temp = sqrt(denom);
    tempb = ZMAT(knew, 0) / temp;
    tempa = tau / temp;
    bq_sync<WAVE>();
    {
        const double ta = tempa, tb = tempb;
        bq_par<WAVE>(npt, [&](int i) { ZMAT(i, 0) = ta * ZMAT(i, 0) - tb * vlag[i]; });
    }
    for (int j = 0; j < n; j++) {
        const int jp = npt + j;
        const double wj = BMAT(knew, j);
        bq_sync<WAVE>();
        w[jp] = wj;
        const double ta = (alpha * vlag[jp] - tau * wj) / denom;
        const double tb = (-beta * wj - tau * vlag[jp]) / denom;
        bq_sync<WAVE>();
        bq_par<WAVE>(jp + 1, [&](int i) {
            BMAT(i, j) = BMAT(i, j) + ta * vlag[i] + tb * w[i];
            if (i >= npt) BMAT(jp, i - npt) = BMAT(i, j);
        });
    }
    (void)par;
}

/* ---- RESCUE, its first part (labels 10-250: no evaluations) -------------------------------------------------- *
 * Powell's RESCUE as bobyqa_oracle.c bq_rescue restates it, up to label 260: XBASE moves to XBASE + XOPT, the
 * provisional points along the coordinate directions (PTSAUX = ptsaux[2 j], ptsaux[2 j + 1]; PTSID = Powell's
 * encoded doubles) replace the interpolation set in BMAT / ZMAT, and the original points that keep the UPDATE
 * denominators healthy are reinstated. W(NDIM + k) = w[ndim + k]. bq_fit runs 260-340 (one evaluation per
 * provisional point left) in its own loop so the evaluations stay at its single evaluation site. Rare (a damaged
 * denominator): the scalar code, which every lane of a wave runs alike in the wave layout. */
template <int NN, bool WAVE = false>
__device__ __noinline__ void bq_rescue_setup(BqState<NN> &S, int kopt, double delta, double *ptsaux, double *ptsid) {
    constexpr int n = NN, npt = 2 * NN + 1, np = n + 1, nptm = npt - np, ndim = npt + n;
    const double sfrac = 0.5 / (double)np;
    double *xbase = S.xbase, *xpt = S.xpt, *xopt = S.xopt, *hq = S.hq, *pq = S.pq, *bmat = S.bmat, *zmat = S.zmat,
           *sl = S.sl, *su = S.su, *vlag = S.vlag, *w = S.w;
    double sumpq = 0.0, winc = 0.0;
    bq_sync<WAVE>();
    for (int k = 0; k < npt; k++) {                            /* 10-20 */
        double distsq = 0.0;
        for (int j = 0; j < n; j++) {
            XPT(k, j) = XPT(k, j) - xopt[j];
            distsq = distsq + XPT(k, j) * XPT(k, j);
        }
        sumpq = sumpq + pq[k];
        w[ndim + k] = distsq;
        winc = bq_jmax(winc, distsq);
        for (int j = 0; j < nptm; j++) ZMAT(k, j) = 0.0;
    }
    {                                                          /* 30-40 */
        int ih = 0;
        for (int j = 0; j < n; j++) {
            w[j] = 0.5 * sumpq * xopt[j];
            for (int k = 0; k < npt; k++) w[j] = w[j] + pq[k] * XPT(k, j);
            for (int i = 0; i <= j; i++) {
                hq[ih] = hq[ih] + w[i] * xopt[j] + w[j] * xopt[i];
                ih++;
            }
        }
    }
    for (int j = 0; j < n; j++) {                              /* 50 */
        xbase[j] = xbase[j] + xopt[j];
        sl[j] = sl[j] - xopt[j];
        su[j] = su[j] - xopt[j];
        xopt[j] = 0.0;
        ptsaux[2 * j] = bq_jmin(delta, su[j]);
        ptsaux[2 * j + 1] = bq_jmax(-delta, sl[j]);
        if (ptsaux[2 * j] + ptsaux[2 * j + 1] < 0.0) {
            const double temp = ptsaux[2 * j];
            ptsaux[2 * j] = ptsaux[2 * j + 1];
            ptsaux[2 * j + 1] = temp;
        }
        if (fabs(ptsaux[2 * j + 1]) < 0.5 * fabs(ptsaux[2 * j])) ptsaux[2 * j + 1] = 0.5 * ptsaux[2 * j];
        for (int i = 0; i < ndim; i++) BMAT(i, j) = 0.0;
    }
    ptsid[0] = sfrac;                                          /* 60 (70: nothing left for npt = 2n + 1) */
    for (int j = 0; j < n; j++) {
        const int jp = j + 1, jpn = jp + n;
        ptsid[jp] = (double)(j + 1) + sfrac;
        ptsid[jpn] = (double)(j + 1) / (double)np + sfrac;
        const double temp = 1.0 / (ptsaux[2 * j] - ptsaux[2 * j + 1]);
        BMAT(jp, j) = -temp + 1.0 / ptsaux[2 * j];
        BMAT(jpn, j) = temp + 1.0 / ptsaux[2 * j + 1];
        BMAT(0, j) = -BMAT(jp, j) - BMAT(jpn, j);
        ZMAT(0, j) = sqrt(2.0) / fabs(ptsaux[2 * j] * ptsaux[2 * j + 1]);
        ZMAT(jp, j) = ZMAT(0, j) * ptsaux[2 * j + 1] * temp;
        ZMAT(jpn, j) = -ZMAT(0, j) * ptsaux[2 * j] * temp;
    }
    int nrem = npt, kold = 0, knew = kopt;
    double beta = 0.0, denom = 0.0;
    for (;;) {
        for (int j = 0; j < n; j++) {                          /* 80-110 */
            const double temp = BMAT(kold, j);
            BMAT(kold, j) = BMAT(knew, j);
            BMAT(knew, j) = temp;
        }
        for (int j = 0; j < nptm; j++) {
            const double temp = ZMAT(kold, j);
            ZMAT(kold, j) = ZMAT(knew, j);
            ZMAT(knew, j) = temp;
        }
        ptsid[kold] = ptsid[knew];
        ptsid[knew] = 0.0;
        w[ndim + knew] = 0.0;
        nrem--;
        if (knew != kopt) {
            const double temp = vlag[kold];
            vlag[kold] = vlag[knew];
            vlag[knew] = temp;
            bq_sync<WAVE>();
            bq_update<NN, WAVE>(bmat, zmat, vlag, beta, denom, knew, w, S.par);
            bq_sync<WAVE>();
            if (nrem == 0) break;
            for (int k = 0; k < npt; k++) w[ndim + k] = fabs(w[ndim + k]);
        }
        bool reinstate = false;
        for (;;) {
            double dsqmin = 0.0;                               /* 120-130 */
            for (int k = 0; k < npt; k++) {
                if (w[ndim + k] > 0.0) {
                    if (dsqmin == 0.0 || w[ndim + k] < dsqmin) {
                        knew = k;
                        dsqmin = w[ndim + k];
                    }
                }
            }
            if (dsqmin == 0.0) break;
            for (int j = 0; j < n; j++) w[npt + j] = XPT(knew, j);   /* 140-160 */
            for (int k = 0; k < npt; k++) {
                double sum = 0.0;
                if (k == kopt) {
                } else if (ptsid[k] == 0.0) {
                    for (int j = 0; j < n; j++) sum = sum + w[npt + j] * XPT(k, j);
                } else {
                    const int ip = (int)ptsid[k];
                    if (ip > 0) sum = w[npt + ip - 1] * ptsaux[2 * (ip - 1)];
                    const int iq = (int)((double)np * ptsid[k] - (double)(ip * np));
                    if (iq > 0) {
                        const int iw = (ip == 0) ? 1 : 0;
                        sum = sum + w[npt + iq - 1] * ptsaux[2 * (iq - 1) + iw];
                    }
                }
                w[k] = 0.5 * sum * sum;
            }
            for (int k = 0; k < npt; k++) {                    /* 170-230 */
                double sum = 0.0;
                for (int j = 0; j < n; j++) sum = sum + BMAT(k, j) * w[npt + j];
                vlag[k] = sum;
            }
            beta = 0.0;
            for (int j = 0; j < nptm; j++) {
                double sum = 0.0;
                for (int k = 0; k < npt; k++) sum = sum + ZMAT(k, j) * w[k];
                beta = beta - sum * sum;
                for (int k = 0; k < npt; k++) vlag[k] = vlag[k] + sum * ZMAT(k, j);
            }
            double bsum = 0.0, distsq = 0.0;
            for (int j = 0; j < n; j++) {
                double sum = 0.0;
                for (int k = 0; k < npt; k++) sum = sum + BMAT(k, j) * w[k];
                const int jp = j + npt;
                bsum = bsum + sum * w[jp];
                for (int ip = npt; ip < ndim; ip++) sum = sum + BMAT(ip, j) * w[ip];
                bsum = bsum + sum * w[jp];
                vlag[jp] = sum;
                distsq = distsq + XPT(knew, j) * XPT(knew, j);
            }
            beta = 0.5 * distsq * distsq + beta - bsum;
            vlag[kopt] = vlag[kopt] + 1.0;
            denom = 0.0;                                       /* 240-250 */
            double vlmxsq = 0.0;
            for (int k = 0; k < npt; k++) {
                if (ptsid[k] != 0.0) {
                    double hdiag = 0.0;
                    for (int j = 0; j < nptm; j++) hdiag = hdiag + ZMAT(k, j) * ZMAT(k, j);
                    const double den = beta * hdiag + vlag[k] * vlag[k];
                    if (den > denom) {
                        kold = k;
                        denom = den;
                    }
                }
                vlmxsq = bq_jmax(vlmxsq, vlag[k] * vlag[k]);
            }
            if (denom <= 1.0e-2 * vlmxsq) {
                w[ndim + knew] = -w[ndim + knew] - winc;
                continue;
            }
            reinstate = true;
            break;
        }
        if (!reinstate) break;
    }
    bq_sync<WAVE>();
}

/* RESCUE 260-280 for provisional point kpt: fold PQ(kpt) into HQ, move XPT(kpt, .) to its new position; returns the
 * model's value there (VQUAD) */
template <int NN>
__device__ __forceinline__ double bq_rescue_point(BqState<NN> &S, int kpt, double fbase, const double *ptsaux,
                                                  const double *ptsid) {
    constexpr int n = NN, npt = 2 * NN + 1, np = n + 1;
    double *xpt = S.xpt, *hq = S.hq, *pq = S.pq, *gopt = S.gopt, *w = S.w;
    int ih = 0;
    for (int j = 0; j < n; j++) {
        w[j] = XPT(kpt, j);
        XPT(kpt, j) = 0.0;
        const double temp = pq[kpt] * w[j];
        for (int i = 0; i <= j; i++) {
            hq[ih] = hq[ih] + temp * w[i];
            ih++;
        }
    }
    pq[kpt] = 0.0;
    const int ip = (int)ptsid[kpt];
    const int iq = (int)((double)np * ptsid[kpt] - (double)(ip * np));
    double xp = 0.0, xq = 0.0;
    if (ip > 0) {
        xp = ptsaux[2 * (ip - 1)];
        XPT(kpt, ip - 1) = xp;
    }
    if (iq > 0) {
        xq = ptsaux[2 * (iq - 1)];
        if (ip == 0) xq = ptsaux[2 * (iq - 1) + 1];
        XPT(kpt, iq - 1) = xq;
    }
    double vquad = fbase;
    int ihp = 0;
    if (ip > 0) {
        ihp = (ip + ip * ip) / 2;
        vquad = vquad + xp * (gopt[ip - 1] + 0.5 * xp * hq[ihp - 1]);
    }
    if (iq > 0) {
        const int ihq = (iq + iq * iq) / 2;
        vquad = vquad + xq * (gopt[iq - 1] + 0.5 * xq * hq[ihq - 1]);
        if (ip > 0) {
            const int iw = (ihp > ihq ? ihp : ihq) - abs(ip - iq);
            vquad = vquad + xp * xq * hq[iw - 1];
        }
    }
    for (int k = 0; k < npt; k++) {
        double temp = 0.0;
        if (ip > 0) temp = temp + xp * XPT(k, ip - 1);
        if (iq > 0) temp = temp + xq * XPT(k, iq - 1);
        vquad = vquad + 0.5 * pq[k] * temp * temp;
    }
    return vquad;
}

/* RESCUE 300-340: F at provisional point kpt folded into GOPT / HQ / PQ; PTSID(kpt) = 0 */
template <int NN>
__device__ __forceinline__ void bq_rescue_fold(BqState<NN> &S, int kpt, double diff, const double *ptsaux,
                                               double *ptsid) {
    constexpr int n = NN, npt = 2 * NN + 1, np = n + 1, nptm = npt - np;
    double *hq = S.hq, *pq = S.pq, *gopt = S.gopt, *bmat = S.bmat, *zmat = S.zmat;
    for (int i = 0; i < n; i++) gopt[i] = gopt[i] + diff * BMAT(kpt, i);
    for (int k = 0; k < npt; k++) {
        double sum = 0.0;
        for (int j = 0; j < nptm; j++) sum = sum + ZMAT(k, j) * ZMAT(kpt, j);
        const double temp = diff * sum;
        if (ptsid[k] == 0.0) {
            pq[k] = pq[k] + temp;
        } else {
            const int kp = (int)ptsid[k];
            const int kq = (int)((double)np * ptsid[k] - (double)(kp * np));
            const int ihq = (kq * kq + kq) / 2;
            if (kp == 0) {
                hq[ihq - 1] = hq[ihq - 1] + temp * (ptsaux[2 * (kq - 1) + 1] * ptsaux[2 * (kq - 1) + 1]);
            } else {
                const int khp = (kp * kp + kp) / 2;
                hq[khp - 1] = hq[khp - 1] + temp * (ptsaux[2 * (kp - 1)] * ptsaux[2 * (kp - 1)]);
                if (kq > 0) {
                    hq[ihq - 1] = hq[ihq - 1] + temp * (ptsaux[2 * (kq - 1)] * ptsaux[2 * (kq - 1)]);
                    const int iw = (khp > ihq ? khp : ihq) - abs(kq - kp);
                    hq[iw - 1] = hq[iw - 1] + temp * ptsaux[2 * (kp - 1)] * ptsaux[2 * (kq - 1)];
                }
            }
        }
    }
    ptsid[kpt] = 0.0;
}

/* ---- BOBYQA driver + PRELIM + BOBYQB, unbounded, npt = 2n + 1 ------------------------------------------- *
 * Returns ARIMA_ST_*; x (in: the initial point, out: the optimum), n_eval_out = objective evaluations. */
template <int NN, bool WAVE = false>
__device__ __forceinline__ int bq_fit(const double *y, int len, int p, int q, int I, const double *x0, double *x_out,
                                      int *n_eval_out, BqState<NN> &S) {
    constexpr int n = NN;                                      /* = I + p + q (the launcher's instantiation) */
    *n_eval_out = 0;
    if (n < 2) return ARIMA_ST_TOO_FEW_PARAMS;                 /* BOBYQAOptimizer.setup: dimension >= 2 */
    constexpr int npt = 2 * n + 1, np = n + 1, nptm = npt - np, nh = (n * np) / 2, ndim = npt + n;
    /* math.min(0.96, 0.2 * initParams.map(math.abs).max) (:147): Scala's max is reduceLeft((x, y) => if (x >= y) x
     * else y) with IEEE comparisons, Java's Math.min(a, b) is (a <= b ? a : b) for a = 0.96 -- NaN propagates as there */
    double amax = fabs(x0[0]);
    for (int j = 1; j < n; j++) amax = (amax >= fabs(x0[j])) ? amax : fabs(x0[j]);
    const double r02 = 0.2 * amax;
    const double rhobeg = (0.96 <= r02) ? 0.96 : r02;
    const double rhoend = rhobeg * 1e-6;                       /* :148 */
    BqObj ob{y, len, p, q, I, 0, 10000};
    double *xbase = S.xbase, *xpt = S.xpt, *fval = S.fval, *xopt = S.xopt, *gopt = S.gopt, *hq = S.hq, *pq = S.pq,
           *bmat = S.bmat, *zmat = S.zmat, *sl = S.sl, *su = S.su, *xnew = S.xnew, *xalt = S.xalt, *d = S.d,
           *vlag = S.vlag, *w = S.w, *x = S.x, *tw = S.tw;
    for (int i = 0; i < BqState<NN>::NPT * BqState<NN>::N1; i++) xpt[i] = 0.0;
    for (int i = 0; i < BqState<NN>::NDIM * BqState<NN>::N1; i++) bmat[i] = 0.0;
    for (int i = 0; i < BqState<NN>::NPT * BqState<NN>::N1; i++) zmat[i] = 0.0;
    for (int j = 0; j < n; j++) {                              /* BOBYQA: SL = XL - X, SU = XU - X (unbounded) */
        x[j] = x0[j];
        sl[j] = -__builtin_inf();
        su[j] = __builtin_inf();
    }
    (void)ndim;
    /* ---- PRELIM ---- */
    const double rhosq = rhobeg * rhobeg;
    double fbeg = 0.0, stepa = 0.0, stepb = 0.0, f = 0.0;
    int kopt = 0, nf = 0;
    for (int j = 0; j < n; j++) {
        xbase[j] = x[j];
    }
    for (int ih = 0; ih < nh; ih++) hq[ih] = 0.0;
    for (int k = 0; k < npt; k++) pq[k] = 0.0;
    for (;;) {
        const int nfm = nf, nfx = nf - n;
        nf++;
        /* nfm <= 2n always (npt = 2n + 1) */
        if (nfm >= 1 && nfm <= n) {
            stepa = rhobeg;
            if (su[nfm - 1] == 0.0) stepa = -stepa;
            XPT(nf - 1, nfm - 1) = stepa;
        } else if (nfm > n) {
            stepa = XPT(nf - n - 1, nfx - 1);
            stepb = -rhobeg;
            if (sl[nfx - 1] == 0.0) stepb = bq_jmin(2.0 * rhobeg, su[nfx - 1]);
            if (su[nfx - 1] == 0.0) stepb = bq_jmax(-2.0 * rhobeg, sl[nfx - 1]);
            XPT(nf - 1, nfx - 1) = stepb;
        }
        for (int j = 0; j < n; j++) x[j] = xbase[j] + XPT(nf - 1, j);   /* min(max(XL, .), XU): unbounded */
        if (!bq_eval<NN>(&ob, x, &f)) { *n_eval_out = ob.n_eval - 1; return ARIMA_ST_MAX_EVAL; }
        fval[nf - 1] = f;
        if (nf == 1) {
            fbeg = f;
            kopt = 0;
        } else if (f < fval[kopt]) {
            kopt = nf - 1;
        }
        if (nf >= 2 && nf <= n + 1) {
            gopt[nfm - 1] = (f - fbeg) / stepa;
            if (npt < nf + n) {
                BMAT(0, nfm - 1) = -1.0 / stepa;
                BMAT(nf - 1, nfm - 1) = 1.0 / stepa;
                BMAT(npt + nfm - 1, nfm - 1) = -0.5 * rhosq;
            }
        } else if (nf >= n + 2) {
            const int ih = (nfx * (nfx + 1)) / 2 - 1;
            const double temp = (f - fbeg) / stepb;
            const double diff = stepb - stepa;
            hq[ih] = 2.0 * (temp - gopt[nfx - 1]) / diff;
            gopt[nfx - 1] = (gopt[nfx - 1] * stepb - temp * stepa) / diff;
            if (stepa * stepb < 0.0) {
                if (f < fval[nf - n - 1]) {
                    fval[nf - 1] = fval[nf - n - 1];
                    fval[nf - n - 1] = f;
                    if (kopt == nf - 1) kopt = nf - n - 1;
                    XPT(nf - n - 1, nfx - 1) = stepb;
                    XPT(nf - 1, nfx - 1) = stepa;
                }
            }
            BMAT(0, nfx - 1) = -(stepa + stepb) / (stepa * stepb);
            BMAT(nf - 1, nfx - 1) = -0.5 / XPT(nf - n - 1, nfx - 1);
            BMAT(nf - n - 1, nfx - 1) = -BMAT(0, nfx - 1) - BMAT(nf - 1, nfx - 1);
            ZMAT(0, nfx - 1) = sqrt(2.0) / (stepa * stepb);
            ZMAT(nf - 1, nfx - 1) = sqrt(0.5) / rhosq;
            ZMAT(nf - n - 1, nfx - 1) = -ZMAT(0, nfx - 1) - ZMAT(nf - 1, nfx - 1);
        }
        if (nf >= npt) break;
    }
    /* ---- BOBYQB ---- */
    double xoptsq = 0.0;
    for (int i = 0; i < n; i++) {
        xopt[i] = XPT(kopt, i);
        xoptsq = xoptsq + xopt[i] * xopt[i];
    }
    double fsave = fval[0];
    int kbase = 0;
    double rho = rhobeg, delta = rho;
    int nresc = nf, ntrits = 0, itest = 0, nfsav = nf, knew = 0, ksav;
    double diffa = 0.0, diffb = 0.0, diffc = 0.0, ratio = 0.0, dnorm = 0.0, dsq = 0.0, crvmin = 0.0, distsq = 0.0,
           adelt = 0.0, alpha = 0.0, cauchy = 0.0, beta = 0.0, denom = 0.0, vquad = 0.0, diff = 0.0, fopt, densav;
    int state = 20;
    int status = ARIMA_ST_OK;
    int rk = -1;                                               /* RESCUE's provisional point being evaluated */
    double rfbase = 0.0, rvquad = 0.0;
    // Every evaluation of BOBYQB happens at ONE point of the loop, after the lane's state machine has run to its next
    // evaluation request (state 360) or to its end: the lanes of a wave take different trust-region paths, and with the
    // evaluation inside the switch a wave paid one full CSS pass per lane per request (the lanes' requests fall on
    // different trips). Now the lanes reconverge before the pass and share it. Operation order per lane unchanged.
    for (;;) {
      while (state >= 0 && state != 360) {
        switch (state) {
        case 20:
            if (kopt != kbase) {
                int ih = 0;
                for (int j = 0; j < n; j++)
                    for (int i = 0; i <= j; i++) {
                        if (i < j) gopt[j] = gopt[j] + hq[ih] * xopt[i];
                        gopt[i] = gopt[i] + hq[ih] * xopt[j];
                        ih++;
                    }
                if (nf > npt) {
                    for (int k = 0; k < npt; k++) {
                        double temp = 0.0;
                        for (int j = 0; j < n; j++) temp = temp + XPT(k, j) * xopt[j];
                        temp = pq[k] * temp;
                        for (int i = 0; i < n; i++) gopt[i] = gopt[i] + temp * XPT(k, i);
                    }
                }
            }
            /* fallthrough */
        case 60:
            bq_trsbox<NN, WAVE>(xpt, xopt, gopt, hq, pq, sl, su, delta, xnew, d, tw, tw + n, tw + 2 * n, tw + 3 * n,
                      tw + 4 * n, &dsq, &crvmin, S.par);
            dnorm = bq_jmin(delta, sqrt(dsq));
            if (dnorm < 0.5 * rho) {
                ntrits = -1;
                distsq = (10.0 * rho) * (10.0 * rho);
                if (nf <= nfsav + 2) { state = 650; break; }
                const double errbig = bq_jmax(bq_jmax(diffa, diffb), diffc);
                const double frhosq = 0.125 * rho * rho;
                if (crvmin > 0.0 && errbig > frhosq * crvmin) { state = 650; break; }
                const double bdtol = errbig / rho;
                int go650 = 0;
                for (int j = 0; j < n; j++) {
                    double bdtest = bdtol;
                    if (xnew[j] == sl[j]) bdtest = tw[j];
                    if (xnew[j] == su[j]) bdtest = -tw[j];
                    if (bdtest < bdtol) {
                        double curv = hq[(j + 1 + (j + 1) * (j + 1)) / 2 - 1];
                        for (int k = 0; k < npt; k++) curv = curv + pq[k] * XPT(k, j) * XPT(k, j);
                        bdtest = bdtest + 0.5 * curv * rho;
                        if (bdtest < bdtol) { go650 = 1; break; }
                    }
                }
                state = go650 ? 650 : 680;
                break;
            }
            ntrits++;
            /* fallthrough */
        case 90:
            if (dsq <= 1.0e-3 * xoptsq) {
                const double fracsq = 0.25 * xoptsq;
                double sumpq = 0.0;
                for (int k = 0; k < npt; k++) {
                    sumpq = sumpq + pq[k];
                    double sum = -0.5 * xoptsq;
                    for (int i = 0; i < n; i++) sum = sum + XPT(k, i) * xopt[i];
                    w[npt + k] = sum;
                    const double temp = fracsq - 0.5 * sum;
                    for (int i = 0; i < n; i++) {
                        w[i] = BMAT(k, i);
                        vlag[i] = sum * XPT(k, i) + temp * xopt[i];
                        const int ip = npt + i;
                        for (int j = 0; j <= i; j++) BMAT(ip, j) = BMAT(ip, j) + w[i] * vlag[j] + vlag[i] * w[j];
                    }
                }
                for (int jj = 0; jj < nptm; jj++) {
                    double sumz = 0.0, sumw = 0.0;
                    for (int k = 0; k < npt; k++) {
                        sumz = sumz + ZMAT(k, jj);
                        vlag[k] = w[npt + k] * ZMAT(k, jj);
                        sumw = sumw + vlag[k];
                    }
                    for (int j = 0; j < n; j++) {
                        double sum = (fracsq * sumz - 0.5 * sumw) * xopt[j];
                        for (int k = 0; k < npt; k++) sum = sum + vlag[k] * XPT(k, j);
                        w[j] = sum;
                        for (int k = 0; k < npt; k++) BMAT(k, j) = BMAT(k, j) + sum * ZMAT(k, jj);
                    }
                    for (int i = 0; i < n; i++) {
                        const int ip = i + npt;
                        const double temp = w[i];
                        for (int j = 0; j <= i; j++) BMAT(ip, j) = BMAT(ip, j) + temp * w[j];
                    }
                }
                int ih = 0;
                for (int j = 0; j < n; j++) {
                    w[j] = -0.5 * sumpq * xopt[j];
                    for (int k = 0; k < npt; k++) {
                        w[j] = w[j] + pq[k] * XPT(k, j);
                        XPT(k, j) = XPT(k, j) - xopt[j];
                    }
                    for (int i = 0; i <= j; i++) {
                        hq[ih] = hq[ih] + w[i] * xopt[j] + xopt[i] * w[j];
                        BMAT(npt + i, j) = BMAT(npt + j, i);
                        ih++;
                    }
                }
                for (int i = 0; i < n; i++) {
                    xbase[i] = xbase[i] + xopt[i];
                    xnew[i] = xnew[i] - xopt[i];
                    sl[i] = sl[i] - xopt[i];
                    su[i] = su[i] - xopt[i];
                    xopt[i] = 0.0;
                }
                xoptsq = 0.0;
            }
            if (ntrits == 0) { state = 210; break; }
            state = 230;
            break;
        case 190:                                                  /* RESCUE (bobyqa_oracle.c bq_rescue) */
            nfsav = nf;
            kbase = kopt;
            rfbase = fval[kopt];
            bq_rescue_setup<NN, WAVE>(S, kopt, delta, tw, S.par);
            rk = -1;
            /* fallthrough */
        case 193:                                                  /* 260: the next provisional point left */
            rk++;
            while (rk < npt && S.par[rk] == 0.0) rk++;
            if (rk < npt) {
                rvquad = bq_rescue_point<NN>(S, rk, rfbase, tw, S.par);
                state = 360;                                       /* evaluated at XBASE + XPT(rk, .) */
                break;
            }
            rk = -1;
            bq_sync<WAVE>();
            /* XOPT now, in case of the branch to 720; GOPT's update follows the branch to 20 */
            xoptsq = 0.0;
            if (kopt != kbase) {
                for (int i = 0; i < n; i++) {
                    xopt[i] = XPT(kopt, i);
                    xoptsq = xoptsq + xopt[i] * xopt[i];
                }
            }
            nresc = nf;
            if (nfsav < nf) {
                nfsav = nf;
                state = 20;
                break;
            }
            if (ntrits > 0) { state = 60; break; }
            state = 210;
            break;
        case 194:                                                  /* RESCUE 290-340, after the evaluation */
            nf++;
            fval[rk] = f;
            if (f < fval[kopt]) kopt = rk;
            bq_rescue_fold<NN>(S, rk, f - rvquad, tw, S.par);
            state = 193;
            break;
        case 210:
            bq_altmov<NN>(xpt, xopt, bmat, zmat, sl, su, kopt, knew, adelt, xnew, xalt, &alpha, &cauchy, tw,
                      tw + n, w);
            for (int i = 0; i < n; i++) d[i] = xnew[i] - xopt[i];
            /* fallthrough */
        case 230: {
            bq_sync<WAVE>();
            bq_par<WAVE>(npt, [&](int k) {
                double suma = 0.0, sumb = 0.0, sum = 0.0;
                for (int j = 0; j < n; j++) {
                    suma = suma + XPT(k, j) * d[j];
                    sumb = sumb + XPT(k, j) * xopt[j];
                    sum = sum + BMAT(k, j) * d[j];
                }
                w[k] = suma * (0.5 * suma + sumb);
                vlag[k] = sum;
                w[npt + k] = suma;
            });
            beta = 0.0;
            for (int jj = 0; jj < nptm; jj++) {
                double sum = 0.0;
                for (int k = 0; k < npt; k++) sum = sum + ZMAT(k, jj) * w[k];
                beta = beta - sum * sum;
                bq_par<WAVE>(npt, [&](int k) { vlag[k] = vlag[k] + sum * ZMAT(k, jj); });
            }
            dsq = 0.0;
            double bsum = 0.0, dx = 0.0;
            if constexpr (WAVE) {                // the column sums by lane j, then the three folds over j in order
                double *par = S.par;
                bq_par<true>(n, [&](int j) {
                    double sum = 0.0;
                    for (int k = 0; k < npt; k++) sum = sum + w[k] * BMAT(k, j);
                    par[j] = sum;
                    const int jp = npt + j;
                    for (int i = 0; i < n; i++) sum = sum + BMAT(jp, i) * d[i];
                    vlag[jp] = sum;
                });
                for (int j = 0; j < n; j++) {
                    dsq = dsq + d[j] * d[j];
                    bsum = bsum + par[j] * d[j];
                    bsum = bsum + vlag[npt + j] * d[j];
                    dx = dx + d[j] * xopt[j];
                }
            } else {
                for (int j = 0; j < n; j++) {
                    dsq = dsq + d[j] * d[j];
                    double sum = 0.0;
                    for (int k = 0; k < npt; k++) sum = sum + w[k] * BMAT(k, j);
                    bsum = bsum + sum * d[j];
                    const int jp = npt + j;
                    for (int i = 0; i < n; i++) sum = sum + BMAT(jp, i) * d[i];
                    vlag[jp] = sum;
                    bsum = bsum + sum * d[j];
                    dx = dx + d[j] * xopt[j];
                }
            }
            beta = dx * dx + dsq * (xoptsq + dx + dx + 0.5 * dsq) + beta - bsum;
            vlag[kopt] = vlag[kopt] + 1.0;
            bq_sync<WAVE>();
            if (ntrits == 0) {
                denom = vlag[knew] * vlag[knew] + alpha * beta;
                if (denom < cauchy && cauchy > 0.0) {
                    for (int i = 0; i < n; i++) {
                        xnew[i] = xalt[i];
                        d[i] = xnew[i] - xopt[i];
                    }
                    cauchy = 0.0;
                    state = 230;
                    break;
                }
                if (denom <= 0.5 * vlag[knew] * vlag[knew]) {
                    if (nf > nresc) { state = 190; break; }
                    state = 720;
                    break;
                }
            } else {
                const double delsq = delta * delta;
                double scaden = 0.0, biglsq = 0.0;
                // KNEW = 0 in Powell's 1-based code; a 0-based translation resets to index 0 (a NaN model never
                // replaces it, and the point index stays in range)
                knew = 0;
                if constexpr (WAVE) {            // every point's den and weight by lane k (the scan below reads them)
                    double *par = S.par;
                    const double bt = beta;
                    bq_par<true>(npt, [&](int k) {
                        double hdiag = 0.0;
                        for (int jj = 0; jj < nptm; jj++) hdiag = hdiag + ZMAT(k, jj) * ZMAT(k, jj);
                        par[k] = bt * hdiag + vlag[k] * vlag[k];
                        double ds2 = 0.0;
                        for (int j = 0; j < n; j++) ds2 = ds2 + (XPT(k, j) - xopt[j]) * (XPT(k, j) - xopt[j]);
                        par[BqState<NN>::NDIM + k] = bq_jmax(1.0, (ds2 / delsq) * (ds2 / delsq));
                    });
                }
                for (int k = 0; k < npt; k++) {
                    if (k == kopt) continue;
                    double den, temp;
                    if constexpr (WAVE) {
                        den = S.par[k];
                        temp = S.par[BqState<NN>::NDIM + k];
                    } else {
                        double hdiag = 0.0;
                        for (int jj = 0; jj < nptm; jj++) hdiag = hdiag + ZMAT(k, jj) * ZMAT(k, jj);
                        den = beta * hdiag + vlag[k] * vlag[k];
                        double ds2 = 0.0;
                        for (int j = 0; j < n; j++) ds2 = ds2 + (XPT(k, j) - xopt[j]) * (XPT(k, j) - xopt[j]);
                        temp = bq_jmax(1.0, (ds2 / delsq) * (ds2 / delsq));
                    }
                    if (temp * den > scaden) {
                        scaden = temp * den;
                        knew = k;
                        denom = den;
                    }
                    biglsq = bq_jmax(biglsq, temp * vlag[k] * vlag[k]);
                }
                if (scaden <= 0.5 * biglsq) {
                    if (nf > nresc) { state = 190; break; }
                    state = 720;
                    break;
                }
            }
            state = 360;
            break;
        }
        case 361:                                                  /* after the evaluation at label 360 */
            nf++;
            if (ntrits == -1) {
                fsave = f;
                state = 720;
                break;
            }
            fopt = fval[kopt];
            vquad = 0.0;
            {
                int ih = 0;
                for (int j = 0; j < n; j++) {
                    vquad = vquad + d[j] * gopt[j];
                    for (int i = 0; i <= j; i++) {
                        double temp = d[i] * d[j];
                        if (i == j) temp = 0.5 * temp;
                        vquad = vquad + hq[ih] * temp;
                        ih++;
                    }
                }
            }
            for (int k = 0; k < npt; k++) vquad = vquad + 0.5 * pq[k] * w[npt + k] * w[npt + k];
            diff = f - fopt - vquad;
            diffc = diffb;
            diffb = diffa;
            diffa = fabs(diff);
            if (dnorm > rho) nfsav = nf;
            if (ntrits > 0) {
                if (vquad >= 0.0) { state = 720; break; }
                ratio = (f - fopt) / vquad;
                if (ratio <= 0.1) delta = bq_jmin(0.5 * delta, dnorm);
                else if (ratio <= 0.7) delta = bq_jmax(0.5 * delta, dnorm);
                else delta = bq_jmax(0.5 * delta, dnorm + dnorm);
                if (delta <= 1.5 * rho) delta = rho;
                if (f < fopt) {
                    ksav = knew;
                    densav = denom;
                    const double delsq = delta * delta;
                    double scaden = 0.0, biglsq = 0.0;
                    knew = 0;
                    if constexpr (WAVE) {
                        double *par = S.par;
                        const double bt = beta;
                        bq_par<true>(npt, [&](int k) {
                            double hdiag = 0.0;
                            for (int jj = 0; jj < nptm; jj++) hdiag = hdiag + ZMAT(k, jj) * ZMAT(k, jj);
                            par[k] = bt * hdiag + vlag[k] * vlag[k];
                            double ds2 = 0.0;
                            for (int j = 0; j < n; j++) ds2 = ds2 + (XPT(k, j) - xnew[j]) * (XPT(k, j) - xnew[j]);
                            par[BqState<NN>::NDIM + k] = bq_jmax(1.0, (ds2 / delsq) * (ds2 / delsq));
                        });
                    }
                    for (int k = 0; k < npt; k++) {
                        double den, temp;
                        if constexpr (WAVE) {
                            den = S.par[k];
                            temp = S.par[BqState<NN>::NDIM + k];
                        } else {
                            double hdiag = 0.0;
                            for (int jj = 0; jj < nptm; jj++) hdiag = hdiag + ZMAT(k, jj) * ZMAT(k, jj);
                            den = beta * hdiag + vlag[k] * vlag[k];
                            double ds2 = 0.0;
                            for (int j = 0; j < n; j++) ds2 = ds2 + (XPT(k, j) - xnew[j]) * (XPT(k, j) - xnew[j]);
                            temp = bq_jmax(1.0, (ds2 / delsq) * (ds2 / delsq));
                        }
                        if (temp * den > scaden) {
                            scaden = temp * den;
                            knew = k;
                            denom = den;
                        }
                        biglsq = bq_jmax(biglsq, temp * vlag[k] * vlag[k]);
                    }
                    if (scaden <= 0.5 * biglsq) {
                        knew = ksav;
                        denom = densav;
                    }
                }
            }
            bq_update<NN, WAVE>(bmat, zmat, vlag, beta, denom, knew, w, S.par);
            {
                const double pqold = pq[knew];
                bq_sync<WAVE>();
                pq[knew] = 0.0;
                bq_sync<WAVE>();
                bq_par<WAVE>(nh, [&](int ih) {   // hq[ih], ih = i (i + 1) / 2 + j, j <= i
                    int i = 0;
                    while ((i + 1) * (i + 2) / 2 <= ih) i++;
                    const int j = ih - i * (i + 1) / 2;
                    const double temp = pqold * XPT(knew, i);
                    hq[ih] = hq[ih] + temp * XPT(knew, j);
                });
                bq_par<WAVE>(npt, [&](int k) {
                    double pk = pq[k];
                    for (int jj = 0; jj < nptm; jj++) {
                        const double temp = diff * ZMAT(knew, jj);
                        pk = pk + temp * ZMAT(k, jj);
                    }
                    pq[k] = pk;
                });
            }
            fval[knew] = f;
            for (int i = 0; i < n; i++) {
                const double xi = xnew[i], bi = BMAT(knew, i);
                bq_sync<WAVE>();
                XPT(knew, i) = xi;
                w[i] = bi;
            }
            bq_sync<WAVE>();
            if constexpr (WAVE) {                // per-point scalars by lane k, then w[i] folded over k by lane i
                double *par = S.par;
                bq_par<true>(npt, [&](int k) {
                    double suma = 0.0;
                    for (int jj = 0; jj < nptm; jj++) suma = suma + ZMAT(knew, jj) * ZMAT(k, jj);
                    double sumb = 0.0;
                    for (int j = 0; j < n; j++) sumb = sumb + XPT(k, j) * xopt[j];
                    par[k] = suma * sumb;
                });
                bq_par<true>(n, [&](int i) {
                    double wi = w[i];
                    for (int k = 0; k < npt; k++) wi = wi + par[k] * XPT(k, i);
                    w[i] = wi;
                });
            } else {
                for (int k = 0; k < npt; k++) {
                    double suma = 0.0;
                    for (int jj = 0; jj < nptm; jj++) suma = suma + ZMAT(knew, jj) * ZMAT(k, jj);
                    double sumb = 0.0;
                    for (int j = 0; j < n; j++) sumb = sumb + XPT(k, j) * xopt[j];
                    const double temp = suma * sumb;
                    for (int i = 0; i < n; i++) w[i] = w[i] + temp * XPT(k, i);
                }
            }
            for (int i = 0; i < n; i++) gopt[i] = gopt[i] + diff * w[i];
            if (f < fopt) {
                kopt = knew;
                xoptsq = 0.0;
                int ih = 0;
                for (int j = 0; j < n; j++) {
                    xopt[j] = xnew[j];
                    xoptsq = xoptsq + xopt[j] * xopt[j];
                    for (int i = 0; i <= j; i++) {
                        if (i < j) gopt[j] = gopt[j] + hq[ih] * d[i];
                        gopt[i] = gopt[i] + hq[ih] * d[j];
                        ih++;
                    }
                }
                bq_sync<WAVE>();
                if constexpr (WAVE) {
                    double *par = S.par;
                    bq_par<true>(npt, [&](int k) {
                        double temp = 0.0;
                        for (int j = 0; j < n; j++) temp = temp + XPT(k, j) * d[j];
                        par[k] = pq[k] * temp;
                    });
                    bq_par<true>(n, [&](int i) {
                        double g = gopt[i];
                        for (int k = 0; k < npt; k++) g = g + par[k] * XPT(k, i);
                        gopt[i] = g;
                    });
                } else {
                    for (int k = 0; k < npt; k++) {
                        double temp = 0.0;
                        for (int j = 0; j < n; j++) temp = temp + XPT(k, j) * d[j];
                        temp = pq[k] * temp;
                        for (int i = 0; i < n; i++) gopt[i] = gopt[i] + temp * XPT(k, i);
                    }
                }
            }
            if (ntrits > 0) {
                bq_sync<WAVE>();
                bq_par<WAVE>(npt, [&](int k) {
                    vlag[k] = fval[k] - fval[kopt];
                    w[k] = 0.0;
                });
                for (int j = 0; j < nptm; j++) {
                    double sum = 0.0;
                    for (int k = 0; k < npt; k++) sum = sum + ZMAT(k, j) * vlag[k];
                    bq_par<WAVE>(npt, [&](int k) { w[k] = w[k] + sum * ZMAT(k, j); });
                }
                bq_par<WAVE>(npt, [&](int k) {
                    double sum = 0.0;
                    for (int j = 0; j < n; j++) sum = sum + XPT(k, j) * xopt[j];
                    w[k + npt] = w[k];
                    w[k] = sum * w[k];
                });
                if constexpr (WAVE) {
                    double *par = S.par;
                    bq_par<true>(n, [&](int i) {
                        double sum = 0.0;
                        for (int k = 0; k < npt; k++) sum = sum + BMAT(k, i) * vlag[k] + XPT(k, i) * w[k];
                        par[i] = sum;
                    });
                }
                double gqsq = 0.0, gisq = 0.0;
                for (int i = 0; i < n; i++) {
                    double sum = 0.0;
                    if constexpr (WAVE) {
                        sum = S.par[i];
                    } else {
                        for (int k = 0; k < npt; k++) sum = sum + BMAT(k, i) * vlag[k] + XPT(k, i) * w[k];
                    }
                    if (xopt[i] == sl[i]) {
                        gqsq = gqsq + bq_jmin(0.0, gopt[i]) * bq_jmin(0.0, gopt[i]);
                        gisq = gisq + bq_jmin(0.0, sum) * bq_jmin(0.0, sum);
                    } else if (xopt[i] == su[i]) {
                        gqsq = gqsq + bq_jmax(0.0, gopt[i]) * bq_jmax(0.0, gopt[i]);
                        gisq = gisq + bq_jmax(0.0, sum) * bq_jmax(0.0, sum);
                    } else {
                        gqsq = gqsq + gopt[i] * gopt[i];
                        gisq = gisq + sum * sum;
                    }
                    vlag[npt + i] = sum;
                }
                itest++;
                if (gqsq < 10.0 * gisq) itest = 0;
                if (itest >= 3) {
                    const int mx = npt > nh ? npt : nh;
                    for (int i = 0; i < mx; i++) {
                        if (i < n) gopt[i] = vlag[npt + i];
                        if (i < npt) pq[i] = w[npt + i];
                        if (i < nh) hq[i] = 0.0;
                        itest = 0;
                    }
                }
            }
            if (ntrits == 0) { state = 60; break; }
            if (f <= fopt + 0.1 * vquad) { state = 60; break; }
            distsq = bq_jmax((2.0 * delta) * (2.0 * delta), (10.0 * rho) * (10.0 * rho));
            /* fallthrough */
        case 650: {
            knew = -1;
            for (int k = 0; k < npt; k++) {
                double sum = 0.0;
                for (int j = 0; j < n; j++) sum = sum + (XPT(k, j) - xopt[j]) * (XPT(k, j) - xopt[j]);
                if (sum > distsq) {
                    knew = k;
                    distsq = sum;
                }
            }
            if (knew >= 0) {
                const double dist = sqrt(distsq);
                if (ntrits == -1) {
                    delta = bq_jmin(0.1 * delta, 0.5 * dist);
                    if (delta <= 1.5 * rho) delta = rho;
                }
                ntrits = 0;
                adelt = bq_jmax(bq_jmin(0.1 * dist, delta), rho);
                dsq = adelt * adelt;
                state = 90;
                break;
            }
            if (ntrits == -1) { state = 680; break; }
            if (ratio > 0.0) { state = 60; break; }
            if (bq_jmax(delta, dnorm) > rho) { state = 60; break; }
        }
            /* fallthrough */
        case 680:
            if (rho > rhoend) {
                delta = 0.5 * rho;
                ratio = rho / rhoend;
                if (ratio <= 16.0) rho = rhoend;
                else if (ratio <= 250.0) rho = sqrt(ratio) * rhoend;
                else rho = 0.1 * rho;
                delta = bq_jmax(delta, rho);
                ntrits = 0;
                nfsav = nf;
                state = 60;
                break;
            }
            if (ntrits == -1) { state = 360; break; }
            /* fallthrough */
        case 720:
            if (fval[kopt] <= fsave) {
                for (int i = 0; i < n; i++) x[i] = xbase[i] + xopt[i];
                f = fval[kopt];
            }
            state = -2;
            break;
        default:
            break;
        }
      }
      if (state < 0) break;
      /* label 360 (or RESCUE's 290): the evaluation, the wave's lanes together */
      if (rk >= 0) {
          for (int i = 0; i < n; i++) x[i] = xbase[i] + XPT(rk, i);
      } else {
          for (int i = 0; i < n; i++) x[i] = xbase[i] + xnew[i];   /* min(max(XL, .), XU): unbounded */
      }
      if (!bq_eval<NN>(&ob, x, &f)) {
          status = ARIMA_ST_MAX_EVAL;
          state = -1;
          break;
      }
      state = rk >= 0 ? 194 : 361;
    }
    *n_eval_out = ob.n_eval > ob.max_eval ? ob.max_eval : ob.n_eval;
    if (state == -1) return status;
    for (int j = 0; j < n; j++) x_out[j] = x[j];
    return ARIMA_ST_OK;
}

// ARIMAModel.isStationary / isInvertible (ARIMA.scala:777-815) at runtime orders: model_flags' Schur-Cohn step-down
__device__ bool bq_roots_outside(const double *poly, int deg) {
    double a[6];
    for (int i = 0; i <= 5; ++i) a[i] = i <= deg ? poly[i] : 0.0;
    for (int i = 0; i <= deg; ++i)
        if (!finite(a[i])) return false;
    for (int mm = deg; mm >= 1; --mm) {
        const double kk = a[mm];
        if (!(fabs(kk) < 1.0)) return false;
        const double den = 1.0 - kk * kk;
        double b[6];
        for (int i = 0; i <= 5; ++i) b[i] = (i < mm) ? (a[i] - kk * a[mm - i]) / den : 0.0;
        for (int i = 0; i <= 5; ++i) a[i] = b[i];
    }
    return true;
}

__device__ uint8_t bq_model_flags(const double *c, int p, int q, int I) {
    if (p > 5 || q > 5) return gen_model_flags(c, p, q, I);      // the same step-down at any order
    double poly[6];
    bool st = true, inv = true;
    if (p > 0) {
        poly[0] = 1.0;
        for (int j = 0; j < p; ++j) poly[1 + j] = -1.0 * c[I + j];
        st = bq_roots_outside(poly, p);
    }
    if (q > 0) {
        poly[0] = 1.0;
        for (int j = 0; j < q; ++j) poly[1 + j] = c[I + p + j];
        inv = bq_roots_outside(poly, q);
    }
    return (uint8_t)((st ? ARIMA_FLAG_STATIONARY : 0) | (inv ? ARIMA_FLAG_INVERTIBLE : 0));
}

// fitModel's css-bobyqa branch after the initial parameters (ARIMA.scala:99-109): the Hannan-Rissanen init (or the
// user's) from init / init_status. refit_status (optional, ARIMA.autoFit's fitTryBothStrategies, :315-319): only the
// series whose css-cgd fit threw in the optimizer are refitted, in place.
// WAVE = false: a lane per series, the state in the lane's private memory. WAVE = true: a wave per series, the state
// in LDS; every lane runs the same (uniform) code on the same values, so the wave never diverges and every access
// to the interpolation matrices is an LDS broadcast instead of a scratch round trip; lane 0 writes the outputs.
// resident waves per SIMD the wave kernels are compiled for (a register cap): 1 (512 VGPRs) / 2 (256) / 4 (128, with
// spills): css-bobyqa fits of 65 536 C2 series 5.86 / 3.56 / 7.00 s, autoFit of 65 536 12.25 / 11.98 / 13.4 s
// (profiles/r05/q_wave, r_occ2, r_occ4)
constexpr int kBqWaveOcc = 2;

__device__ __forceinline__ bool bq_refit_wanted(int rs) {
    return rs == ARIMA_ST_MAX_EVAL || rs == ARIMA_ST_BRACKET_MAX_EVAL || rs == ARIMA_ST_MAX_ITER ||
           rs == ARIMA_ST_BAD_INTERVAL;
}

template <int NN, bool WAVE>
__global__ __launch_bounds__(64, WAVE ? kBqWaveOcc : 1) void k_bobyqa_fit(const double *__restrict__ y, int64_t ld, int n, int64_t N, int p,
                                                   int q, int I, const double *__restrict__ init,
                                                   const int32_t *__restrict__ init_status,
                                                   const int32_t *__restrict__ refit_status,
                                                   double *__restrict__ coef_out, double *__restrict__ ll_out,
                                                   int32_t *__restrict__ status_out, int32_t *__restrict__ n_eval_out,
                                                   int32_t *__restrict__ n_grad_out, uint8_t *__restrict__ flags_out) {
    const int64_t sid = WAVE ? (int64_t)blockIdx.x : (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sid >= N) return;
    if (refit_status && !bq_refit_wanted(refit_status[sid])) return;
    const int k = I + p + q;
    int st = init_status ? init_status[sid] : ARIMA_ST_OK;
    double x0[BQ_KMAX], x[BQ_KMAX];
    int nev = 0;
    for (int j = 0; j < BQ_KMAX; ++j) x0[j] = j < k ? init[sid * k + j] : 0.0;
    if constexpr (WAVE) {
        __shared__ BqState<NN> S;
        if (st == ARIMA_ST_OK) st = bq_fit<NN, true>(y + sid * ld, n, p, q, I, x0, x, &nev, S);
    } else {
        BqState<NN> S;
        if (st == ARIMA_ST_OK) st = bq_fit<NN>(y + sid * ld, n, p, q, I, x0, x, &nev, S);
    }
    const bool ok = st == ARIMA_ST_OK;
    const double ll = ok ? bq_css_ll(y + sid * ld, n, p, q, I, x) : __builtin_nan("");
    const uint8_t fl = ok ? bq_model_flags(x, p, q, I) : (uint8_t)0;
    if (WAVE && threadIdx.x != 0) return;
    for (int j = 0; j < k; ++j) coef_out[sid * k + j] = ok ? x[j] : __builtin_nan("");
    ll_out[sid] = ll;
    status_out[sid] = st;
    if (n_eval_out) n_eval_out[sid] = nev;
    if (n_grad_out) n_grad_out[sid] = 0;
    if (flags_out) flags_out[sid] = fl;
}

// ---- autoFit's css-bobyqa retries of one round of the stepwise walk, in one launch ------------------------------
// The round's candidate orders are fitted with css-cgd as separate batches (rows of order cb at [off[cb], off[cb+1])
// of the round's result arrays, coefficients and inits k-strided from off[cb] * 11). A per-order css-bobyqa launch
// would make each order wait for its slowest lane; instead the failing rows of every order are listed and refitted
// together. Per row the same computation as k_bobyqa_fit with refit_status.
__device__ __forceinline__ int af_row_combo(const int64_t *off, int ncombos, int64_t r) {   // the last order whose rows start <= r
    int cb = 0;
    for (int c = 1; c < ncombos; ++c)
        if (off[c] <= r) cb = c;
    return cb;
}

// One dimension's retries (the rows of bucket K of the round's retry list, k_af_refit_list): per row the computation of
// k_bobyqa_fit with refit_status. One kernel per dimension (arima_bobyqa_k<K>.hip) so the build parallelises; the
// runtime launches the dimensions present in a round on different streams, so they run together.
template <int K, bool WAVE>
__global__ __launch_bounds__(64, WAVE ? kBqWaveOcc : 1) void k_bobyqa_refit_k(const double *__restrict__ rows, int64_t ld,
                                                                             int n, const int32_t *__restrict__ lists,
                                                                             int64_t N, const int64_t *__restrict__ off,
                                                                             int ncombos, int kc,
                                                                             const int32_t *__restrict__ list,
                                                                             const unsigned *__restrict__ count,
                                                                             const double *__restrict__ init,
                                                                             const int32_t *__restrict__ init_status,
                                                                             double *__restrict__ coef,
                                                                             double *__restrict__ ll,
                                                                             int32_t *__restrict__ status,
                                                                             uint8_t *__restrict__ flags) {
    const int64_t cnt = (int64_t)count[K];
    const int64_t i0 = WAVE ? (int64_t)blockIdx.x : (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t istep = WAVE ? (int64_t)gridDim.x : (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = i0; i < cnt; i += istep) {
        const int64_t r = list[i];
        const int cb = af_row_combo(off, ncombos, r);
        const int p = (cb / 2) / 3, q = (cb / 2) % 3, I = cb % 2;
        const int64_t slot = r - off[cb];
        const double *y = rows + (int64_t)lists[(int64_t)cb * N + slot] * ld;
        const int64_t base = off[cb] * kc + slot * K;
        int st = init_status[r];
        double x0[BQ_KMAX], x[BQ_KMAX];
        int nev = 0;
        for (int j = 0; j < BQ_KMAX; ++j) x0[j] = j < K ? init[base + j] : 0.0;
        if (st == ARIMA_ST_OK) {
            if constexpr (WAVE) {
                __shared__ BqState<K> S;
                st = bq_fit<K, true>(y, n, p, q, I, x0, x, &nev, S);
            } else {
                BqState<K> S;
                st = bq_fit<K>(y, n, p, q, I, x0, x, &nev, S);
            }
        }
        const bool ok = st == ARIMA_ST_OK;
        const double llv = ok ? bq_css_ll(y, n, p, q, I, x) : __builtin_nan("");
        const uint8_t fl = ok ? bq_model_flags(x, p, q, I) : (uint8_t)0;
        if (!WAVE || threadIdx.x == 0) {
            for (int j = 0; j < K; ++j) coef[base + j] = ok ? x[j] : __builtin_nan("");
            ll[r] = llv;
            status[r] = st;
            flags[r] = fl;
        }
        if constexpr (WAVE) __syncthreads();       // the next row reuses the LDS state
    }
}

// ---- launchers of one dimension K (explicitly instantiated in arima_bobyqa_k<K>.hip) ----------------------------
template <int K>
int launch_bobyqa_fit_k(const double *y, int64_t ld, int n, int64_t N, int p, int q, int I, const double *init,
                        const int32_t *init_status, const int32_t *refit_status, double *coef_out, double *ll_out,
                        int32_t *status_out, int32_t *n_eval_out, int32_t *n_grad_out, uint8_t *flags_out, bool wave,
                        hipStream_t s) {
    if (wave)
        hipLaunchKernelGGL((k_bobyqa_fit<K, true>), dim3((unsigned)N), dim3(64), 0, s, y, ld, n, N, p, q, I, init,
                           init_status, refit_status, coef_out, ll_out, status_out, n_eval_out, n_grad_out, flags_out);
    else
        hipLaunchKernelGGL((k_bobyqa_fit<K, false>), dim3((unsigned)((N + 63) / 64)), dim3(64), 0, s, y, ld, n, N, p, q,
                           I, init, init_status, refit_status, coef_out, ll_out, status_out, n_eval_out, n_grad_out,
                           flags_out);
    return hipGetLastError() == hipSuccess ? ARIMA_OK : ARIMA_E_DEVICE;
}

// rows: bucket K's retry count, read back by the host (one workgroup per retry in the wave layout)
template <int K>
int launch_bobyqa_refit_k(const double *rows_, int64_t ld, int n, const int32_t *lists, int64_t N, const int64_t *off,
                          int ncombos, int kc, const int32_t *list, const unsigned *count, int64_t rows,
                          const double *init, const int32_t *init_status, double *coef, double *ll, int32_t *status,
                          uint8_t *flags, bool wave, hipStream_t s) {
    if (rows <= 0) return ARIMA_OK;
    if (wave)
        hipLaunchKernelGGL((k_bobyqa_refit_k<K, true>), dim3((unsigned)std::min<int64_t>(rows, 1 << 20)), dim3(64), 0,
                           s, rows_, ld, n, lists, N, off, ncombos, kc, list, count, init, init_status, coef, ll, status,
                           flags);
    else
        hipLaunchKernelGGL((k_bobyqa_refit_k<K, false>), dim3((unsigned)std::min<int64_t>((rows + 63) / 64, 1 << 16)),
                           dim3(64), 0, s, rows_, ld, n, lists, N, off, ncombos, kc, list, count, init, init_status,
                           coef, ll, status, flags);
    return hipGetLastError() == hipSuccess ? ARIMA_OK : ARIMA_E_DEVICE;
}

#define STS_BQ_DECLARE(KK, EXT)                                                                                        \
    EXT template int launch_bobyqa_fit_k<KK>(const double *, int64_t, int, int64_t, int, int, int, const double *,      \
                                             const int32_t *, const int32_t *, double *, double *, int32_t *,         \
                                             int32_t *, int32_t *, uint8_t *, bool, hipStream_t);                     \
    EXT template int launch_bobyqa_refit_k<KK>(const double *, int64_t, int, const int32_t *, int64_t, const int64_t *, \
                                               int, int, const int32_t *, const unsigned *, int64_t, const double *,  \
                                               const int32_t *, double *, double *, int32_t *, uint8_t *, bool,       \
                                               hipStream_t);

}  // namespace sts
