/*
 * oracle/bobyqa_oracle.c — CPU restatement of the css-bobyqa fit (ARIMA.fitWithCSSBOBYQA, ARIMA.scala:130-160).
 *
 * TEST INFRASTRUCTURE ONLY (see arima_oracle.c's header): the checker of the device css-bobyqa fit, never the product.
 *
 * The reference configures commons-math3 3.4.1's BOBYQAOptimizer (not vendored; pom.xml:466-470):
 *   npt = 2k + 1 interpolation points, rhobeg = min(0.96, 0.2 * max|init|), rhoend = 1e-6 * rhobeg,
 *   SimpleBounds.unbounded(k), GoalType.MAXIMIZE of logLikelihoodCSSARMA, MaxEval(10000), MaxIter(10000).
 * BOBYQAOptimizer is a Java translation of M.J.D. Powell's BOBYQA (bobyqa.f, 2009: BOBYQB, PRELIM, TRSBOX, ALTMOV,
 * UPDATE, RESCUE); this file restates that algorithm routine by routine in its published operation order, for the
 * configuration above: with infinite bounds every bound test of PRELIM / TRSBOX / ALTMOV is inactive, and npt = 2k+1
 * never reaches PRELIM's npt > 2n+1 branch. Commons-specific behaviour restated: the objective is negated for
 * MAXIMIZE (f = -LL), every objective evaluation counts toward MaxEval and the 10001st throws
 * TooManyEvaluationsException (commons drops Powell's NF >= MAXFUN return), and BOBYQAOptimizer.setup rejects
 * dimension < 2 (NumberIsTooSmallException).
 *
 * RESCUE (bobyqb label 190, reached when rounding has damaged an updating denominator) is restated too (bq_rescue);
 * its evaluations count toward MaxEval like every other (commons drops Powell's NF >= MAXFUN return there as well).
 *
 * Parity pinning: the algorithm is restated from Powell's published Fortran as recalled, not from commons' source
 * (absent here); the only reference pin is ARIMASuite.scala:58-74 (css-bobyqa within 0.1 of css-cgd on the
 * sampled ARIMA(2,1,2), tests/test_oracle_kats.py). Bit-level agreement with the JVM is unpinned.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/sparkts_arima.h"

#define BQ_KMAX 11
#define BQ_NPTMAX (2 * BQ_KMAX + 1)
#define BQ_NDIMMAX (BQ_NPTMAX + BQ_KMAX)

double orc_loglik_css_arma(const double *y, int n, int p, int q, int I, const double *coef);

typedef struct {
    const double *y;
    int n, p, q, I;
    int n_eval, max_eval;
    int failed;                        /* TooManyEvaluationsException thrown */
} bq_obj;

/* BaseOptimizer.computeObjectiveValue: counts, throws past MaxEval; f = -LL (GoalType.MAXIMIZE) */
static int bq_eval(bq_obj *o, const double *x, double *f) {
    if (++o->n_eval > o->max_eval) { o->failed = 1; return 0; }
    *f = -orc_loglik_css_arma(o->y, o->n, o->p, o->q, o->I, x);
    return 1;
}

#define XPT(k, j) xpt[(k) * BQ_KMAX + (j)]
#define BMAT(i, j) bmat[(i) * BQ_KMAX + (j)]
#define ZMAT(k, j) zmat[(k) * BQ_KMAX + (j)]

/* commons FastMath.max / min (NaN-propagating; max(-0, +0) = +0, min(+0, -0) = -0) */
static double jmax(double a, double b) {
    if (a > b) return a;
    if (a < b) return b;
    if (a != b) return NAN;
    uint64_t bits;
    memcpy(&bits, &a, 8);
    return bits == 0x8000000000000000ull ? b : a;
}
static double jmin(double a, double b) {
    if (a > b) return b;
    if (a < b) return a;
    if (a != b) return NAN;
    uint64_t bits;
    memcpy(&bits, &a, 8);
    return bits == 0x8000000000000000ull ? a : b;
}

/* ---- TRSBOX (trust-region step of the quadratic model, bound tests inactive) ---------------------------- */
static void bq_trsbox(int n, int npt, const double *xpt, const double *xopt, const double *gopt, const double *hq,
                      const double *pq, const double *sl, const double *su, double delta, double *xnew, double *d,
                      double *gnew, double *xbdi, double *s, double *hs, double *hred, double *dsq_out,
                      double *crvmin_out) {
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
            if (shs > 0.0) stplen = jmin(blen, gredsq / shs);
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
                    crvmin = jmin(crvmin, temp);
                    if (crvmin == -1.0) crvmin = temp;
                }
                ggsav = gredsq;
                gredsq = 0.0;
                for (int i = 0; i < n; i++) {
                    gnew[i] = gnew[i] + stplen * hs[i];
                    if (xbdi[i] == 0.0) gredsq = gredsq + gnew[i] * gnew[i];
                    d[i] = d[i] + stplen * s[i];
                }
                sdec = jmax(stplen * (ggsav - 0.5 * stplen * shs), 0.0);
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
                xnew[i] = jmax(jmin(xopt[i] + d[i], su[i]), sl[i]);
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
            for (int k = 0; k < npt; k++) {
                if (pq[k] != 0.0) {
                    temp = 0.0;
                    for (int j = 0; j < n; j++) temp = temp + XPT(k, j) * s[j];
                    temp = temp * pq[k];
                    for (int i = 0; i < n; i++) hs[i] = hs[i] + temp * XPT(k, i);
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
static void bq_altmov(int n, int npt, const double *xpt, const double *xopt, const double *bmat, const double *zmat,
                      const double *sl, const double *su, int kopt, int knew, double adelt, double *xnew,
                      double *xalt, double *alpha_out, double *cauchy_out, double *glag, double *hcol, double *w) {
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
        const double sumin = jmin(1.0, subd);
        for (int i = 0; i < n; i++) {
            temp = XPT(k, i) - xopt[i];
            if (temp > 0.0) {
                if (slbd * temp < sl[i] - xopt[i]) { slbd = (sl[i] - xopt[i]) / temp; ilbd = -(i + 1); }
                if (subd * temp > su[i] - xopt[i]) { subd = jmax(sumin, (su[i] - xopt[i]) / temp); iubd = i + 1; }
            } else if (temp < 0.0) {
                if (slbd * temp > su[i] - xopt[i]) { slbd = (su[i] - xopt[i]) / temp; ilbd = i + 1; }
                if (subd * temp < sl[i] - xopt[i]) { subd = jmax(sumin, (sl[i] - xopt[i]) / temp); iubd = -(i + 1); }
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
        xnew[i] = jmax(sl[i], jmin(su[i], temp));
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
            tempa = jmin(xopt[i] - sl[i], glag[i]);
            tempb = jmax(xopt[i] - su[i], glag[i]);
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
                xalt[i] = jmax(sl[i], jmin(su[i], xopt[i] + w[i]));
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
                xalt[i] = jmax(sl[i], jmin(su[i], temp));
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
static void bq_update(int n, int npt, double *bmat, double *zmat, double *vlag, double beta, double denom, int knew,
                      double *w) {
    const int nptm = npt - n - 1;
    double ztest = 0.0, temp, tempa, tempb, alpha, tau;
    for (int k = 0; k < npt; k++)
        for (int j = 0; j < nptm; j++) ztest = jmax(ztest, fabs(ZMAT(k, j)));
    ztest = 1.0e-20 * ztest;
    for (int j = 1; j < nptm; j++) {
        if (fabs(ZMAT(knew, j)) > ztest) {
            temp = sqrt(ZMAT(knew, 0) * ZMAT(knew, 0) + ZMAT(knew, j) * ZMAT(knew, j));
            tempa = ZMAT(knew, 0) / temp;
            tempb = ZMAT(knew, j) / temp;
            for (int i = 0; i < npt; i++) {
                temp = tempa * ZMAT(i, 0) + tempb * ZMAT(i, j);
                ZMAT(i, j) = tempa * ZMAT(i, j) - tempb * ZMAT(i, 0);
                ZMAT(i, 0) = temp;
            }
        }
        ZMAT(knew, j) = 0.0;
    }
    for (int i = 0; i < npt; i++) w[i] = ZMAT(knew, 0) * ZMAT(i, 0);
    alpha = w[knew];
    tau = vlag[knew];
    vlag[knew] = vlag[knew] - 1.0;
    temp = sqrt(denom);
    tempb = ZMAT(knew, 0) / temp;
    tempa = tau / temp;
    for (int i = 0; i < npt; i++) ZMAT(i, 0) = tempa * ZMAT(i, 0) - tempb * vlag[i];
    for (int j = 0; j < n; j++) {
        const int jp = npt + j;
        w[jp] = BMAT(knew, j);
        tempa = (alpha * vlag[jp] - tau * w[jp]) / denom;
        tempb = (-beta * w[jp] - tau * vlag[jp]) / denom;
        for (int i = 0; i <= jp; i++) {
            BMAT(i, j) = BMAT(i, j) + tempa * vlag[i] + tempb * w[i];
            if (i >= npt) BMAT(jp, i - npt) = BMAT(i, j);
        }
    }
}

/* ---- RESCUE (bobyqb label 190: rebuild BMAT / ZMAT when rounding has damaged an updating denominator) ------ *
 * Powell's RESCUE for npt = 2n + 1: XBASE moves to XBASE + XOPT, the interpolation set is replaced by provisional
 * points along the coordinate directions (PTSAUX, PTSID) whose BMAT / ZMAT are known in closed form, then as many of
 * the original points as keep the UPDATE denominators healthy are reinstated one by one (the 80-250 loop), and the
 * objective is evaluated at the provisional points that remain (260-340), each value updating GOPT / HQ / PQ.
 * PTSAUX(1..2, j) = ptsaux[2 j], ptsaux[2 j + 1]; PTSID holds Powell's encoded doubles (decoded with his truncating
 * conversions); W(NDIM + k) = w[ndim + k]. Every evaluation counts toward MaxEval like BOBYQB's (commons: the
 * 10001st throws, Powell's NF >= MAXFUN return is not restated). Returns 0 when an evaluation threw. */
static int bq_rescue(int n, int npt, bq_obj *ob, double *xbase, double *xpt, double *fval, double *xopt, double *gopt,
                     double *hq, double *pq, double *bmat, double *zmat, double *sl, double *su, int *nf_io,
                     double delta, int *kopt_io, double *vlag, double *ptsaux, double *ptsid, double *w) {
    const int np = n + 1, nptm = npt - np, ndim = npt + n;
    const double sfrac = 0.5 / (double)np;
    int kopt = *kopt_io, nf = *nf_io;
    const int kentry = kopt;
    (void)kentry;
    double sumpq = 0.0, winc = 0.0;
    for (int k = 0; k < npt; k++) {                            /* 10-20: XOPT to the origin, ZMAT = 0 */
        double distsq = 0.0;
        for (int j = 0; j < n; j++) {
            XPT(k, j) = XPT(k, j) - xopt[j];
            distsq = distsq + XPT(k, j) * XPT(k, j);
        }
        sumpq = sumpq + pq[k];
        w[ndim + k] = distsq;
        winc = jmax(winc, distsq);
        for (int j = 0; j < nptm; j++) ZMAT(k, j) = 0.0;
    }
    {                                                          /* 30-40: HQ for the shifted XBASE */
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
    for (int j = 0; j < n; j++) {                              /* 50: shift XBASE, SL, SU, XOPT; PTSAUX; BMAT = 0 */
        xbase[j] = xbase[j] + xopt[j];
        sl[j] = sl[j] - xopt[j];
        su[j] = su[j] - xopt[j];
        xopt[j] = 0.0;
        ptsaux[2 * j] = jmin(delta, su[j]);
        ptsaux[2 * j + 1] = jmax(-delta, sl[j]);
        if (ptsaux[2 * j] + ptsaux[2 * j + 1] < 0.0) {
            const double temp = ptsaux[2 * j];
            ptsaux[2 * j] = ptsaux[2 * j + 1];
            ptsaux[2 * j + 1] = temp;
        }
        if (fabs(ptsaux[2 * j + 1]) < 0.5 * fabs(ptsaux[2 * j])) ptsaux[2 * j + 1] = 0.5 * ptsaux[2 * j];
        for (int i = 0; i < ndim; i++) BMAT(i, j) = 0.0;
    }
    const double fbase = fval[kopt];
    ptsid[0] = sfrac;                                          /* 60: the provisional points along e_j */
    for (int j = 0; j < n; j++) {
        const int jp = j + 1, jpn = jp + n;                    /* 0-based rows of Powell's JP, JPN (jpn < npt) */
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
    /* 70: npt = 2n + 1 leaves no further identifiers (K = 2 NP .. NPT is empty) */
    int nrem = npt, kold = 0, knew = kopt;
    double beta = 0.0, denom = 0.0;
    for (;;) {
        /* 80-110: exchange PTSID(KOLD) with PTSID(KNEW); reinstate the original point KNEW */
        for (int j = 0; j < n; j++) {
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
            bq_update(n, npt, bmat, zmat, vlag, beta, denom, knew, w);
            if (nrem == 0) goto done;
            for (int k = 0; k < npt; k++) w[ndim + k] = fabs(w[ndim + k]);
        }
        for (;;) {
            /* 120-130: the nearest original point not yet tried (W(NDIM+K) > 0) */
            double dsqmin = 0.0;
            for (int k = 0; k < npt; k++) {
                if (w[ndim + k] > 0.0) {
                    if (dsqmin == 0.0 || w[ndim + k] < dsqmin) {
                        knew = k;
                        dsqmin = w[ndim + k];
                    }
                }
            }
            if (dsqmin == 0.0) goto evaluate;
            /* 140-160: its W-vector */
            for (int j = 0; j < n; j++) w[npt + j] = XPT(knew, j);
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
            /* 170-230: VLAG and BETA for reinstating XPT(KNEW, .) */
            for (int k = 0; k < npt; k++) {
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
            /* 240-250: KOLD, the provisional point whose deletion keeps the denominator largest */
            denom = 0.0;
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
                vlmxsq = jmax(vlmxsq, vlag[k] * vlag[k]);
            }
            if (denom <= 1.0e-2 * vlmxsq) {
                w[ndim + knew] = -w[ndim + knew] - winc;
                continue;
            }
            break;
        }
    }
evaluate:
    /* 260-340: the provisional points that remain, each evaluated and folded into the model */
    for (int kpt = 0; kpt < npt; kpt++) {
        if (ptsid[kpt] == 0.0) continue;
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
        double vquad = fbase;                                  /* the model at the new point */
        int ihp = 0;
        if (ip > 0) {
            ihp = (ip + ip * ip) / 2;                          /* Powell's 1-based packed index */
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
        double x[BQ_KMAX], f;                                  /* 290: XBASE + XPT(KPT, .), unbounded */
        for (int i = 0; i < n; i++) x[i] = xbase[i] + XPT(kpt, i);
        nf++;
        if (!bq_eval(ob, x, &f)) {
            *nf_io = nf;
            *kopt_io = kopt;
            return 0;
        }
        fval[kpt] = f;
        if (f < fval[kopt]) kopt = kpt;
        const double diff = f - vquad;
        for (int i = 0; i < n; i++) gopt[i] = gopt[i] + diff * BMAT(kpt, i);     /* 310-330: the model update */
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
done:
#ifdef BQ_RESCUE_CHECK_HOOK                                    /* debug builds: the rebuilt model's identities */
    BQ_RESCUE_CHECK_HOOK(n, npt, xpt, fval, gopt, hq, pq, bmat, zmat, kentry, fbase);
#endif
    *nf_io = nf;
    *kopt_io = kopt;
    return 1;
}

/* ---- BOBYQA driver + PRELIM + BOBYQB, unbounded, npt = 2n + 1 ------------------------------------------- *
 * Returns ARIMA_ST_*; x (in: the initial point, out: the optimum), n_eval_out = objective evaluations;
 * n_rescue (may be NULL) = how many times BOBYQB entered RESCUE. */
int orc_bobyqa_ex(const double *y, int len, int p, int q, int I, const double *x0, double *x_out, int *n_eval_out,
                  int *n_rescue);
static _Thread_local int bq_last_rescues;                      /* the calling thread's last fit (tests, tools) */
int orc_bobyqa_last_rescues(void) { return bq_last_rescues; }

int orc_bobyqa(const double *y, int len, int p, int q, int I, const double *x0, double *x_out, int *n_eval_out) {
    return orc_bobyqa_ex(y, len, p, q, I, x0, x_out, n_eval_out, &bq_last_rescues);
}

int orc_bobyqa_ex(const double *y, int len, int p, int q, int I, const double *x0, double *x_out, int *n_eval_out,
                  int *n_rescue) {
    if (n_rescue) *n_rescue = 0;
    const int n = I + p + q;
    *n_eval_out = 0;
    if (n < 2) return ARIMA_ST_TOO_FEW_PARAMS;                 /* BOBYQAOptimizer.setup: dimension >= 2 */
    const int npt = 2 * n + 1, np = n + 1, nptm = npt - np, nh = (n * np) / 2, ndim = npt + n;
    /* math.min(0.96, 0.2 * initParams.map(math.abs).max) (:147): Scala's max is reduceLeft((x, y) => if (x >= y) x
     * else y) with IEEE comparisons, Java's Math.min(a, b) is (a <= b ? a : b) for a = 0.96 -- NaN propagates as there */
    double amax = fabs(x0[0]);
    for (int j = 1; j < n; j++) amax = (amax >= fabs(x0[j])) ? amax : fabs(x0[j]);
    const double r02 = 0.2 * amax;
    const double rhobeg = (0.96 <= r02) ? 0.96 : r02;
    const double rhoend = rhobeg * 1e-6;                       /* :148 */
    bq_obj ob = {y, len, p, q, I, 0, 10000, 0};
    double xbase[BQ_KMAX], xpt[BQ_NPTMAX * BQ_KMAX], fval[BQ_NPTMAX], xopt[BQ_KMAX], gopt[BQ_KMAX],
        hq[BQ_KMAX * (BQ_KMAX + 1) / 2], pq[BQ_NPTMAX], bmat[BQ_NDIMMAX * BQ_KMAX], zmat[BQ_NPTMAX * BQ_KMAX],
        sl[BQ_KMAX], su[BQ_KMAX], xnew[BQ_KMAX], xalt[BQ_KMAX], d[BQ_KMAX], vlag[BQ_NDIMMAX],
        w[3 * BQ_NDIMMAX], x[BQ_KMAX], tw[5 * BQ_KMAX];
    memset(xpt, 0, sizeof xpt);
    memset(bmat, 0, sizeof bmat);
    memset(zmat, 0, sizeof zmat);
    for (int j = 0; j < n; j++) {                              /* BOBYQA: SL = XL - X, SU = XU - X (unbounded) */
        x[j] = x0[j];
        sl[j] = -INFINITY;
        su[j] = INFINITY;
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
            if (sl[nfx - 1] == 0.0) stepb = jmin(2.0 * rhobeg, su[nfx - 1]);
            if (su[nfx - 1] == 0.0) stepb = jmax(-2.0 * rhobeg, sl[nfx - 1]);
            XPT(nf - 1, nfx - 1) = stepb;
        }
        for (int j = 0; j < n; j++) x[j] = xbase[j] + XPT(nf - 1, j);   /* min(max(XL, .), XU): unbounded */
        if (!bq_eval(&ob, x, &f)) { *n_eval_out = ob.n_eval - 1; return ARIMA_ST_MAX_EVAL; }
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
    for (;;) {
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
            bq_trsbox(n, npt, xpt, xopt, gopt, hq, pq, sl, su, delta, xnew, d, tw, tw + n, tw + 2 * n, tw + 3 * n,
                      tw + 4 * n, &dsq, &crvmin);
            dnorm = jmin(delta, sqrt(dsq));
            if (dnorm < 0.5 * rho) {
                ntrits = -1;
                distsq = (10.0 * rho) * (10.0 * rho);
                if (nf <= nfsav + 2) { state = 650; break; }
                const double errbig = jmax(jmax(diffa, diffb), diffc);
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
        case 190: {
            nfsav = nf;
            kbase = kopt;
            double ptsid[BQ_NPTMAX];
            if (n_rescue) (*n_rescue)++;
            if (!bq_rescue(n, npt, &ob, xbase, xpt, fval, xopt, gopt, hq, pq, bmat, zmat, sl, su, &nf, delta, &kopt,
                           vlag, tw, ptsid, w)) {
                status = ARIMA_ST_MAX_EVAL;
                state = -1;
                break;
            }
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
        }
        case 210:
            bq_altmov(n, npt, xpt, xopt, bmat, zmat, sl, su, kopt, knew, adelt, xnew, xalt, &alpha, &cauchy, tw,
                      tw + n, w);
            for (int i = 0; i < n; i++) d[i] = xnew[i] - xopt[i];
            /* fallthrough */
        case 230: {
            for (int k = 0; k < npt; k++) {
                double suma = 0.0, sumb = 0.0, sum = 0.0;
                for (int j = 0; j < n; j++) {
                    suma = suma + XPT(k, j) * d[j];
                    sumb = sumb + XPT(k, j) * xopt[j];
                    sum = sum + BMAT(k, j) * d[j];
                }
                w[k] = suma * (0.5 * suma + sumb);
                vlag[k] = sum;
                w[npt + k] = suma;
            }
            beta = 0.0;
            for (int jj = 0; jj < nptm; jj++) {
                double sum = 0.0;
                for (int k = 0; k < npt; k++) sum = sum + ZMAT(k, jj) * w[k];
                beta = beta - sum * sum;
                for (int k = 0; k < npt; k++) vlag[k] = vlag[k] + sum * ZMAT(k, jj);
            }
            dsq = 0.0;
            double bsum = 0.0, dx = 0.0;
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
            beta = dx * dx + dsq * (xoptsq + dx + dx + 0.5 * dsq) + beta - bsum;
            vlag[kopt] = vlag[kopt] + 1.0;
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
                for (int k = 0; k < npt; k++) {
                    if (k == kopt) continue;
                    double hdiag = 0.0;
                    for (int jj = 0; jj < nptm; jj++) hdiag = hdiag + ZMAT(k, jj) * ZMAT(k, jj);
                    const double den = beta * hdiag + vlag[k] * vlag[k];
                    double ds2 = 0.0;
                    for (int j = 0; j < n; j++) ds2 = ds2 + (XPT(k, j) - xopt[j]) * (XPT(k, j) - xopt[j]);
                    const double temp = jmax(1.0, (ds2 / delsq) * (ds2 / delsq));
                    if (temp * den > scaden) {
                        scaden = temp * den;
                        knew = k;
                        denom = den;
                    }
                    biglsq = jmax(biglsq, temp * vlag[k] * vlag[k]);
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
        case 360:
            for (int i = 0; i < n; i++) x[i] = xbase[i] + xnew[i];     /* min(max(XL, .), XU): unbounded */
            if (!bq_eval(&ob, x, &f)) { status = ARIMA_ST_MAX_EVAL; state = -1; break; }
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
                if (ratio <= 0.1) delta = jmin(0.5 * delta, dnorm);
                else if (ratio <= 0.7) delta = jmax(0.5 * delta, dnorm);
                else delta = jmax(0.5 * delta, dnorm + dnorm);
                if (delta <= 1.5 * rho) delta = rho;
                if (f < fopt) {
                    ksav = knew;
                    densav = denom;
                    const double delsq = delta * delta;
                    double scaden = 0.0, biglsq = 0.0;
                    knew = 0;
                    for (int k = 0; k < npt; k++) {
                        double hdiag = 0.0;
                        for (int jj = 0; jj < nptm; jj++) hdiag = hdiag + ZMAT(k, jj) * ZMAT(k, jj);
                        const double den = beta * hdiag + vlag[k] * vlag[k];
                        double ds2 = 0.0;
                        for (int j = 0; j < n; j++) ds2 = ds2 + (XPT(k, j) - xnew[j]) * (XPT(k, j) - xnew[j]);
                        const double temp = jmax(1.0, (ds2 / delsq) * (ds2 / delsq));
                        if (temp * den > scaden) {
                            scaden = temp * den;
                            knew = k;
                            denom = den;
                        }
                        biglsq = jmax(biglsq, temp * vlag[k] * vlag[k]);
                    }
                    if (scaden <= 0.5 * biglsq) {
                        knew = ksav;
                        denom = densav;
                    }
                }
            }
            bq_update(n, npt, bmat, zmat, vlag, beta, denom, knew, w);
            {
                int ih = 0;
                const double pqold = pq[knew];
                pq[knew] = 0.0;
                for (int i = 0; i < n; i++) {
                    const double temp = pqold * XPT(knew, i);
                    for (int j = 0; j <= i; j++) {
                        hq[ih] = hq[ih] + temp * XPT(knew, j);
                        ih++;
                    }
                }
                for (int jj = 0; jj < nptm; jj++) {
                    const double temp = diff * ZMAT(knew, jj);
                    for (int k = 0; k < npt; k++) pq[k] = pq[k] + temp * ZMAT(k, jj);
                }
            }
            fval[knew] = f;
            for (int i = 0; i < n; i++) {
                XPT(knew, i) = xnew[i];
                w[i] = BMAT(knew, i);
            }
            for (int k = 0; k < npt; k++) {
                double suma = 0.0;
                for (int jj = 0; jj < nptm; jj++) suma = suma + ZMAT(knew, jj) * ZMAT(k, jj);
                double sumb = 0.0;
                for (int j = 0; j < n; j++) sumb = sumb + XPT(k, j) * xopt[j];
                const double temp = suma * sumb;
                for (int i = 0; i < n; i++) w[i] = w[i] + temp * XPT(k, i);
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
                for (int k = 0; k < npt; k++) {
                    double temp = 0.0;
                    for (int j = 0; j < n; j++) temp = temp + XPT(k, j) * d[j];
                    temp = pq[k] * temp;
                    for (int i = 0; i < n; i++) gopt[i] = gopt[i] + temp * XPT(k, i);
                }
            }
            if (ntrits > 0) {
                for (int k = 0; k < npt; k++) {
                    vlag[k] = fval[k] - fval[kopt];
                    w[k] = 0.0;
                }
                for (int j = 0; j < nptm; j++) {
                    double sum = 0.0;
                    for (int k = 0; k < npt; k++) sum = sum + ZMAT(k, j) * vlag[k];
                    for (int k = 0; k < npt; k++) w[k] = w[k] + sum * ZMAT(k, j);
                }
                for (int k = 0; k < npt; k++) {
                    double sum = 0.0;
                    for (int j = 0; j < n; j++) sum = sum + XPT(k, j) * xopt[j];
                    w[k + npt] = w[k];
                    w[k] = sum * w[k];
                }
                double gqsq = 0.0, gisq = 0.0;
                for (int i = 0; i < n; i++) {
                    double sum = 0.0;
                    for (int k = 0; k < npt; k++) sum = sum + BMAT(k, i) * vlag[k] + XPT(k, i) * w[k];
                    if (xopt[i] == sl[i]) {
                        gqsq = gqsq + jmin(0.0, gopt[i]) * jmin(0.0, gopt[i]);
                        gisq = gisq + jmin(0.0, sum) * jmin(0.0, sum);
                    } else if (xopt[i] == su[i]) {
                        gqsq = gqsq + jmax(0.0, gopt[i]) * jmax(0.0, gopt[i]);
                        gisq = gisq + jmax(0.0, sum) * jmax(0.0, sum);
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
            distsq = jmax((2.0 * delta) * (2.0 * delta), (10.0 * rho) * (10.0 * rho));
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
                    delta = jmin(0.1 * delta, 0.5 * dist);
                    if (delta <= 1.5 * rho) delta = rho;
                }
                ntrits = 0;
                adelt = jmax(jmin(0.1 * dist, delta), rho);
                dsq = adelt * adelt;
                state = 90;
                break;
            }
            if (ntrits == -1) { state = 680; break; }
            if (ratio > 0.0) { state = 60; break; }
            if (jmax(delta, dnorm) > rho) { state = 60; break; }
        }
            /* fallthrough */
        case 680:
            if (rho > rhoend) {
                delta = 0.5 * rho;
                ratio = rho / rhoend;
                if (ratio <= 16.0) rho = rhoend;
                else if (ratio <= 250.0) rho = sqrt(ratio) * rhoend;
                else rho = 0.1 * rho;
                delta = jmax(delta, rho);
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
        if (state < 0) break;
    }
    *n_eval_out = ob.n_eval > ob.max_eval ? ob.max_eval : ob.n_eval;
    if (state == -1) return status;
    for (int j = 0; j < n; j++) x_out[j] = x[j];
    return ARIMA_ST_OK;
}
