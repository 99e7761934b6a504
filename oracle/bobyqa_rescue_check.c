/*
 * oracle/bobyqa_rescue_check.c — TEST INFRASTRUCTURE ONLY: the oracle's css-bobyqa fit built with a check of every
 * RESCUE it runs (tests/test_oracle_rescue.py). Powell's RESCUE (bobyqa_oracle.c bq_rescue) rebuilds the inverse KKT
 * matrix H (BMAT, ZMAT) and the quadratic model for a new interpolation set; the rebuild is right when
 *   - every Lagrange function interpolates: L_j(x_i) = delta_ij with L_j(x) = [j == kbase] + BMAT(j, .) x
 *     + 1/2 sum_k (Z Z^T)_jk (x_k . x)^2 (x_kbase = 0, XBASE moved there), and
 *   - the model reproduces the value at every point RESCUE evaluated: Q(x) = F(kbase) + GOPT x + 1/2 x^T HESS x,
 *     HESS = HQ + sum_k PQ_k x_k x_k^T (points RESCUE reinstated keep the pre-RESCUE model's rounding, so the test
 *     reads the worst error over the evaluated points only when the set is well scaled).
 * Both are measured against the spread of the set, kappa = (r_max / r_min)^4 over the points' distances from x_kbase
 * (the KKT matrix holds (x_i . x_j)^2 / 2 terms, so its conditioning grows with kappa: a set stretched along a ridge
 * with provisional points at +-DELTA loses that many digits in any H). The worst error / max(1, kappa) over all
 * RESCUE calls of the calling thread is read back with orc_rescue_check_*.
 */
#include <math.h>
static void rescue_check(int n, int npt, const double *xpt, const double *fval, const double *gopt, const double *hq,
                         const double *pq, const double *bmat, const double *zmat, int kbase, double fbase);
#define BQ_RESCUE_CHECK_HOOK(...) rescue_check(__VA_ARGS__)
#include "bobyqa_oracle.c"

static _Thread_local double rc_model, rc_lag;
static _Thread_local int rc_calls;

void orc_rescue_check_reset(void) { rc_model = rc_lag = 0.0; rc_calls = 0; }
int orc_rescue_check_calls(void) { return rc_calls; }
double orc_rescue_check_lagrange(void) { return rc_lag; }
double orc_rescue_check_model(void) { return rc_model; }

static void rescue_check(int n, int npt, const double *xpt, const double *fval, const double *gopt, const double *hq,
                         const double *pq, const double *bmat, const double *zmat, int kbase, double fbase) {
    const int nptm = npt - n - 1;
    double fscale = 0.0, rmax = 0.0, rmin = INFINITY;
    for (int i = 0; i < npt; i++) fscale = fabs(fval[i]) > fscale ? fabs(fval[i]) : fscale;
    for (int i = 0; i < npt; i++) {
        double r = 0.0;
        for (int a = 0; a < n; a++) r += XPT(i, a) * XPT(i, a);
        r = sqrt(r);
        if (r > rmax) rmax = r;
        if (r > 0.0 && r < rmin) rmin = r;
    }
    const double kr = rmax / rmin, kappa = kr * kr * kr * kr > 1.0 ? kr * kr * kr * kr : 1.0;
    rc_calls++;
    for (int i = 0; i < npt; i++) {
        const double *x = &XPT(i, 0);
        double qv = fbase;
        for (int a = 0; a < n; a++) qv += gopt[a] * x[a];
        int ih = 0;
        for (int j = 0; j < n; j++)
            for (int a = 0; a <= j; a++) {
                const double t = hq[ih++] * x[a] * x[j];
                qv += (a == j) ? 0.5 * t : t;
            }
        for (int k = 0; k < npt; k++) {
            double s = 0.0;
            for (int a = 0; a < n; a++) s += XPT(k, a) * x[a];
            qv += 0.5 * pq[k] * s * s;
        }
        const double em = fabs(qv - fval[i]) / fscale / kappa;
        if (em > rc_model) rc_model = em;
        for (int j = 0; j < npt; j++) {
            double l = (j == kbase) ? 1.0 : 0.0;
            for (int a = 0; a < n; a++) l += BMAT(j, a) * x[a];
            for (int k = 0; k < npt; k++) {
                double om = 0.0, s = 0.0;
                for (int c = 0; c < nptm; c++) om += ZMAT(j, c) * ZMAT(k, c);
                for (int a = 0; a < n; a++) s += XPT(k, a) * x[a];
                l += 0.5 * om * s * s;
            }
            const double el = fabs(l - (i == j ? 1.0 : 0.0)) / kappa;
            if (el > rc_lag) rc_lag = el;
        }
    }
}
