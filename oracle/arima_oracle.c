/*
 * oracle/arima_oracle.c — CPU restatement of the spark-ts ARIMA CSS-CGD fit path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / the timed CPU baseline — never as the product path.
 *
 * What it restates (every function cites the reference file:line it follows; paths relative to the
 * reference root):
 *   - UnivariateTimeSeries.differencesOfOrderD / inverseDifferencesOfOrderD     (.scala:384-495)
 *   - Lag.lagMatTrimBoth (index arithmetic)                                    (Lag.scala:33-99)
 *   - Autoregression.fitModel                                                   (Autoregression.scala:38-53)
 *   - ARIMA.hannanRissanenInit                                                  (ARIMA.scala:216-242)
 *   - ARIMAModel.logLikelihoodCSSARMA / iterateARMA / updateMAErrors            (ARIMA.scala:430-618)
 *   - ARIMAModel.gradientlogLikelihoodCSSARMA                                   (ARIMA.scala:465-534)
 *   - ARIMA.fitWithCSSCGD + ARIMA.fitModel dispatch                             (ARIMA.scala:79-116,174-200)
 *   - ARIMAModel.forecast / addTimeDependentEffects / removeTimeDependentEffects (ARIMA.scala:629-764)
 *   - TimeSeriesStatisticalTests.kpsstest + neweyWestVarianceEstimator (stats/TimeSeriesStatisticalTests.scala:369-431),
 *     the differencing-order test of ARIMA.autoFit (the stepwise walk itself is restated in oracle.py: autofit)
 *   - third-party algorithms the path calls, which are NOT vendored in the reference:
 *       commons-math3 3.4.1 (pom.xml:466-470): NonLinearConjugateGradientOptimizer (FLETCHER_REEVES),
 *       LineSearch, BracketFinder, BrentOptimizer, SimpleValueChecker, SimpleUnivariateValueChecker,
 *       Precision.equals, OLSMultipleLinearRegression + QRDecomposition (Householder, threshold 0);
 *       Breeze 0.12 (pom.xml:58): the overlapping row-slice copy at ARIMA.scala:526 (see `smear` below);
 *       fdlibm __ieee754_log (java.lang.StrictMath.log) for `math.log` at ARIMA.scala:444.
 *     They are restated from their published algorithms.
 *
 * Parity pinning: the reference (Scala/JVM) cannot be built or run in this container (no JDK, no jars; see
 * SURVEY.md 8(c)). This restatement is pinned by the reference's own known-answer tests and data files
 * (tests/test_oracle_kats.py): ARIMASuite.scala:27-156, UnivariateTimeSeriesSuite.scala:31-158,
 * AutoregressionSuite.scala:26-44, python/sparkts/models/test/test_ARIMA.py:20-64, including the
 * path-dependent user-init test (test_ARIMA.py:27-32). Those tests pin results to tolerances (0.01-0.1), not
 * bit patterns, so bit-level agreement with the JVM is unpinned; the two known ambiguities are
 *   (1) Breeze's overlapping `dEdTheta(1 to -1, ::) := dEdTheta(0 to -2, ::)` (shift vs smear, q >= 2;
 *       decided for smear from Breeze 0.12's slice and OpSet implementation; shift kept),
 *   (2) HotSpot's Math.log intrinsic vs fdlibm (<= 1 ulp on rare inputs).
 *
 * Numerics: compile with -ffp-contract=off and no -ffast-math (Java never contracts a*b+c into an FMA).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/sparkts_arima.h"

#define ORC_MAX_EVAL 10000     /* new MaxEval(10000)   ARIMA.scala:196 */
#define ORC_MAX_ITER 10000     /* new MaxIter(10000)   ARIMA.scala:195 */
#define ORC_BRACKET_MAX 500    /* BracketFinder() = BracketFinder(100, 500) */
#define ORC_KMAX 64

int orc_bobyqa(const double *y, int len, int p, int q, int I, const double *x0, double *x_out, int *n_eval_out);

/* ===================================================================================================== */
/* fdlibm __ieee754_log (e_log.c), the algorithm behind java.lang.StrictMath.log                           */
/* ===================================================================================================== */
static const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                    two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
                    Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                    Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
                    Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;

static inline int32_t hi_word(double x) { uint64_t u; memcpy(&u, &x, 8); return (int32_t)(u >> 32); }
static inline uint32_t lo_word(double x) { uint64_t u; memcpy(&u, &x, 8); return (uint32_t)u; }
static inline double with_hi(double x, int32_t hi) {
    uint64_t u; memcpy(&u, &x, 8);
    u = ((uint64_t)(uint32_t)hi << 32) | (u & 0xffffffffull);
    memcpy(&x, &u, 8); return x;
}

double orc_log(double x) {
    double hfsq, f, s, z, R, w, t1, t2, dk;
    int32_t k, hx, i, j;
    uint32_t lx;
    hx = hi_word(x);
    lx = lo_word(x);
    k = 0;
    if (hx < 0x00100000) {                       /* x < 2**-1022  */
        if (((hx & 0x7fffffff) | lx) == 0) return -two54 / 0.0;   /* log(+-0) = -inf */
        if (hx < 0) return (x - x) / 0.0;                           /* log(-#) = NaN   */
        k -= 54; x *= two54;                                         /* subnormal: scale up */
        hx = hi_word(x);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    i = (hx + 0x95f64) & 0x100000;
    x = with_hi(x, hx | (i ^ 0x3ff00000));       /* normalize x or x/2 */
    k += (i >> 20);
    f = x - 1.0;
    if ((0x000fffff & (2 + hx)) < 3) {           /* |f| < 2**-20 */
        if (f == 0.0) {
            if (k == 0) return 0.0;
            dk = (double)k; return dk * ln2_hi + dk * ln2_lo;
        }
        R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        dk = (double)k; return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    s = f / (2.0 + f);
    dk = (double)k;
    z = s * s;
    i = hx - 0x6147a;
    w = z * z;
    j = 0x6b851 - hx;
    t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    R = t2 + t1;
    if (i > 0) {
        hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

/* ===================================================================================================== */
/* Differencing — UnivariateTimeSeries.scala                                                             */
/* ===================================================================================================== */

/* differencesAtLag(ts, dest, lag, startIndex)  UnivariateTimeSeries.scala:384-405 */
static void differences_at_lag(const double *ts, double *dest, int n, int lag, int start) {
    if (lag == 0) { memcpy(dest, ts, sizeof(double) * (size_t)n); return; }
    for (int i = 0; i < n; i++) dest[i] = (i < start) ? ts[i] : ts[i] - ts[i - lag];
}

/* differencesOfOrderD  UnivariateTimeSeries.scala:468-480 (ping-pong copies, size preserving) */
void orc_differences_of_order_d(const double *ts, int T, int d, double *out) {
    double *diffed = (double *)malloc(sizeof(double) * (size_t)(T > 0 ? T : 1));
    double *orig = (double *)malloc(sizeof(double) * (size_t)(T > 0 ? T : 1));
    if (T > 0) {                                  /* (an empty series may come with a null pointer) */
        memcpy(diffed, ts, sizeof(double) * (size_t)T);
        memcpy(orig, ts, sizeof(double) * (size_t)T);
    }
    for (int i = 1; i <= d; i++) {
        double *swap = orig; orig = diffed; diffed = swap;
        differences_at_lag(orig, diffed, T, 1, i);
    }
    if (T > 0) memcpy(out, diffed, sizeof(double) * (size_t)T);
    free(diffed); free(orig);
}

/* inverseDifferencesOfOrderD  UnivariateTimeSeries.scala:489-495 (+ inverseDifferencesAtLag :426-447, in place) */
void orc_inverse_differences_of_order_d(const double *in, int L, int d, double *out) {
    if (L > 0) memcpy(out, in, sizeof(double) * (size_t)L);
    for (int i = d; i >= 1; i--)
        for (int j = 0; j < L; j++) out[j] = (j < i) ? out[j] : out[j] + out[j - 1];
}

/* ===================================================================================================== */
/* CSS log-likelihood and gradient — ARIMA.scala:430-554                                                  */
/* ===================================================================================================== */

/* updateMAErrors  ARIMA.scala:544-554.  NOTE: the loop runs i = 0 .. n-2 ascending with errs(i+1) = errs(i),
 * so for q >= 3 positions 1..q-1 all end up holding the previous errs(0) (a smear, not a shift). Restated
 * exactly as written. */
static void update_ma_errors(double *errs, int n, double new_error) {
    for (int i = 0; i < n - 1; i++) errs[i + 1] = errs[i];
    if (n > 0) errs[0] = new_error;
}

/* logLikelihoodCSSARMA  ARIMA.scala:430-445 (+ iterateARMA :581-618 with op = +, goldStandard = y) */
double orc_loglik_css_arma(const double *y, int n, int p, int q, int I, const double *coef) {
    int M = p > q ? p : q;
    double ma[ORC_KMAX];
    for (int j = 0; j < q; j++) ma[j] = 0.0;
    double css = 0.0;
    for (int i = M; i < n; i++) {
        double dest = 0.0;                               /* yHat = Array.fill(n)(0.0)              */
        dest = dest + (double)I * coef[0];               /* :600 op(dest(i), intercept * coef(0))  */
        for (int j = 0; j < p && i - j - 1 >= 0; j++)   /* :602-605                               */
            dest = dest + y[i - j - 1] * coef[I + j];
        for (int j = 0; j < q; j++)                      /* :608-611                               */
            dest = dest + ma[j] * coef[I + p + j];
        double err = y[i] - dest;                        /* :613                                    */
        update_ma_errors(ma, q, err);
        double r = y[i] - dest;                          /* :440-442 pow(obs - pred, 2), folded left */
        css = css + r * r;
    }
    double sigma2 = css / (double)n;                     /* :443 */
    return (double)(-n / 2) * orc_log(2.0 * 3.141592653589793 * sigma2) - css / (2.0 * sigma2); /* :444 */
}

/* gradientlogLikelihoodCSSARMA  ARIMA.scala:465-534.
 * `dEdTheta(1 to -1, ::) := dEdTheta(0 to -2, ::)` (:526) under Breeze 0.12: both slices are
 * strided views of the same (q+1) x k column-major array (canSliceRows: offset = first row, majorStride =
 * q + 1); the DenseMatrix OpSet walks columns outer, rows inner ascending, with no overlap check, so row r+1
 * receives the already overwritten row r:
 * smear == 1 (default): element-wise ascending copy (every lag row becomes row 0);
 * smear == 0: memmove-like row shift (what a copy-on-overlap implementation would give). */
void orc_gradient_css_arma(const double *y, int n, int p, int q, int I, const double *coef, int smear,
                           double *grad) {
    int k = I + p + q;
    int M = p > q ? p : q;
    double dE[ORC_KMAX * ORC_KMAX];                /* (q+1) x k, row-major dE[r*k + j] */
    double ma[ORC_KMAX];
    for (int j = 0; j < (q + 1) * k; j++) dE[j] = 0.0;
    for (int j = 0; j < q; j++) ma[j] = 0.0;
    for (int j = 0; j < k; j++) grad[j] = 0.0;
    double sigma2 = 0.0;
    for (int i = M; i < n; i++) {
        for (int j = 0; j < k; j++)                                     /* :492-499 */
            for (int kk = 0; kk < q; kk++)
                dE[j] = dE[j] - coef[I + p + kk] * dE[(kk + 1) * k + j];
        double yh = 0.0;
        yh = yh + (double)I * coef[0];                                   /* :502 */
        dE[0] = dE[0] - (double)I;                                       /* :503 */
        for (int j = 0; j < p && i - j - 1 >= 0; j++) {                  /* :506-510 */
            yh = yh + y[i - j - 1] * coef[I + j];
            dE[I + j] = dE[I + j] - y[i - j - 1];
        }
        for (int j = 0; j < q; j++) {                                    /* :514-518 */
            yh = yh + ma[j] * coef[I + p + j];
            dE[I + p + j] = dE[I + p + j] - ma[j];
        }
        double err = y[i] - yh;                                          /* :520 */
        sigma2 = sigma2 + (err * err) / (double)n;                       /* :521 */
        update_ma_errors(ma, q, err);                                    /* :522 */
        for (int j = 0; j < k; j++) grad[j] = grad[j] + dE[j] * err;    /* :524 */
        if (smear) {                                                     /* :526 */
            for (int r = 1; r <= q; r++)
                for (int j = 0; j < k; j++) dE[r * k + j] = dE[(r - 1) * k + j];
        } else {
            for (int r = q; r >= 1; r--)
                for (int j = 0; j < k; j++) dE[r * k + j] = dE[(r - 1) * k + j];
        }
        for (int j = 0; j < k; j++) dE[j] = 0.0;                         /* :528 */
    }
    for (int j = 0; j < k; j++) grad[j] = grad[j] / -sigma2;             /* :532 */
}

/* ===================================================================================================== */
/* OLS — commons-math3 3.4.1 OLSMultipleLinearRegression + QRDecomposition(threshold = 0)                 */
/* ===================================================================================================== */

/* Y: rows; X: rows x ncx row-major predictors (no intercept column). beta: ncx + intercept entries,
 * ordered [intercept?, columns...]. Returns ARIMA_ST_*. */
int orc_ols(const double *Y, const double *X, int rows, int ncx, int intercept, double *beta) {
    /* AbstractMultipleLinearRegression.validateSampleData */
    if (rows <= 0) return ARIMA_ST_NO_DATA;
    if (ncx + 1 > rows) return ARIMA_ST_NOT_ENOUGH_DATA;
    /* newXSampleData: Array2DRowRealMatrix(x) rejects zero columns */
    if (!intercept && ncx == 0) return ARIMA_ST_NO_DATA;
    int cols = ncx + (intercept ? 1 : 0);
    double *qrt = (double *)malloc(sizeof(double) * (size_t)cols * (size_t)rows);  /* qrt[c*rows + r] = X^T */
    for (int r = 0; r < rows; r++) {
        int c0 = 0;
        if (intercept) { qrt[0 * rows + r] = 1.0; c0 = 1; }
        for (int c = 0; c < ncx; c++) qrt[(size_t)(c + c0) * rows + r] = X[(size_t)r * ncx + c];
    }
    int nd = cols < rows ? cols : rows;
    double rdiag[ORC_KMAX];
    /* QRDecomposition.decompose -> performHouseholderReflection(minor, qrt) */
    for (int minor = 0; minor < nd; minor++) {
        double *qm = qrt + (size_t)minor * rows;
        double xNormSqr = 0.0;
        for (int row = minor; row < rows; row++) { double c = qm[row]; xNormSqr = xNormSqr + c * c; }
        double a = (qm[minor] > 0) ? -sqrt(xNormSqr) : sqrt(xNormSqr);
        rdiag[minor] = a;
        if (a != 0.0) {
            qm[minor] = qm[minor] - a;
            for (int col = minor + 1; col < cols; col++) {
                double *qc = qrt + (size_t)col * rows;
                double alpha = 0.0;
                for (int row = minor; row < rows; row++) alpha = alpha - qc[row] * qm[row];
                alpha = alpha / (a * qm[minor]);
                for (int row = minor; row < rows; row++) qc[row] = qc[row] - alpha * qm[row];
            }
        }
    }
    /* Solver.solve: isNonSingular (|rDiag| <= threshold == 0 -> singular) */
    for (int i = 0; i < nd; i++)
        if (fabs(rdiag[i]) <= 0.0) { free(qrt); return ARIMA_ST_SINGULAR; }
    double *yv = (double *)malloc(sizeof(double) * (size_t)rows);
    memcpy(yv, Y, sizeof(double) * (size_t)rows);
    for (int minor = 0; minor < nd; minor++) {
        const double *qm = qrt + (size_t)minor * rows;
        double dot = 0.0;
        for (int row = minor; row < rows; row++) dot = dot + yv[row] * qm[row];
        dot = dot / (rdiag[minor] * qm[minor]);
        for (int row = minor; row < rows; row++) yv[row] = yv[row] + dot * qm[row];
    }
    for (int row = nd - 1; row >= 0; --row) {
        yv[row] = yv[row] / rdiag[row];
        double yRow = yv[row];
        const double *qr = qrt + (size_t)row * rows;
        beta[row] = yRow;
        for (int i = 0; i < row; i++) yv[i] = yv[i] - yRow * qr[i];
    }
    free(yv); free(qrt);
    return ARIMA_ST_OK;
}

/* Lag.lagMatTrimBoth(x, maxLag, includeOriginal)  Lag.scala:33-49 (Array[Array[Double]] form, row-major out:
 * rows n - maxLag, cols maxLag (+1); lagMat(r)(c - initialLag) = x(r + maxLag - c) for c = initialLag..maxLag) */
static void lag_mat_trim_both(const double *x, int n, int maxLag, int includeOriginal, double *out) {
    const int rows = n - maxLag, cols = maxLag + (includeOriginal ? 1 : 0), initialLag = includeOriginal ? 0 : 1;
    for (int r = 0; r < rows; r++)
        for (int c = initialLag; c <= maxLag; c++) out[(size_t)r * cols + (c - initialLag)] = x[r + maxLag - c];
}

/* UnivariateTimeSeries.lag(ts, maxLag, includeOriginal) = Lag.lagMatTrimBoth(Vector, ...)  Lag.scala:62-99:
 * the same matrix as a column-major DenseMatrix (numTruncatedRows = x.size - numRows = maxLag). Returns rows. */
int orc_lag_matrix(const double *x, int n, int maxLag, int includeOriginal, double *out_colmajor) {
    const int rows = n - maxLag, cols = maxLag + (includeOriginal ? 1 : 0);
    if (rows < 0) return -1;
    double *rm = (double *)malloc(sizeof(double) * (size_t)(rows > 0 ? rows : 1) * (size_t)(cols > 0 ? cols : 1));
    lag_mat_trim_both(x, n, maxLag, includeOriginal, rm);
    for (int r = 0; r < rows; r++)
        for (int c = 0; c < cols; c++) out_colmajor[(size_t)c * rows + r] = rm[(size_t)r * cols + c];
    free(rm);
    return rows;
}

/* Autoregression.fitModel(ts, maxLag, noIntercept)  Autoregression.scala:38-53
 * (Y = ts(maxLag until n); X = Lag.lagMatTrimBoth(ts, maxLag), Lag.scala:33-49: X(r)(l-1) = ts(r+maxLag-l)) */
int orc_ar_fit(const double *ts, int n, int maxLag, int noIntercept, double *c_out, double *coef_out) {
    int rows = n - maxLag;
    if (rows < 0) return ARIMA_ST_SERIES_TOO_SHORT;
    double *X = (double *)malloc(sizeof(double) * (size_t)(rows > 0 ? rows : 1) * (size_t)(maxLag > 0 ? maxLag : 1));
    lag_mat_trim_both(ts, n, maxLag, 0, X);
    double beta[ORC_KMAX];
    int st = orc_ols(ts + maxLag, X, rows, maxLag, !noIntercept, beta);
    free(X);
    if (st != ARIMA_ST_OK) return st;
    if (noIntercept) { *c_out = 0.0; for (int j = 0; j < maxLag; j++) coef_out[j] = beta[j]; }
    else { *c_out = beta[0]; for (int j = 0; j < maxLag; j++) coef_out[j] = beta[1 + j]; }
    return ARIMA_ST_OK;
}

/* ARIMA.hannanRissanenInit  ARIMA.scala:216-242 */
int orc_hannan_rissanen(const double *y, int n, int p, int q, int I, double *params) {
    int M = p > q ? p : q;
    int m = M + 1;                                             /* :223 */
    double car, a[ORC_KMAX];
    int st = orc_ar_fit(y, n, m, 0, &car, a);                  /* :225 AR(m) always WITH intercept */
    if (st != ARIMA_ST_OK) return st;
    int nt = n - m;                                            /* yTrunc = y.drop(m), :227 */
    const double *yTrunc = y + m;
    double *errors = (double *)malloc(sizeof(double) * (size_t)(nt > 0 ? nt : 1));
    for (int r = 0; r < nt; r++) {                             /* :228-232 */
        double s = 0.0;
        for (int j = 0; j < m; j++) s = s + y[r + m - 1 - j] * a[j];   /* Lag.lagMatTrimBoth(y, m, false) */
        double est = s + car;
        errors[r] = yTrunc[r] - est;
    }
    /* :234-236 lag matrices; negative sizes throw in Array.ofDim */
    if (nt - p < 0 || nt - q < 0) { free(errors); return ARIMA_ST_SERIES_TOO_SHORT; }
    int rows = nt - M;                                         /* rows after drop(max(q-p,0)) / drop(max(p-q,0)) */
    if (rows < 0) rows = 0;
    int ncx = p + q;
    double *X = (double *)malloc(sizeof(double) * (size_t)(rows > 0 ? rows : 1) * (size_t)(ncx > 0 ? ncx : 1));
    for (int r = 0; r < rows; r++) {
        for (int c = 1; c <= p; c++) X[(size_t)r * ncx + (c - 1)] = yTrunc[r + M - c];
        for (int c = 1; c <= q; c++) X[(size_t)r * ncx + p + (c - 1)] = errors[r + M - c];
    }
    st = orc_ols(yTrunc + M, X, rows, ncx, I, params);        /* :237-240, noIntercept = !includeIntercept */
    free(X); free(errors);
    return st;
}

/* ===================================================================================================== */
/* TimeSeriesStatisticalTests.kpsstest  stats/TimeSeriesStatisticalTests.scala:369-431 (used by ARIMA.autoFit)   */
/* ===================================================================================================== */

/* method 0 = "c" (regressors: a column of ones), 1 = "ct" (ones and the time trend 1..n), both fitted by
 * OLSMultipleLinearRegression with setNoIntercept(true) (:375-385). Writes the statistic; returns ARIMA_ST_*
 * (the OLS shape checks throw for n <= number of regressors). */
int orc_kpss(const double *ts, int n, int method, double *stat_out) {
    const int ncx = method == 1 ? 2 : 1;
    double *X = (double *)calloc((size_t)(n > 0 ? n : 1) * 2, sizeof(double));
    for (int r = 0; r < n; r++) {
        X[(size_t)r * ncx] = 1.0;                                   /* Array.fill(n)(1.0)                  :374 */
        if (ncx == 2) X[(size_t)r * ncx + 1] = 1.0 + (double)r;     /* Array.tabulate(n)(x => 1.0 + x)     :379 */
    }
    double beta[2];
    int st = orc_ols(ts, X, n, ncx, 0, beta);
    if (st != ARIMA_ST_OK) { free(X); return st; }
    /* estimateResiduals: y - X.operate(b) (Array2DRowRealMatrix.operate: sum = 0; sum += x_rj * b_j)      :384 */
    double *e = (double *)malloc(sizeof(double) * (size_t)n);
    for (int r = 0; r < n; r++) {
        double sum = 0.0;
        for (int j = 0; j < ncx; j++) sum = sum + X[(size_t)r * ncx + j] * beta[j];
        e[r] = ts[r] - sum;
    }
    free(X);
    /* s2 = residuals.scanLeft(0.0)(_ + _).tail.map(math.pow(_, 2)).sum (left folds; pow(x, 2) = x * x)   :386 */
    double cum = 0.0, s2 = 0.0;
    for (int r = 0; r < n; r++) { cum = cum + e[r]; s2 = s2 + cum * cum; }
    /* lag = (3 * math.sqrt(n) / 13).toInt                                                                 :390 */
    const int lag = (int)(3.0 * sqrt((double)n) / 13.0);
    /* neweyWestVarianceEstimator(residuals, lag)                                                        :405-431 */
    double sumOfTerms = 0.0;
    for (int i = 1; i <= lag; i++) {
        double cell = 0.0;
        for (int j = i; j < n; j++) cell = cell + e[j] * e[j - i];
        sumOfTerms = sumOfTerms + cell * (1.0 - ((double)i / (double)(lag + 1)));
    }
    const double partial = (sumOfTerms * 2.0) / (double)n;
    double sq = 0.0;
    for (int r = 0; r < n; r++) sq = sq + e[r] * e[r];
    const double lrv = partial + sq / (double)n;
    free(e);
    /* (s2 / longRunVariance) / (n * n): n * n is an Int product (32-bit)                                   :392 */
    const int32_t nn = (int32_t)((uint32_t)n * (uint32_t)n);
    *stat_out = (s2 / lrv) / (double)nn;
    return ARIMA_ST_OK;
}

/* ===================================================================================================== */
/* commons-math3 3.4.1 NonLinearConjugateGradientOptimizer(FLETCHER_REEVES, SimpleValueChecker(1e-7,1e-7))  */
/* ===================================================================================================== */

typedef struct {
    const double *y;
    int n, p, q, I, k, smear;
    int n_eval, n_grad, n_iter;
    /* optional evaluation trace (analysis only): phase (0 top, 1 bracket, 2 brent, 3 gradient), alpha */
    int *tr_phase;
    double *tr_alpha;
    int tr_len, tr_cap, tr_cur_phase;
    double tr_cur_alpha;
    /* optional per-iteration state trace (analysis only, tools/maxeval_study.py): at the top of every CG iteration
     * [point (k), searchDirection (k), delta, previous objective, n_eval] */
    double *st_buf;
    int st_cap, st_len;
} orc_ctx;

static void trace(orc_ctx *c, int phase, double alpha) {
    if (c->tr_phase && c->tr_len < c->tr_cap) {
        c->tr_phase[c->tr_len] = phase;
        c->tr_alpha[c->tr_len] = alpha;
        c->tr_len++;
    }
}

/* BaseOptimizer.computeObjectiveValue: evaluations.incrementCount() (throws past MaxEval) then f */
static int cg_obj(orc_ctx *c, const double *x, double *f) {
    if (c->n_eval + 1 > ORC_MAX_EVAL) return ARIMA_ST_MAX_EVAL;
    c->n_eval++;
    *f = orc_loglik_css_arma(c->y, c->n, c->p, c->q, c->I, x);
    return ARIMA_ST_OK;
}

/* LineSearch.search's univariate function: x[i] = startPoint[i] + alpha * direction[i] */
static int ls_f(orc_ctx *c, const double *start, const double *dir, double alpha, double *f) {
    double x[ORC_KMAX];
    trace(c, c->tr_cur_phase, alpha);
    for (int i = 0; i < c->k; i++) x[i] = start[i] + alpha * dir[i];
    return cg_obj(c, x, f);
}

/* BracketFinder.eval: own Incrementor(500) first, then the function */
static int br_eval(orc_ctx *c, int *bcount, const double *start, const double *dir, double alpha, double *f) {
    if (*bcount + 1 > ORC_BRACKET_MAX) return ARIMA_ST_BRACKET_MAX_EVAL;
    (*bcount)++;
    c->tr_cur_phase = 1;
    int st = ls_f(c, start, dir, alpha, f);
    c->tr_cur_phase = 2;
    return st;
}

/* Precision.equals(x, y) with maxUlps = 1 */
static int prec_equals(double x, double y) {
    int64_t xi, yi;
    memcpy(&xi, &x, 8); memcpy(&yi, &y, 8);
    int eq;
    if (((xi ^ yi) & (int64_t)0x8000000000000000ull) == 0) {
        int64_t dd = xi - yi;
        eq = (dd < 0 ? -dd : dd) <= 1;
    } else {
        int64_t dplus, dminus;
        const int64_t NEG0 = (int64_t)0x8000000000000000ull;
        if (xi < yi) { dplus = yi; dminus = xi - NEG0; }
        else { dplus = xi; dminus = yi - NEG0; }
        eq = (dplus > 1) ? 0 : (dminus <= (1 - dplus));
    }
    return eq && !isnan(x) && !isnan(y);
}

/* FastMath.max semantics: NaN if either is NaN */
static double jmax(double a, double b) {
    if (a > b) return a;
    if (a < b) return b;
    if (a != b) return NAN;
    return a;   /* equal (sign of zero irrelevant for the <= tests below) */
}

/* SimpleValueChecker / SimpleUnivariateValueChecker .converged (value part; no iteration cap) */
static int value_converged(double p, double c, double rel, double abs_) {
    double difference = fabs(p - c);
    double size = jmax(fabs(p), fabs(c));
    return (difference <= size * rel) || (difference <= abs_);
}

/* LineSearch.search(startPoint, direction): BracketFinder.search(f, MAXIMIZE, 0, 1e-8) then
 * BrentOptimizer(1e-15, Double.MIN_VALUE, SimpleUnivariateValueChecker(1e-8, 1e-8)) on SearchInterval. */
static int line_search(orc_ctx *c, const double *start, const double *dir, double *step_out) {
    const double GOLD = 1.618034, EPS_MIN = 1e-21, growLimit = 100.0;
    int bcount = 0, st;
    double xA = 0.0, xB = 1e-8, fA, fB, fC, fW, tmp;
    /* BracketFinder.search, isMinim = false */
    if ((st = br_eval(c, &bcount, start, dir, xA, &fA))) return st;
    if ((st = br_eval(c, &bcount, start, dir, xB, &fB))) return st;
    if (fA > fB) { tmp = xA; xA = xB; xB = tmp; tmp = fA; fA = fB; fB = tmp; }
    double xC = xB + GOLD * (xB - xA);
    if ((st = br_eval(c, &bcount, start, dir, xC, &fC))) return st;
    while (fC > fB) {
        double tmp1 = (xB - xA) * (fB - fC);
        double tmp2 = (xB - xC) * (fB - fA);
        double val = tmp2 - tmp1;
        double denom = fabs(val) < EPS_MIN ? 2 * EPS_MIN : val;
        double w = xB - ((xB - xC) * tmp2 - (xB - xA) * tmp1) / (2 * denom);
        double wLim = xB + growLimit * (xC - xB);
        if ((w - xC) * (xB - w) > 0) {
            if ((st = br_eval(c, &bcount, start, dir, w, &fW))) return st;
            if (fW > fC) { xA = xB; xB = w; fA = fB; fB = fW; break; }
            else if (fW < fB) { xC = w; fC = fW; break; }
            w = xC + GOLD * (xC - xB);
            if ((st = br_eval(c, &bcount, start, dir, w, &fW))) return st;
        } else if ((w - wLim) * (wLim - xC) >= 0) {
            w = wLim;
            if ((st = br_eval(c, &bcount, start, dir, w, &fW))) return st;
        } else if ((w - wLim) * (xC - w) > 0) {
            if ((st = br_eval(c, &bcount, start, dir, w, &fW))) return st;
            if (fW > fC) {
                xB = xC; xC = w; w = xC + GOLD * (xC - xB); fB = fC; fC = fW;
                if ((st = br_eval(c, &bcount, start, dir, w, &fW))) return st;
            }
        } else {
            w = xC + GOLD * (xC - xB);
            if ((st = br_eval(c, &bcount, start, dir, w, &fW))) return st;
        }
        xA = xB; fA = fB; xB = xC; fB = fC; xC = w; fC = fW;
    }
    double lo = xA, mid = xB, hi = xC;
    if (lo > hi) { tmp = lo; lo = hi; hi = tmp; }
    /* SearchInterval(lo, hi, mid) */
    if (lo >= hi) return ARIMA_ST_BAD_INTERVAL;
    if (mid < lo || mid > hi) return ARIMA_ST_BAD_INTERVAL;

    /* BrentOptimizer.doOptimize, GoalType.MAXIMIZE */
    const double GS = 0.5 * (3 - sqrt(5.0));
    const double relT = 1e-15, absT = 4.9e-324;   /* 2*ulp(1) <= 1e-15; Double.MIN_VALUE */
    double a, b;
    if (lo < hi) { a = lo; b = hi; } else { a = hi; b = lo; }
    double x = mid, v = x, w = x, d = 0, e = 0;
    double fx;
    if ((st = ls_f(c, start, dir, x, &fx))) return st;
    fx = -fx;
    double fv = fx, fw = fx;
    int have_prev = 0;
    double prev_x = 0, prev_f = 0, cur_x = x, cur_f = -fx, best_x = x, best_f = -fx;
    int iter = 0;
    (void)iter;
    for (;;) {
        double m = 0.5 * (a + b);
        double tol1 = relT * fabs(x) + absT;
        double tol2 = 2 * tol1;
        int stop = fabs(x - m) <= tol2 - 0.5 * (b - a);
        if (!stop) {
            double p = 0, q = 0, r = 0, u = 0;
            if (fabs(e) > tol1) {
                r = (x - w) * (fx - fv);
                q = (x - v) * (fx - fw);
                p = (x - v) * q - (x - w) * r;
                q = 2 * (q - r);
                if (q > 0) p = -p; else q = -q;
                r = e;
                e = d;
                if (p > q * (a - x) && p < q * (b - x) && fabs(p) < fabs(0.5 * q * r)) {
                    d = p / q;
                    u = x + d;
                    if (u - a < tol2 || b - u < tol2) d = (x <= m) ? tol1 : -tol1;
                } else {
                    e = (x < m) ? b - x : a - x;
                    d = GS * e;
                }
            } else {
                e = (x < m) ? b - x : a - x;
                d = GS * e;
            }
            if (fabs(d) < tol1) u = (d >= 0) ? x + tol1 : x - tol1;
            else u = x + d;
            double fu;
            if ((st = ls_f(c, start, dir, u, &fu))) return st;
            fu = -fu;
            /* previous = current; current = (u, f(u)); best = best(best, best(previous, current)) */
            prev_x = cur_x; prev_f = cur_f; have_prev = 1;
            cur_x = u; cur_f = -fu;
            {
                double bx2, bf2;
                if (prev_f >= cur_f) { bx2 = prev_x; bf2 = prev_f; } else { bx2 = cur_x; bf2 = cur_f; }
                if (!(best_f >= bf2)) { best_x = bx2; best_f = bf2; }
            }
            if (value_converged(prev_f, cur_f, 1e-8, 1e-8)) { *step_out = best_x; return ARIMA_ST_OK; }
            if (fu <= fx) {
                if (u < x) b = x; else a = x;
                v = w; fv = fw; w = x; fw = fx; x = u; fx = fu;
            } else {
                if (u < x) a = u; else b = u;
                if (fu <= fw || prec_equals(w, x)) { v = w; fv = fw; w = u; fw = fu; }
                else if (fu <= fv || prec_equals(v, x) || prec_equals(v, w)) { v = u; fv = fu; }
            }
        } else {
            if (have_prev) {
                double bx2, bf2;
                if (prev_f >= cur_f) { bx2 = prev_x; bf2 = prev_f; } else { bx2 = cur_x; bf2 = cur_f; }
                if (!(best_f >= bf2)) { best_x = bx2; best_f = bf2; }
            } else {
                if (!(best_f >= cur_f)) { best_x = cur_x; best_f = cur_f; }
            }
            *step_out = best_x;
            return ARIMA_ST_OK;
        }
        ++iter;
    }
}

/* gradient function call (not counted as an evaluation) */
static void cg_grad(orc_ctx *c, const double *x, double *g) {
    c->n_grad++;
    trace(c, 3, 0.0);
    orc_gradient_css_arma(c->y, c->n, c->p, c->q, c->I, x, c->smear, g);
}

/* NonLinearConjugateGradientOptimizer.doOptimize (FLETCHER_REEVES, identity preconditioner, MAXIMIZE) */
static int cg_optimize(orc_ctx *c, const double *init, double *point_out, double *obj_out) {
    int k = c->k;
    double point[ORC_KMAX], r[ORC_KMAX], steepest[ORC_KMAX], dir[ORC_KMAX];
    memcpy(point, init, sizeof(double) * (size_t)k);
    cg_grad(c, point, r);
    for (int i = 0; i < k; i++) { steepest[i] = r[i]; dir[i] = steepest[i]; }
    double delta = 0;
    for (int i = 0; i < k; ++i) delta = delta + r[i] * dir[i];
    int have_cur = 0;
    double cur_obj = 0;
    int st;
    for (;;) {
        if (c->n_iter + 1 > ORC_MAX_ITER) return ARIMA_ST_MAX_ITER;
        c->n_iter++;
        if (c->st_buf && c->st_len < c->st_cap) {
            double *o = c->st_buf + (size_t)c->st_len * (size_t)(2 * k + 3);
            for (int i = 0; i < k; i++) { o[i] = point[i]; o[k + i] = dir[i]; }
            o[2 * k] = delta;
            o[2 * k + 1] = have_cur ? cur_obj : NAN;
            o[2 * k + 2] = (double)c->n_eval;
            c->st_len++;
        }
        double objective;
        trace(c, 0, 0.0);
        if ((st = cg_obj(c, point, &objective))) return st;
        int converged = have_cur && value_converged(cur_obj, objective, 1e-7, 1e-7);
        cur_obj = objective; have_cur = 1;
        if (converged) {
            memcpy(point_out, point, sizeof(double) * (size_t)k);
            *obj_out = objective;
            return ARIMA_ST_OK;
        }
        double step;
        if ((st = line_search(c, point, dir, &step))) return st;
        for (int i = 0; i < k; ++i) point[i] = point[i] + step * dir[i];
        cg_grad(c, point, r);
        double deltaOld = delta;
        delta = 0;
        for (int i = 0; i < k; ++i) delta = delta + r[i] * r[i];
        double beta = delta / deltaOld;
        for (int i = 0; i < k; i++) steepest[i] = r[i];
        if (c->n_iter % k == 0 || beta < 0) {
            for (int i = 0; i < k; i++) dir[i] = steepest[i];
        } else {
            for (int i = 0; i < k; ++i) dir[i] = steepest[i] + beta * dir[i];
        }
    }
}

/* ===================================================================================================== */
/* ARIMA.fitModel  ARIMA.scala:79-116 (method "css-cgd"); one series                                       */
/* ===================================================================================================== */
/* Returns ARIMA_ST_*. coef_out has k entries (NaN on failure); ll_out = logLikelihoodCSS at coef_out.
 * counters: [n_eval, n_grad, n_iter]. */
int orc_fit(const double *ts, int T, int p, int d, int q, int I, int method, const double *user_init,
            int smear, double *coef_out, double *ll_out, int *counters) {
    int k = I + p + q;
    for (int j = 0; j < k; j++) coef_out[j] = NAN;
    *ll_out = NAN;
    counters[0] = counters[1] = counters[2] = 0;
    double *tmp = (double *)malloc(sizeof(double) * (size_t)(T > 0 ? T : 1));
    orc_differences_of_order_d(ts, T, d, tmp);                    /* :88 */
    int n = T - d; if (n < 0) n = 0;
    const double *y = tmp + (T - n);                              /* .drop(d) */
    int st;
    if (p > 0 && q == 0) {                                        /* :90-96 AR shortcut (method not checked) */
        double c, a[ORC_KMAX];
        st = orc_ar_fit(y, n, p, !I, &c, a);
        if (st == ARIMA_ST_OK) {
            int o = 0;
            if (I) coef_out[o++] = c;
            for (int j = 0; j < p; j++) coef_out[o++] = a[j];
            *ll_out = orc_loglik_css_arma(y, n, p, q, I, coef_out);
        }
        free(tmp);
        return st;
    }
    double init[ORC_KMAX];
    if (user_init == NULL) {                                      /* :99-103 */
        st = orc_hannan_rissanen(y, n, p, q, I, init);
        if (st != ARIMA_ST_OK) { free(tmp); return st; }
    } else {
        memcpy(init, user_init, sizeof(double) * (size_t)k);
    }
    if (method == ARIMA_METHOD_CSS_BOBYQA) {                      /* :106 fitWithCSSBOBYQA, :130-160 */
        double pt[ORC_KMAX];
        st = orc_bobyqa(y, n, p, q, I, init, pt, &counters[0]);
        if (st == ARIMA_ST_OK) {
            memcpy(coef_out, pt, sizeof(double) * (size_t)k);
            *ll_out = orc_loglik_css_arma(y, n, p, q, I, coef_out);
        }
        free(tmp);
        return st;
    }
    if (method != ARIMA_METHOD_CSS_CGD) { free(tmp); return ARIMA_ST_UNSUPPORTED_METHOD; }  /* :105-109 */
    if (k == 0) { free(tmp); return ARIMA_ST_ZERO_PARAMS; }
    orc_ctx c = {y, n, p, q, I, k, smear, 0, 0, 0, NULL, NULL, 0, 0, 2, 0.0, NULL, 0, 0};
    double pt[ORC_KMAX], obj;
    st = cg_optimize(&c, init, pt, &obj);                         /* :174-200 */
    counters[0] = c.n_eval; counters[1] = c.n_grad; counters[2] = c.n_iter;
    if (st == ARIMA_ST_OK) {
        memcpy(coef_out, pt, sizeof(double) * (size_t)k);
        *ll_out = obj;
    }
    free(tmp);
    return st;
}

/* Same as orc_fit (CG path only, user_init or HR init) with an evaluation trace (analysis tool). */
int orc_fit_trace(const double *ts, int T, int p, int d, int q, int I, int smear, int *tr_phase,
                  double *tr_alpha, int tr_cap, int *tr_len) {
    int k = I + p + q;
    double *tmp = (double *)malloc(sizeof(double) * (size_t)(T > 0 ? T : 1));
    orc_differences_of_order_d(ts, T, d, tmp);
    int n = T - d;
    const double *y = tmp + d;
    double init[ORC_KMAX];
    int st = orc_hannan_rissanen(y, n, p, q, I, init);
    if (st) { free(tmp); *tr_len = 0; return st; }
    orc_ctx c = {y, n, p, q, I, k, smear, 0, 0, 0, tr_phase, tr_alpha, 0, tr_cap, 2, 0.0, NULL, 0, 0};
    double pt[ORC_KMAX], obj;
    st = cg_optimize(&c, init, pt, &obj);
    *tr_len = c.tr_len;
    free(tmp);
    return st;
}

/* Same CG fit (HR init) recording the optimizer's state at the top of every iteration into st_buf (2k + 3 doubles per
 * iteration, at most st_cap iterations): the MaxEval periodicity study (tools/maxeval_study.py). counters: n_eval,
 * n_grad, n_iter. */
int orc_fit_state_trace(const double *ts, int T, int p, int d, int q, int I, int smear, double *st_buf, int st_cap,
                        int *st_len, int *counters) {
    int k = I + p + q;
    double *tmp = (double *)malloc(sizeof(double) * (size_t)(T > 0 ? T : 1));
    orc_differences_of_order_d(ts, T, d, tmp);
    int n = T - d;
    const double *y = tmp + d;
    double init[ORC_KMAX];
    int st = orc_hannan_rissanen(y, n, p, q, I, init);
    *st_len = 0;
    counters[0] = counters[1] = counters[2] = 0;
    if (st) { free(tmp); return st; }
    orc_ctx c = {y, n, p, q, I, k, smear, 0, 0, 0, NULL, NULL, 0, 0, 2, 0.0, st_buf, st_cap, 0};
    double pt[ORC_KMAX], obj;
    st = cg_optimize(&c, init, pt, &obj);
    *st_len = c.st_len;
    counters[0] = c.n_eval; counters[1] = c.n_grad; counters[2] = c.n_iter;
    free(tmp);
    return st;
}

/* Thread count of the batch wrapper (bench.py's CPU baseline times it on the lease's share and on one core). */
#ifdef _OPENMP
#include <omp.h>
#endif
void orc_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* Batch wrapper (OpenMP over series when compiled with -fopenmp): the CPU baseline leg of bench.py. */
int orc_fit_batch(const double *series, long long n_series, int T, int p, int d, int q, int I, int method,
                  const double *user_init, int smear, double *coef_out, double *ll_out, int *status_out,
                  int *counters_out) {
    int k = I + p + q;
#pragma omp parallel for schedule(dynamic, 4)
    for (long long i = 0; i < n_series; i++) {
        status_out[i] = orc_fit(series + (size_t)i * T, T, p, d, q, I, method,
                                user_init ? user_init + (size_t)i * k : NULL, smear,
                                coef_out + (size_t)i * k, ll_out + i, counters_out + 3 * (size_t)i);
    }
    return 0;
}

/* ===================================================================================================== */
/* ARIMAModel: forecast / add & removeTimeDependentEffects  ARIMA.scala:581-764                           */
/* ===================================================================================================== */

/* iterateARMA  ARIMA.scala:581-618. op: +1 for _ + _, -1 for _ - _. gold or errors (one non-NULL). */
static void iterate_arma(const double *ts, double *dest, int n, int op, const double *gold,
                         const double *errors, double *init_ma, int p, int q, int I, const double *coef) {
    double ma[ORC_KMAX];
    if (init_ma) memcpy(ma, init_ma, sizeof(double) * (size_t)q); else for (int j = 0; j < q; j++) ma[j] = 0.0;
    int M = p > q ? p : q;
    for (int i = M; i < n; i++) {
        double t = (double)I * coef[0];
        dest[i] = op > 0 ? dest[i] + t : dest[i] - t;
        for (int j = 0; j < p && i - j - 1 >= 0; j++) {
            t = ts[i - j - 1] * coef[I + j];
            dest[i] = op > 0 ? dest[i] + t : dest[i] - t;
        }
        for (int j = 0; j < q; j++) {
            t = ma[j] * coef[I + p + j];
            dest[i] = op > 0 ? dest[i] + t : dest[i] - t;
        }
        double err = gold == NULL ? errors[i] : gold[i] - dest[i];
        update_ma_errors(ma, q, err);
    }
}

/* ARIMAModel.forecast(ts, nFuture)  ARIMA.scala:696-764; out has T + nFuture entries */
void orc_forecast(const double *ts, int T, int p, int d, int q, int I, const double *coef, int nFuture,
                  double *out) {
    int M = p > q ? p : q;
    double *dts = (double *)malloc(sizeof(double) * (size_t)(T + 1));
    orc_differences_of_order_d(ts, T, d, dts);
    int n = T - d;
    double intercept_amt = I ? coef[0] : 0.0;
    int histLen = M + n;
    double *ext = (double *)malloc(sizeof(double) * (size_t)(histLen + 1));
    double *hist = (double *)calloc((size_t)(histLen + 1), sizeof(double));
    for (int i = 0; i < M; i++) ext[i] = intercept_amt;
    for (int i = 0; i < n; i++) ext[M + i] = dts[d + i];
    iterate_arma(ext, hist, histLen, +1, ext, NULL, NULL, p, q, I, coef);          /* :708 */
    double maTerms[ORC_KMAX];
    for (int i = histLen - M, j = 0; i < histLen; i++, j++) maTerms[j] = ext[i] - hist[i];  /* :711-713 */
    int fl = nFuture + M;
    double *fwd = (double *)calloc((size_t)(fl + 1), sizeof(double));
    for (int i = 0; i < M; i++) fwd[i] = hist[histLen - M + i];                     /* :717 */
    /* :720 iterateARMA(forward, forward, +, goldStandard = forward, initMATerms = maTerms).
     * maTerms has maxLag entries; iterateARMA uses the array as given (length maxLag >= q). */
    {
        double ma[ORC_KMAX];
        for (int j = 0; j < M; j++) ma[j] = maTerms[j];
        for (int i = M; i < fl; i++) {
            double t = (double)I * coef[0];
            fwd[i] = fwd[i] + t;
            for (int j = 0; j < p && i - j - 1 >= 0; j++) fwd[i] = fwd[i] + fwd[i - j - 1] * coef[I + j];
            for (int j = 0; j < q; j++) fwd[i] = fwd[i] + ma[j] * coef[I + p + j];
            double err = fwd[i] - fwd[i];
            update_ma_errors(ma, M, err);   /* updateMAErrors(maTerms) works on the array's own length */
        }
    }
    int L = T + nFuture;
    for (int i = 0; i < L; i++) out[i] = 0.0;
    for (int i = 0; i < d && i < T; i++) out[i] = ts[i];                             /* :724 */
    for (int i = 0; i < histLen - M; i++) out[d + i] = hist[M + i];                  /* :726 */
    for (int i = 0; i < nFuture; i++) out[T + i] = fwd[M + i];                       /* :728 */
    if (d != 0) {                                                                    /* :730-762 */
        /* diffMatrix(i, i to -1) := differencesOfOrderD(diffMatrix(i-1, i to -1), 1) */
        double *dm = (double *)calloc((size_t)(d + 1) * (size_t)T, sizeof(double));
        for (int t = 0; t < T; t++) dm[t] = ts[t];
        double *buf = (double *)malloc(sizeof(double) * (size_t)T);
        for (int i = 1; i <= d; i++) {
            int len = T - i;
            if (len > 0) {
                orc_differences_of_order_d(dm + (size_t)(i - 1) * T + i, len, 1, buf);
                for (int t = 0; t < len; t++) dm[(size_t)i * T + i + t] = buf[t];
            }
        }
        for (int i = d; i < histLen - M; i++) {                                      /* :745-751 */
            /* sum(diffMatrix(0 until d, i - 1)) — Breeze sum over a column slice, sequential from 0 */
            double s = 0.0;
            for (int r = 0; r < d; r++) s = s + dm[(size_t)r * T + (i - 1)];
            out[i] = s + hist[M + i];
        }
        /* diag(diffMatrix(0 until d, -d to -1)) */
        double *fi = (double *)malloc(sizeof(double) * (size_t)(d + nFuture));
        for (int r = 0; r < d; r++) fi[r] = dm[(size_t)r * T + (T - d + r)];
        for (int i = 0; i < nFuture; i++) fi[d + i] = fwd[M + i];
        double *fo = (double *)malloc(sizeof(double) * (size_t)(d + nFuture));
        orc_inverse_differences_of_order_d(fi, d + nFuture, d, fo);
        for (int i = 0; i < d + nFuture; i++) out[L - (d + nFuture) + i] = fo[i];    /* :761 */
        free(fi); free(fo); free(dm); free(buf);
    }
    free(dts); free(ext); free(hist); free(fwd);
}

/* ARIMAModel.addTimeDependentEffects(ts, dest)  ARIMA.scala:655-667 (the `sample` generator) */
void orc_add_time_dependent_effects(const double *ts, int n, int p, int d, int q, int I, const double *coef,
                                    double *out) {
    int M = p > q ? p : q;
    double ia = I ? coef[0] : 0.0;
    double *ch = (double *)malloc(sizeof(double) * (size_t)(M + n + 1));
    double *er = (double *)malloc(sizeof(double) * (size_t)(M + n + 1));
    for (int i = 0; i < M; i++) ch[i] = ia;
    for (int i = 0; i < n; i++) ch[M + i] = ts[i];
    memcpy(er, ch, sizeof(double) * (size_t)(M + n));
    iterate_arma(ch, ch, M + n, +1, NULL, er, NULL, p, q, I, coef);
    orc_inverse_differences_of_order_d(ch + M, n, d, out);
    free(ch); free(er);
}

/* ARIMAModel.removeTimeDependentEffects(ts, dest)  ARIMA.scala:629-644 */
void orc_remove_time_dependent_effects(const double *ts, int n, int p, int d, int q, int I,
                                       const double *coef, double *out) {
    int M = p > q ? p : q;
    double ia = I ? coef[0] : 0.0;
    double *df = (double *)malloc(sizeof(double) * (size_t)(n + 1));
    orc_differences_of_order_d(ts, n, d, df);
    double *ext = (double *)malloc(sizeof(double) * (size_t)(M + n + 1));
    double *ch = (double *)malloc(sizeof(double) * (size_t)(M + n + 1));
    for (int i = 0; i < M; i++) ext[i] = ia;
    for (int i = 0; i < n; i++) ext[M + i] = df[i];
    memcpy(ch, ext, sizeof(double) * (size_t)(M + n));
    iterate_arma(ext, ch, M + n, -1, NULL, ch, NULL, p, q, I, coef);
    for (int i = 0; i < n; i++) out[i] = ch[M + i];
    free(df); free(ext); free(ch);
}
