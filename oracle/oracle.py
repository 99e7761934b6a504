"""ctypes wrapper of the CPU restatement (oracle/arima_oracle.c) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, as the checker or
as the timed CPU baseline; the product path (spark-timeseries_amd/) never does.

Parity pinning: see the header of arima_oracle.c. The functions here add the stationarity / invertibility
oracle, restated the way the reference computes it: eigenvalues of the companion matrix (ARIMA.findRoots,
ARIMA.scala:381-399, commons EigenDecomposition) and `!roots.exists(_.abs() <= 1.0)` (ARIMA.scala:812-815).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libarima_oracle.so")
_lib = None

ST_NAMES = {0: "OK", 1: "MAX_EVAL", 2: "BRACKET_MAX_EVAL", 3: "MAX_ITER", 4: "SINGULAR",
            5: "NOT_ENOUGH_DATA", 6: "NO_DATA", 7: "BAD_INTERVAL", 8: "ZERO_PARAMS",
            9: "UNSUPPORTED_METHOD", 10: "SERIES_TOO_SHORT", 11: "NOT_STATIONARY", 12: "NO_MODEL",
            14: "TOO_FEW_PARAMS"}                          # 13, 15 retired: RESCUE is restated

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)

# Breeze 0.12 semantics of the overlapping row-slice copy at ARIMA.scala:526: 1 = element-wise
# ascending copy (every lag row becomes row 0, "smear"), the default; 0 = memmove-like row shift.
DEFAULT_SMEAR = 1


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_log.restype = ctypes.c_double
        L.orc_log.argtypes = [ctypes.c_double]
        L.orc_loglik_css_arma.restype = ctypes.c_double
        L.orc_loglik_css_arma.argtypes = [_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp]
        L.orc_gradient_css_arma.restype = None
        L.orc_gradient_css_arma.argtypes = [_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp,
                                            ctypes.c_int, _dp]
        L.orc_differences_of_order_d.argtypes = [_dp, ctypes.c_int, ctypes.c_int, _dp]
        L.orc_inverse_differences_of_order_d.argtypes = [_dp, ctypes.c_int, ctypes.c_int, _dp]
        L.orc_ols.restype = ctypes.c_int
        L.orc_ols.argtypes = [_dp, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp]
        L.orc_ar_fit.restype = ctypes.c_int
        L.orc_ar_fit.argtypes = [_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, _dp]
        L.orc_hannan_rissanen.restype = ctypes.c_int
        L.orc_hannan_rissanen.argtypes = [_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp]
        L.orc_fit.restype = ctypes.c_int
        L.orc_fit.argtypes = [_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                              ctypes.c_int, _dp, ctypes.c_int, _dp, _dp, _ip]
        L.orc_fit_batch.restype = ctypes.c_int
        L.orc_fit_batch.argtypes = [_dp, ctypes.c_longlong, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, ctypes.c_int, _dp, _dp, _ip,
                                    _ip]
        L.orc_forecast.argtypes = [_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   _dp, ctypes.c_int, _dp]
        L.orc_add_time_dependent_effects.argtypes = [_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                     ctypes.c_int, ctypes.c_int, _dp, _dp]
        L.orc_remove_time_dependent_effects.argtypes = [_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                        ctypes.c_int, ctypes.c_int, _dp, _dp]
        L.orc_lag_matrix.restype = ctypes.c_int
        L.orc_lag_matrix.argtypes = [_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp]
        L.orc_kpss.restype = ctypes.c_int
        L.orc_kpss.argtypes = [_dp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        L.orc_set_threads.restype = None
        L.orc_set_threads.argtypes = [ctypes.c_int]
        _lib = L
    return _lib


def lag_matrix(x, max_lag, include_original):
    """UnivariateTimeSeries.lag / Lag.lagMatTrimBoth (Lag.scala:33-99): (rows, cols, column-major values) -- the
    layout Matrices.dense(rows, cols, values) takes, and the design the AR / Hannan-Rissanen regressions use."""
    x, px = _c(x)
    cols = max_lag + (1 if include_original else 0)
    out = np.zeros(max(1, (len(x) - max_lag) * cols))
    rows = lib().orc_lag_matrix(px, len(x), max_lag, int(include_original), out.ctypes.data_as(_dp))
    return rows, cols, out[: rows * cols]


def set_threads(n):
    """OpenMP threads of fit_batch (bench.py's CPU baseline: the lease's share, then one core)."""
    lib().orc_set_threads(int(n))


def _c(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(_dp)


def log(x):
    return lib().orc_log(float(x))


def differences_of_order_d(ts, d):
    ts, pt = _c(ts)
    out = np.empty_like(ts)
    lib().orc_differences_of_order_d(pt, len(ts), d, out.ctypes.data_as(_dp))
    return out


def inverse_differences_of_order_d(ts, d):
    ts, pt = _c(ts)
    out = np.empty_like(ts)
    lib().orc_inverse_differences_of_order_d(pt, len(ts), d, out.ctypes.data_as(_dp))
    return out


def loglik_css_arma(diffed, p, q, intercept, coef):
    y, py = _c(diffed)
    c, pc = _c(coef)
    return lib().orc_loglik_css_arma(py, len(y), p, q, int(intercept), pc)


def loglik_css(ts, p, d, q, intercept, coef):
    """ARIMAModel.logLikelihoodCSS (ARIMA.scala:417-420)."""
    return loglik_css_arma(differences_of_order_d(ts, d)[d:], p, q, intercept, coef)


def gradient_css_arma(diffed, p, q, intercept, coef, smear=DEFAULT_SMEAR):
    y, py = _c(diffed)
    c, pc = _c(coef)
    g = np.empty(len(c))
    lib().orc_gradient_css_arma(py, len(y), p, q, int(intercept), pc, int(smear), g.ctypes.data_as(_dp))
    return g


def ols(Y, X, intercept):
    Y, py = _c(Y)
    X = np.ascontiguousarray(X, dtype=np.float64).reshape(len(Y), -1)
    beta = np.empty(X.shape[1] + (1 if intercept else 0) + 1)
    st = lib().orc_ols(py, X.ctypes.data_as(_dp), len(Y), X.shape[1], int(intercept), beta.ctypes.data_as(_dp))
    return st, beta[: X.shape[1] + (1 if intercept else 0)]


def ar_fit(ts, max_lag, no_intercept=False):
    ts, pt = _c(ts)
    c = ctypes.c_double()
    coef = np.empty(max(max_lag, 1))
    st = lib().orc_ar_fit(pt, len(ts), max_lag, int(no_intercept), ctypes.byref(c), coef.ctypes.data_as(_dp))
    return st, c.value, coef[:max_lag]


def hannan_rissanen(diffed, p, q, intercept):
    y, py = _c(diffed)
    k = p + q + (1 if intercept else 0)
    out = np.empty(max(k, 1))
    st = lib().orc_hannan_rissanen(py, len(y), p, q, int(intercept), out.ctypes.data_as(_dp))
    return st, out[:k]


def fit(ts, p, d, q, intercept=True, method=0, user_init=None, smear=DEFAULT_SMEAR):
    """ARIMA.fitModel restated. Returns dict(status, coef, ll, n_eval, n_grad, n_iter)."""
    ts, pt = _c(ts)
    k = p + q + (1 if intercept else 0)
    coef = np.empty(max(k, 1))
    ll = ctypes.c_double()
    cnt = (ctypes.c_int * 3)()
    ui = None
    if user_init is not None:
        ui_arr, ui = _c(user_init)
    st = lib().orc_fit(pt, len(ts), p, d, q, int(intercept), int(method), ui, int(smear),
                       coef.ctypes.data_as(_dp), ctypes.byref(ll), cnt)
    return dict(status=st, coef=coef[:k], ll=ll.value, n_eval=cnt[0], n_grad=cnt[1], n_iter=cnt[2])


def fit_batch(series, p, d, q, intercept=True, method=0, user_init=None, smear=DEFAULT_SMEAR, threads=None):
    """Batch of fits (OpenMP over series). series: (N, T) float64. Returns (status, coef, ll, counters)."""
    series = np.ascontiguousarray(series, dtype=np.float64)
    N, T = series.shape
    k = p + q + (1 if intercept else 0)
    coef = np.empty((N, max(k, 1)))
    if k == 0:
        coef = np.empty((N, 1))
    coef_k = np.empty((N, k)) if k else np.empty((N, 0))
    ll = np.empty(N)
    status = np.empty(N, dtype=np.int32)
    counters = np.empty((N, 3), dtype=np.int32)
    ui = None
    if user_init is not None:
        ui_arr = np.ascontiguousarray(user_init, dtype=np.float64).reshape(N, k)
        ui = ui_arr.ctypes.data_as(_dp)
    if threads is not None:
        os.environ["OMP_NUM_THREADS"] = str(threads)
    buf = np.empty((N, k)) if k else np.empty((N, 1))
    lib().orc_fit_batch(series.ctypes.data_as(_dp), N, T, p, d, q, int(intercept), int(method), ui, int(smear),
                        buf.ctypes.data_as(_dp), ll.ctypes.data_as(_dp), status.ctypes.data_as(_ip),
                        counters.ctypes.data_as(_ip))
    coef_k[:] = buf[:, :k]
    return status, coef_k, ll, counters


def forecast(ts, p, d, q, intercept, coef, n_future):
    ts, pt = _c(ts)
    c, pc = _c(coef)
    out = np.empty(len(ts) + n_future)
    lib().orc_forecast(pt, len(ts), p, d, q, int(intercept), pc, n_future, out.ctypes.data_as(_dp))
    return out


def add_time_dependent_effects(ts, p, d, q, intercept, coef):
    ts, pt = _c(ts)
    c, pc = _c(coef)
    out = np.empty_like(ts)
    lib().orc_add_time_dependent_effects(pt, len(ts), p, d, q, int(intercept), pc, out.ctypes.data_as(_dp))
    return out


def remove_time_dependent_effects(ts, p, d, q, intercept, coef):
    ts, pt = _c(ts)
    c, pc = _c(coef)
    out = np.empty_like(ts)
    lib().orc_remove_time_dependent_effects(pt, len(ts), p, d, q, int(intercept), pc, out.ctypes.data_as(_dp))
    return out


# ---- stationarity / invertibility: ARIMA.findRoots (companion-matrix eigenvalues), ARIMA.scala:381-399 ----
def find_roots(coefficients):
    c = np.asarray(coefficients, dtype=np.float64)
    n = len(c) - 1
    if n < 1:
        return np.zeros(0, dtype=complex)
    comp = np.zeros((n, n))
    a = c[n]
    comp[n - 1, :] = -c[:n] / a
    if n > 1:
        comp[: n - 1, 1:] = np.eye(n - 1)
    return np.linalg.eigvals(comp)


def _all_roots_outside_unit_circle(poly):
    """`!findRoots(poly).exists(_.abs() <= 1.0)` (ARIMA.scala:812-815). Degenerate polynomials, where the reference's
    companion matrix holds infinities or NaNs and commons EigenDecomposition's outcome is not pinned by any test,
    follow the device's rule (arima_device.hpp roots_outside_unit_circle): a non-finite coefficient -> False; a zero
    leading coefficient is a root at infinity (outside), so the degree drops (for p = 1 this is exactly the
    reference: the 1 x 1 companion [-Inf] has |root| = Inf)."""
    poly = np.asarray(poly, dtype=np.float64)
    if not np.all(np.isfinite(poly)):
        return False
    n = len(poly) - 1
    while n >= 1 and poly[n] == 0.0:
        n -= 1
    roots = find_roots(poly[: n + 1])
    return not np.any(np.abs(roots) <= 1.0)


def is_stationary(coef, p, q, intercept):
    """ARIMAModel.isStationary, ARIMA.scala:777-785."""
    if p == 0:
        return True
    off = 1 if intercept else 0
    return _all_roots_outside_unit_circle(np.concatenate([[1.0], -np.asarray(coef[off:off + p])]))


def is_invertible(coef, p, q, intercept):
    """ARIMAModel.isInvertible, ARIMA.scala:795-803."""
    if q == 0:
        return True
    off = 1 if intercept else 0
    return _all_roots_outside_unit_circle(np.concatenate([[1.0], np.asarray(coef[off + p:])]))


def model_flags(coef, p, q, intercept):
    return (1 if is_stationary(coef, p, q, intercept) else 0) | (2 if is_invertible(coef, p, q, intercept) else 0)


def order_search(series, max_p=5, max_d=2, max_q=5, intercept_mode=2, method=0, smear=DEFAULT_SMEAR):
    """Min-approxAIC selection over the (d, p, q, intercept) grid.
    approxAIC = -2 * logLikelihoodCSS + 2 * (p + q + interceptTerm) (ARIMA.scala:826-830) among fits that
    returned normally and are stationary and invertible (ARIMA.scala:342); ties keep the first candidate in
    (d, p, q, intercept) order. Returns (order N x 4, coef N x 11, aic N) like arima_order_search_batch."""
    series = np.ascontiguousarray(np.atleast_2d(series), dtype=np.float64)
    N = series.shape[0]
    order = np.full((N, 4), -1, dtype=np.int32)
    coef_best = np.full((N, 11), np.nan)
    aic_best = np.full(N, np.inf)
    i_vals = {0: [0], 1: [1], 2: [0, 1]}[intercept_mode]
    for d in range(max_d + 1):
        for p in range(max_p + 1):
            for q in range(max_q + 1):
                for I in i_vals:
                    k = p + q + I
                    st, coef, ll, _ = fit_batch(series, p, d, q, I, method, smear=smear)
                    for i in range(N):
                        if st[i] != 0 or model_flags(coef[i], p, q, I) != 3:
                            continue
                        aic = -2.0 * ll[i] + float(2 * k)
                        # `_ < curBestAIC`, curBestAIC starting at Double.MaxValue (ARIMA.scala:323, :344)
                        if aic < aic_best[i] and aic < 1.7976931348623157e308:
                            aic_best[i] = aic
                            order[i] = (p, d, q, I)
                            coef_best[i] = 0.0
                            coef_best[i, :k] = coef[i, :k]
    return order, coef_best, aic_best


# ---- ARIMA.autoFit (ARIMA.scala:280-375) -----------------------------------------------------------------------
KPSS_CRITICAL = {0: {0.10: 0.347, 0.05: 0.463, 0.025: 0.574, 0.01: 0.739},      # "c"   (TimeSeriesStatisticalTests.scala:338-340)
                 1: {0.10: 0.119, 0.05: 0.146, 0.025: 0.176, 0.01: 0.216}}      # "ct"  (:349-351)

# autoFit outcomes beyond fitModel's (include/sparkts_arima.h)
ST_NOT_STATIONARY = 11      # "stationarity not achieved with differencing order <= maxD" (ARIMA.scala:293-296)
ST_NO_MODEL = 12            # no candidate qualified: curBestModel stays null (ARIMA.scala:322, :304 -> NPE)
CGD_FALLBACK_STATUSES = (1, 2, 3, 7)   # MaxEval, BracketFinder cap, MaxIter, SearchInterval: thrown by the optimizer


def kpss(ts, method="c"):
    """TimeSeriesStatisticalTests.kpsstest (stats/TimeSeriesStatisticalTests.scala:369-393): (status, statistic)."""
    ts, pt = _c(ts)
    stat = ctypes.c_double(float("nan"))
    st = lib().orc_kpss(pt, len(ts), 1 if method == "ct" else 0, ctypes.byref(stat))
    return st, stat.value


def autofit_select_d(ts, max_d):
    """autoFit's choice of d (ARIMA.scala:287-297): the first d in 0..max_d whose differencesOfOrderD(ts, d) -- NOT
    dropped -- passes kpsstest(_, "c") at 5 %. Returns (status, d): status != 0 when kpsstest throws (n <= 1) or no
    d passes (ST_NOT_STATIONARY)."""
    for d in range(max_d + 1):
        st, stat = kpss(differences_of_order_d(ts, d), "c")
        if st != 0:
            return st, -1
        if stat < KPSS_CRITICAL[0][0.05]:
            return 0, d
    return ST_NOT_STATIONARY, -1


def autofit(ts, max_p=5, max_d=2, max_q=5, smear=DEFAULT_SMEAR, trace=None):
    """ARIMA.autoFit (ARIMA.scala:280-304) + findBestARMAModel (:310-375), restated with its quirks:
    - the ARMA fits run on differencesOfOrderD(ts, d) WITHOUT .drop(d) (:298): the first d raw values stay in;
    - the intercept is used only if d <= 1 (:300);
    - the first candidates (0,0), (2,2), (1,0), (0,1) are not bounds-checked (:325-327);
    - the neighbourhood varies p and flips the intercept but never q (`curBestModel.q`, :364);
    - a candidate counts if its fit returned normally, it is stationary and invertible (:342) and its approxAIC
      (-2 * logLikelihoodCSS + 2 * (p + q + c), :826-830) is strictly below the incumbent's (starting at
      Double.MaxValue, :323); the new incumbent is the first minimum in candidate order (minBy, :350).
    fitTryBothStrategies (:315-319): when css-cgd throws in the optimizer, the candidate is refitted with css-bobyqa
    (bobyqa_oracle.c, RESCUE included) from the same initial parameters.
    Returns dict(status, order (p, d, q, intercept), coef (11, zero-padded), aic, n_fits)."""
    ts = np.ascontiguousarray(ts, dtype=np.float64)
    out = dict(status=0, order=(-1, -1, -1, -1), coef=np.full(11, np.nan), aic=float("inf"), n_fits=0)
    st, d = autofit_select_d(ts, max_d)
    if st != 0:
        out["status"] = st
        return out
    diffed = differences_of_order_d(ts, d)
    start_i = 1 if d <= 1 else 0
    best_aic = 1.7976931348623157e308
    best = None
    past = set()
    nxt = [(0, 0, start_i), (2, 2, start_i), (1, 0, start_i), (0, 1, start_i)]
    cache = {}
    while True:
        past.update(nxt)
        improving = []
        for (p, q, I) in nxt:
            if (p, q, I) not in cache:
                r = fit(diffed, p, 0, q, I, smear=smear)
                out["n_fits"] += 1
                if r["status"] in CGD_FALLBACK_STATUSES and not (p > 0 and q == 0):
                    r = fit(diffed, p, 0, q, I, method=1)          # Try(... "css-bobyqa")
                cache[(p, q, I)] = r
            r = cache[(p, q, I)]
            if r["status"] != 0 or model_flags(r["coef"], p, q, I) != 3:
                continue
            aic = -2.0 * r["ll"] + float(2 * (p + q + I))
            if aic < best_aic:
                improving.append((aic, (p, q, I), r))
        if trace is not None:
            trace.append(list(nxt))
        if not improving:
            break
        aic, (p, q, I), r = min(improving, key=lambda x: x[0])      # first minimum in list order
        best_aic, best = aic, (p, q, I, r)
        surround = []
        for pd_ in (-1, 0, 1):
            for qd in (-1, 0, 1):
                inc = (1 - I) if (pd_ == 0 and qd == 0) else I
                surround.append((p + pd_, q, inc))
        nxt = [c for c in surround if c not in past and 0 <= c[0] <= max_p and 0 <= c[1] <= max_q]
    if best is None:
        out["status"] = ST_NO_MODEL
        return out
    p, q, I, r = best
    out["order"] = (p, d, q, I)
    out["coef"][:] = 0.0
    out["coef"][: p + q + I] = r["coef"]
    out["aic"] = best_aic
    out["status"] = 0
    return out
