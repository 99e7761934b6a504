"""MI355X-native mirror of python/sparkts/models/ARIMA.py (spark-ts) over the HIP engine.

Same names, argument meaning and error behaviour as the reference's Python binding (which forwards to
com.cloudera.sparkts.models.ARIMA over py4j, python/sparkts/models/ARIMA.py:62-104, 106-262); `sc` is accepted
and ignored (there is no JVM). Where the reference throws a Java exception, the mirror raises an exception of
the same name (subclass of ARIMAFitError). Batched entry points (`fit_models`) are the drop-in for
TimeSeriesRDD.mapSeries over ARIMA fits (one ABI call per partition, TimeSeriesRDD.scala:249-260).
"""
import numpy as np

from .. import _lib


class ARIMAFitError(RuntimeError):
    """Base of the per-series failures (status != OK)."""

    status = None


class TooManyEvaluationsException(ARIMAFitError):
    pass


class TooManyIterationsException(ARIMAFitError):
    pass


class SingularMatrixException(ARIMAFitError):
    pass


class MathIllegalArgumentException(ARIMAFitError):
    pass


class NoDataException(ARIMAFitError):
    pass


class NumberIsTooLargeException(ARIMAFitError):
    pass


class ArithmeticException(ARIMAFitError):
    pass


class UnsupportedOperationException(ARIMAFitError):
    pass


class IndexOutOfBoundsException(ARIMAFitError):
    pass


class StationarityNotAchieved(ARIMAFitError):
    """autoFit: `throw new Exception(s"stationarity not achieved with differencing order <= $maxD")` (ARIMA.scala:295)."""


class NullPointerException(ARIMAFitError):
    """autoFit: no candidate model qualified, so `bestModel.p` dereferences null (ARIMA.scala:302-304)."""


class NumberIsTooSmallException(ARIMAFitError):
    """css-bobyqa: BOBYQAOptimizer needs at least two parameters."""


_EXC = {
    _lib.ST_MAX_EVAL: TooManyEvaluationsException,
    _lib.ST_BRACKET_MAX_EVAL: TooManyEvaluationsException,
    _lib.ST_MAX_ITER: TooManyIterationsException,
    _lib.ST_SINGULAR: SingularMatrixException,
    _lib.ST_NOT_ENOUGH_DATA: MathIllegalArgumentException,
    _lib.ST_NO_DATA: NoDataException,
    _lib.ST_BAD_INTERVAL: NumberIsTooLargeException,
    _lib.ST_ZERO_PARAMS: ArithmeticException,
    _lib.ST_UNSUPPORTED_METHOD: UnsupportedOperationException,
    _lib.ST_SERIES_TOO_SHORT: IndexOutOfBoundsException,
    _lib.ST_NOT_STATIONARY: StationarityNotAchieved,
    _lib.ST_NO_MODEL: NullPointerException,
    _lib.ST_TOO_FEW_PARAMS: NumberIsTooSmallException,
}


def raise_for_status(status):
    if status != _lib.ST_OK:
        exc = _EXC.get(int(status), ARIMAFitError)
        e = exc(f"ARIMA fit failed: status {int(status)} ({_lib.load().arima_status_name(int(status)).decode()})")
        e.status = int(status)
        raise e


def _method_code(method):
    if method not in _lib.METHODS:
        return 99      # unknown method string -> UnsupportedOperationException (ARIMA.scala:108)
    return _lib.METHODS[method]


def autofit(ts, maxp=5, maxd=2, maxq=5, sc=None, device=None):
    """ARIMA.autoFit (ARIMA.scala:280-375), the reference binding's `autofit` (python/sparkts/models/ARIMA.py:25-60):
    d from the KPSS test, then the stepwise (p, q, intercept) walk with css-cgd fits and fitTryBothStrategies'
    css-bobyqa retries. Raises what the reference throws (StationarityNotAchieved, NullPointerException, the KPSS
    regression's MathIllegalArgumentException)."""
    ts = np.asarray(ts, dtype=np.float64).ravel()
    r = autofit_models(ts[None, :], maxp, maxd, maxq, device=device)
    return r.model(0)


class AutoFitBatchResult:
    """Per-series outputs of a batched autoFit (the arrays arima_autofit_batch fills)."""

    def __init__(self, r, device):
        self.order = r["order"]
        self.coefficients = r["coef"]
        self.aic = r["aic"]
        self.status = r["status"]
        self.n_fits = r["n_fits"]
        self._device = device

    def model(self, i):
        raise_for_status(int(self.status[i]))
        p, d, q, I = (int(v) for v in self.order[i])
        return ARIMAModel(p, d, q, self.coefficients[i, :p + q + I], bool(I), device=self._device)


def autofit_models(series, maxp=5, maxd=2, maxq=5, device=None):
    """Batched ARIMA.autoFit over (N, T) series (one call per partition bucket, the mapSeries drop-in for autofit).
    Never raises for per-series outcomes; inspect `.status`."""
    eng = _lib.Engine.get(device)
    return AutoFitBatchResult(eng.autofit(series, maxp, maxd, maxq), device)


def fit_model(p, d, q, ts, includeIntercept=True, method="css-cgd", userInitParams=None, sc=None, device=None):
    """ARIMA.fitModel (ARIMA.scala:79-116), one series. Raises the reference's exception on failure."""
    ts = np.asarray(ts, dtype=np.float64).ravel()
    res = fit_models(p, d, q, ts[None, :], includeIntercept, method, userInitParams, device=device)
    raise_for_status(res.status[0])
    return ARIMAModel(p, d, q, res.coefficients[0], includeIntercept, device=device)


class FitBatchResult:
    """Per-series outputs of a batched fit (the arrays the C ABI fills)."""

    def __init__(self, p, d, q, include_intercept, r, stats):
        self.p, self.d, self.q, self.has_intercept = p, d, q, include_intercept
        self.coefficients = r["coef"]
        self.css_loglik = r["ll"]
        self.status = r["status"]
        self.n_eval = r["n_eval"]
        self.n_grad = r["n_grad"]
        self.flags = r["flags"]
        self.stats = stats

    def model(self, i):
        raise_for_status(self.status[i])
        return ARIMAModel(self.p, self.d, self.q, self.coefficients[i], self.has_intercept)

    @property
    def converged(self):
        return self.status == _lib.ST_OK


def fit_models(p, d, q, series, includeIntercept=True, method="css-cgd", userInitParams=None, device=None):
    """Batched ARIMA.fitModel: `series` is (N, T) float64, one row per series (one Spark partition bucket).

    Never raises for per-series failures; inspect `.status` (ARIMA_ST_* codes, include/sparkts_arima.h)."""
    eng = _lib.Engine.get(device)
    r = eng.fit_batch(series, p, d, q, includeIntercept, _method_code(method), userInitParams)
    return FitBatchResult(p, d, q, includeIntercept, r, eng.stats())


def order_search(series, maxp=5, maxd=2, maxq=5, intercept_mode=2, device=None):
    """Config C5: per series, fit every (d <= maxd, p <= maxp, q <= maxq, intercept) and keep
    the minimum approxAIC (ARIMA.scala:826-830) among fits that returned normally and are stationary and
    invertible (autoFit's filter, ARIMA.scala:342); ties keep the first in (d, p, q, intercept) order.
    intercept_mode: 0 = without, 1 = with, 2 = both. Returns a list with an ARIMAModel (or None) per series."""
    eng = _lib.Engine.get(device)
    order, coef, _ = eng.order_search(series, maxp, maxd, maxq, intercept_mode)
    out = []
    for i in range(order.shape[0]):
        p, d, q, I = (int(v) for v in order[i])
        if p < 0:
            out.append(None)
        else:
            out.append(ARIMAModel(p, d, q, coef[i, :p + q + I], bool(I), device=device))
    return out


class ARIMAModel:
    """ARIMAModel (ARIMA.scala:402-831) with the reference Python binding's method names."""

    def __init__(self, p=0, d=0, q=0, coefficients=None, hasIntercept=True, jmodel=None, sc=None, device=None):
        self.p, self.d, self.q = int(p), int(d), int(q)
        self.coefficients = np.asarray(coefficients, dtype=np.float64).copy()
        self.has_intercept = bool(hasIntercept)
        self._device = device

    @property
    def _eng(self):
        return _lib.Engine.get(self._device)

    def log_likelihood_css(self, y):
        """logLikelihoodCSS (ARIMA.scala:417-420)."""
        return float(self._eng.css_loglik(np.asarray(y, dtype=np.float64)[None, :], self.p, self.d, self.q,
                                          self.has_intercept, self.coefficients)[0])

    def log_likelihood_css_arma(self, diffedy):
        """logLikelihoodCSSARMA (ARIMA.scala:430-445) on an already differenced series."""
        return float(self._eng.css_loglik(np.asarray(diffedy, dtype=np.float64)[None, :], self.p, 0, self.q,
                                          self.has_intercept, self.coefficients)[0])

    def gradient_log_likelihood_css_arma(self, diffedy):
        """gradientlogLikelihoodCSSARMA (ARIMA.scala:465-534)."""
        return self._eng.css_gradient(np.asarray(diffedy, dtype=np.float64)[None, :], self.p, self.q,
                                      self.has_intercept, self.coefficients)[0]

    def sample(self, n, seed=None):
        """sample (ARIMA.scala:655-678; python/sparkts/models/ARIMA.py:182-194): n values of this ARIMA(p, d, q)
        process -- M copies of the intercept, the ARMA filter over N(0, 1) noise with the noise as the errors, the
        prefix dropped, then inverseDifferencesOfOrderD(., d), in the reference's operation order. The reference
        draws its noise from an unseeded JDKRandomGenerator; here it is Philox4x32-10 + Box-Muller
        (arima_sample_batch_device) under `seed` (a fresh random one by default). Orders up to p, q <= 8."""
        import torch
        if seed is None:
            seed = int.from_bytes(np.random.default_rng().bytes(8), "little")
        n = int(n)
        eng = self._eng
        out = torch.empty((1, max(n, 1)), dtype=torch.float64, device=f"cuda:{eng.device}")
        if n > 0:
            eng.sample_device(out.data_ptr(), 1, n, n, self.p, self.d, self.q, self.has_intercept, self.coefficients,
                              0.0, int(seed) & ((1 << 64) - 1), 0)
        return out[0, :n].cpu().numpy()

    def forecast(self, ts, nfuture):
        """forecast (ARIMA.scala:696-764)."""
        return self._eng.forecast(np.asarray(ts, dtype=np.float64)[None, :], self.p, self.d, self.q,
                                  self.has_intercept, self.coefficients, int(nfuture))[0]

    def is_stationary(self):
        """isStationary (ARIMA.scala:777-785)."""
        f = self._eng.model_flags(self.coefficients[None, :], self.p, self.q, self.has_intercept)[0]
        return bool(f & _lib.FLAG_STATIONARY)

    def is_invertible(self):
        """isInvertible (ARIMA.scala:795-803)."""
        f = self._eng.model_flags(self.coefficients[None, :], self.p, self.q, self.has_intercept)[0]
        return bool(f & _lib.FLAG_INVERTIBLE)

    def approx_aic(self, ts):
        """approxAIC (ARIMA.scala:826-830)."""
        k = self.p + self.q + (1 if self.has_intercept else 0)
        return -2 * self.log_likelihood_css(ts) + 2 * k
