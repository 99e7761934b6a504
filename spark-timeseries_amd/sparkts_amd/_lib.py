"""ctypes binding of libsparkts_arima.so (the C ABI declared in include/sparkts_arima.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU is visible, every compute call
raises. Only symbol loading works without a GPU (used by the CPU test-suite to check the exported ABI).
"""
import ctypes
import os
import threading

import numpy as np

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))      # spark-timeseries_amd/
LIB_PATH = os.environ.get("SPARKTS_ARIMA_LIB", os.path.join(_PKG_ROOT, "libsparkts_arima.so"))

ARIMA_OK = 0
ARIMA_E_INVALID_ARG = -1
ARIMA_E_UNSUPPORTED = -2
ARIMA_E_DEVICE = -3
ARIMA_E_OOM = -4

ST_OK = 0
ST_MAX_EVAL = 1
ST_BRACKET_MAX_EVAL = 2
ST_MAX_ITER = 3
ST_SINGULAR = 4
ST_NOT_ENOUGH_DATA = 5
ST_NO_DATA = 6
ST_BAD_INTERVAL = 7
ST_ZERO_PARAMS = 8
ST_UNSUPPORTED_METHOD = 9
ST_SERIES_TOO_SHORT = 10
ST_NOT_STATIONARY = 11      # autoFit: no d <= max_d passes KPSS
ST_NO_MODEL = 12            # autoFit: no candidate qualified
ST_TOO_FEW_PARAMS = 14      # css-bobyqa needs >= 2 parameters (NumberIsTooSmallException)

METHOD_CSS_CGD = 0
METHOD_CSS_BOBYQA = 1
METHODS = {"css-cgd": METHOD_CSS_CGD, "css-bobyqa": METHOD_CSS_BOBYQA}

FLAG_STATIONARY = 1
FLAG_INVERTIBLE = 2

# arima_set_option("smear", .) default: Breeze 0.12's element-wise copy of the overlapping row slice at
# ARIMA.scala:526; 0 selects the memmove-like row shift.
DEFAULT_SMEAR = 1

# every symbol include/sparkts_arima.h declares (checked by tests/test_abi.py)
EXPORTED = [
    "arima_create", "arima_destroy", "arima_last_error", "arima_status_name", "arima_num_params",
    "arima_get_last_stats", "arima_set_option", "arima_get_option", "arima_fit_batch", "arima_fit_batch_device",
    "arima_difference_batch", "arima_inverse_difference_batch", "arima_css_loglik_batch",
    "arima_css_gradient_batch", "arima_hannan_rissanen_batch", "arima_forecast_batch", "arima_model_flags_batch",
    "arima_sample_batch_device", "arima_order_search_batch", "arima_order_search_batch_device",
    "arima_forecast_batch_device", "arima_synchronize", "arima_autofit_batch", "arima_autofit_batch_device",
    "arima_kpss_batch",
]


class FitStats(ctypes.Structure):
    _fields_ = [("n_series", ctypes.c_int64), ("f_passes", ctypes.c_int64), ("g_passes", ctypes.c_int64),
                ("hr_passes", ctypes.c_int64), ("n_eval", ctypes.c_int64), ("n_grad", ctypes.c_int64),
                ("flops", ctypes.c_double), ("ms_difference", ctypes.c_double), ("ms_hr_init", ctypes.c_double),
                ("ms_cg_fit", ctypes.c_double), ("ms_total", ctypes.c_double),
                ("wave_f_passes", ctypes.c_int64), ("wave_g_passes", ctypes.c_int64), ("grid_blocks", ctypes.c_int64),
                ("spec_hits", ctypes.c_int64), ("wave_multi_passes", ctypes.c_int64), ("spec_chains", ctypes.c_int64),
                ("express_blocks", ctypes.c_int64), ("express_series", ctypes.c_int64),
                ("express_f_passes", ctypes.c_int64), ("express_g_passes", ctypes.c_int64),
                ("fault", ctypes.c_int64), ("fault_info", ctypes.c_int64 * 5),
                ("diag", ctypes.c_int64 * 6), ("ride_passes", ctypes.c_int64), ("series_done", ctypes.c_int64),
                ("express_pit_passes", ctypes.c_int64), ("express_pit_sweeps", ctypes.c_int64),
                ("express_pit_g_passes", ctypes.c_int64), ("wave_chains", ctypes.c_int64),
                ("low_util_passes", ctypes.c_int64), ("diag_step_cycles", ctypes.c_int64),
                ("diag_refill_cycles", ctypes.c_int64), ("merge_series", ctypes.c_int64),
                ("merge_waves", ctypes.c_int64)]

    def as_dict(self):
        d = {name: getattr(self, name) for name, _ in self._fields_}
        d["diag"] = list(self.diag)
        d["fault_info"] = list(self.fault_info)
        return d


class EngineError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()
_dp = ctypes.POINTER(ctypes.c_double)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p
_i32, _i64, _f64, _u64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_uint64


def _single_hip_runtime():
    """PyTorch-ROCm wheels bundle their own libamdhip64/libhsa-runtime64 (same SONAME as /opt/rocm's). If this
    library were loaded first, a later `import torch` would map a SECOND HIP runtime into the process and torch
    would see no GPU. Importing torch first makes the dynamic loader bind this library to torch's runtime, so a
    process that also uses torch (bench.py's torch.distributed plumbing, tests) has exactly one HIP runtime."""
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def load():
    """Load the shared library (no GPU needed). Raises if it is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        _single_hip_runtime()
        if not os.path.exists(LIB_PATH):
            raise EngineError(f"HIP library not built: {LIB_PATH} (run `python -c 'import __graft_entry__ as g; "
                              f"g.build()'` or `make -C spark-timeseries_amd/csrc`)")
        L = ctypes.CDLL(LIB_PATH)
        H = ctypes.c_void_p
        L.arima_create.argtypes = [ctypes.c_int, ctypes.POINTER(H)]
        L.arima_destroy.argtypes = [H]
        L.arima_last_error.argtypes = [H]
        L.arima_last_error.restype = ctypes.c_char_p
        L.arima_status_name.argtypes = [ctypes.c_int]
        L.arima_status_name.restype = ctypes.c_char_p
        L.arima_num_params.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.arima_get_last_stats.argtypes = [H, ctypes.POINTER(FitStats)]
        L.arima_set_option.argtypes = [H, ctypes.c_char_p, _i64]
        L.arima_get_option.argtypes = [H, ctypes.c_char_p, ctypes.POINTER(_i64)]
        L.arima_synchronize.argtypes = [H]
        L.arima_fit_batch.argtypes = [H, _dp, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _dp, _dp, _dp, _i32p,
                                      _i32p, _i32p, _u8p]
        L.arima_fit_batch_device.argtypes = [H, _vp, _i64, _i32, _i64, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp,
                                             _vp, _vp, _vp, _vp, _vp]
        L.arima_difference_batch.argtypes = [H, _dp, _i64, _i32, _i32, _dp]
        L.arima_inverse_difference_batch.argtypes = [H, _dp, _i64, _i32, _i32, _dp]
        L.arima_css_loglik_batch.argtypes = [H, _dp, _i64, _i32, _i32, _i32, _i32, _i32, _dp, _dp]
        L.arima_css_gradient_batch.argtypes = [H, _dp, _i64, _i32, _i32, _i32, _i32, _dp, _dp]
        L.arima_hannan_rissanen_batch.argtypes = [H, _dp, _i64, _i32, _i32, _i32, _i32, _dp, _i32p]
        L.arima_forecast_batch.argtypes = [H, _dp, _i64, _i32, _i32, _i32, _i32, _i32, _dp, _i32, _dp]
        L.arima_model_flags_batch.argtypes = [H, _dp, _i64, _i32, _i32, _i32, _u8p]
        L.arima_sample_batch_device.argtypes = [H, _vp, _i64, _i32, _i64, _i32, _i32, _i32, _i32, _dp, _f64, _u64,
                                                _i64, _vp]
        L.arima_forecast_batch_device.argtypes = [H, _vp, _i64, _i32, _i64, _i32, _i32, _i32, _i32, _vp, _i32, _vp,
                                                  _i64, _vp]
        L.arima_order_search_batch.argtypes = [H, _dp, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _i32p, _dp, _dp]
        L.arima_order_search_batch_device.argtypes = [H, _vp, _i64, _i32, _i64, _i32, _i32, _i32, _i32, _i32, _vp,
                                                      _vp, _vp, _vp]
        L.arima_autofit_batch.argtypes = [H, _dp, _i64, _i32, _i32, _i32, _i32, _i32p, _dp, _dp, _i32p, _i32p]
        L.arima_autofit_batch_device.argtypes = [H, _vp, _i64, _i32, _i64, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp,
                                                 _vp]
        L.arima_kpss_batch.argtypes = [H, _dp, _i64, _i32, _dp, _i32p]
        _lib = L
        return L


def _ptr(a, t=_dp):
    return a.ctypes.data_as(t) if a is not None else None


class Engine:
    """One handle per device (arima_create). Thread-safe: the library serialises calls per handle."""

    _engines = {}

    def __init__(self, device=0):
        self.L = load()
        h = ctypes.c_void_p()
        rc = self.L.arima_create(int(device), ctypes.byref(h))
        if rc != ARIMA_OK:
            raise EngineError(f"arima_create(device={device}) failed with {rc}: no usable HIP device")
        self.h = h
        self.device = device
        # engine-wide knobs from the environment (A/B runs of the test suite and the bench), any option:
        # SPARKTS_OPTIONS="hr_grid=1024,fit_pipeline=2"
        for kv in filter(None, os.environ.get("SPARKTS_OPTIONS", "").split(",")):
            name, _, val = kv.partition("=")
            self.set_option(name.strip(), int(val))

    @classmethod
    def get(cls, device=None):
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        with _lock:
            eng = cls._engines.get(device)
        if eng is None:
            eng = Engine(device)
            with _lock:
                cls._engines[device] = eng
        return eng

    def _check(self, rc, what):
        if rc != ARIMA_OK:
            msg = self.L.arima_last_error(self.h)
            raise EngineError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def set_option(self, name, value):
        self._check(self.L.arima_set_option(self.h, name.encode(), int(value)), "arima_set_option")

    def get_option(self, name):
        v = _i64()
        self._check(self.L.arima_get_option(self.h, name.encode(), ctypes.byref(v)), "arima_get_option")
        return int(v.value)

    def synchronize(self):
        """Wait for the device work of every call issued on this handle (the *_device calls are asynchronous)."""
        self._check(self.L.arima_synchronize(self.h), "arima_synchronize")

    def stats(self):
        s = FitStats()
        self._check(self.L.arima_get_last_stats(self.h, ctypes.byref(s)), "arima_get_last_stats")
        return s.as_dict()

    # ---- ARIMA.fitModel over a batch ---------------------------------------------------------------------
    def fit_batch(self, series, p, d, q, include_intercept=True, method="css-cgd", user_init=None):
        series = np.ascontiguousarray(series, dtype=np.float64)
        if series.ndim == 1:
            series = series[None, :]
        N, T = series.shape
        k = p + q + (1 if include_intercept else 0)
        m = METHODS.get(method, 99) if isinstance(method, str) else int(method)
        coef = np.empty((N, max(k, 1)))
        ll = np.empty(N)
        status = np.empty(N, dtype=np.int32)
        n_eval = np.empty(N, dtype=np.int32)
        n_grad = np.empty(N, dtype=np.int32)
        flags = np.empty(N, dtype=np.uint8)
        ui = None
        if user_init is not None:
            ui = np.ascontiguousarray(np.broadcast_to(np.asarray(user_init, dtype=np.float64), (N, k)))
        rc = self.L.arima_fit_batch(self.h, _ptr(series), N, T, p, d, q, int(bool(include_intercept)), m, _ptr(ui),
                                    _ptr(coef), _ptr(ll), _ptr(status, _i32p), _ptr(n_eval, _i32p),
                                    _ptr(n_grad, _i32p), _ptr(flags, _u8p))
        self._check(rc, "arima_fit_batch")
        return dict(coef=coef[:, :k], ll=ll, status=status, n_eval=n_eval, n_grad=n_grad, flags=flags)

    # The *_device methods below wrap asynchronous ABI calls. With blocking=True (the default) they wait for the
    # call's device work before returning, so results can be read through any stream (torch's included); pass
    # blocking=False to keep the ABI's asynchrony and call synchronize() (or stats()) later.
    def fit_batch_device(self, d_series, n_series, T, ld, p, d, q, include_intercept, d_coef, d_ll, d_status,
                         d_n_eval=None, d_n_grad=None, d_flags=None, d_user_init=None, method=METHOD_CSS_CGD,
                         stream=None, blocking=True):
        """Device-pointer entry (ints = raw HBM addresses, e.g. torch tensor .data_ptr())."""
        rc = self.L.arima_fit_batch_device(self.h, d_series, n_series, T, ld, p, d, q, int(bool(include_intercept)),
                                           method, d_user_init, d_coef, d_ll, d_status, d_n_eval, d_n_grad, d_flags,
                                           stream)
        self._check(rc, "arima_fit_batch_device")
        if blocking:
            self.synchronize()

    def sample_device(self, d_series, n_series, T, ld, p, d, q, include_intercept, base_coef, jitter, seed,
                      first_series=0, stream=None, blocking=True):
        base = np.ascontiguousarray(base_coef, dtype=np.float64)
        rc = self.L.arima_sample_batch_device(self.h, d_series, n_series, T, ld, p, d, q, int(bool(include_intercept)),
                                              _ptr(base), float(jitter), int(seed), int(first_series), stream)
        self._check(rc, "arima_sample_batch_device")
        if blocking:
            self.synchronize()

    # ---- building blocks ---------------------------------------------------------------------------------
    def difference(self, series, d):
        series = np.ascontiguousarray(np.atleast_2d(series), dtype=np.float64)
        out = np.empty_like(series)
        self._check(self.L.arima_difference_batch(self.h, _ptr(series), series.shape[0], series.shape[1], d,
                                                  _ptr(out)), "arima_difference_batch")
        return out

    def inverse_difference(self, series, d):
        series = np.ascontiguousarray(np.atleast_2d(series), dtype=np.float64)
        out = np.empty_like(series)
        self._check(self.L.arima_inverse_difference_batch(self.h, _ptr(series), series.shape[0], series.shape[1],
                                                          d, _ptr(out)), "arima_inverse_difference_batch")
        return out

    def css_loglik(self, series, p, d, q, include_intercept, coef):
        series = np.ascontiguousarray(np.atleast_2d(series), dtype=np.float64)
        N, T = series.shape
        k = p + q + (1 if include_intercept else 0)
        coef = np.ascontiguousarray(np.broadcast_to(np.asarray(coef, dtype=np.float64), (N, k)))
        ll = np.empty(N)
        self._check(self.L.arima_css_loglik_batch(self.h, _ptr(series), N, T, p, d, q, int(bool(include_intercept)),
                                                  _ptr(coef), _ptr(ll)), "arima_css_loglik_batch")
        return ll

    def css_gradient(self, diffed, p, q, include_intercept, coef):
        diffed = np.ascontiguousarray(np.atleast_2d(diffed), dtype=np.float64)
        N, n = diffed.shape
        k = p + q + (1 if include_intercept else 0)
        coef = np.ascontiguousarray(np.broadcast_to(np.asarray(coef, dtype=np.float64), (N, k)))
        g = np.empty((N, k))
        self._check(self.L.arima_css_gradient_batch(self.h, _ptr(diffed), N, n, p, q, int(bool(include_intercept)),
                                                    _ptr(coef), _ptr(g)), "arima_css_gradient_batch")
        return g

    def hannan_rissanen(self, diffed, p, q, include_intercept):
        diffed = np.ascontiguousarray(np.atleast_2d(diffed), dtype=np.float64)
        N, n = diffed.shape
        k = p + q + (1 if include_intercept else 0)
        out = np.empty((N, max(k, 1)))
        st = np.empty(N, dtype=np.int32)
        self._check(self.L.arima_hannan_rissanen_batch(self.h, _ptr(diffed), N, n, p, q,
                                                       int(bool(include_intercept)), _ptr(out), _ptr(st, _i32p)),
                    "arima_hannan_rissanen_batch")
        return out[:, :k], st

    def forecast(self, series, p, d, q, include_intercept, coef, n_future):
        series = np.ascontiguousarray(np.atleast_2d(series), dtype=np.float64)
        N, T = series.shape
        k = p + q + (1 if include_intercept else 0)
        coef = np.ascontiguousarray(np.broadcast_to(np.asarray(coef, dtype=np.float64), (N, k)))
        out = np.empty((N, T + n_future))
        self._check(self.L.arima_forecast_batch(self.h, _ptr(series), N, T, p, d, q, int(bool(include_intercept)),
                                                _ptr(coef), n_future, _ptr(out)), "arima_forecast_batch")
        return out

    def forecast_device(self, d_series, n_series, T, ld, p, d, q, include_intercept, d_coef, n_future, d_out, ld_out,
                        stream=None, blocking=True):
        """Device-pointer forecast (ints = raw HBM addresses)."""
        self._check(self.L.arima_forecast_batch_device(self.h, d_series, n_series, T, ld, p, d, q,
                                                       int(bool(include_intercept)), d_coef, n_future, d_out, ld_out,
                                                       stream), "arima_forecast_batch_device")
        if blocking:
            self.synchronize()

    def order_search_device(self, d_series, n_series, T, ld, max_p, max_d, max_q, intercept_mode, d_order, d_coef,
                            d_aic, method=METHOD_CSS_CGD, stream=None, blocking=True):
        """Device-pointer order search (ints = raw HBM addresses)."""
        self._check(self.L.arima_order_search_batch_device(self.h, d_series, n_series, T, ld, max_p, max_d, max_q,
                                                           intercept_mode, method, d_order, d_coef, d_aic, stream),
                    "arima_order_search_batch_device")
        if blocking:
            self.synchronize()

    def order_search(self, series, max_p=5, max_d=2, max_q=5, intercept_mode=2, method=METHOD_CSS_CGD):
        """Min-approxAIC model over the (d, p, q, intercept) grid per series (see include/sparkts_arima.h).
        Returns order (N x 4: p, d, q, intercept; -1 when nothing qualified), coef (N x 11), aic (N)."""
        series = np.ascontiguousarray(np.atleast_2d(series), dtype=np.float64)
        N, T = series.shape
        order = np.empty((N, 4), dtype=np.int32)
        coef = np.empty((N, 11))
        aic = np.empty(N)
        self._check(self.L.arima_order_search_batch(self.h, _ptr(series), N, T, max_p, max_d, max_q, intercept_mode,
                                                    method, _ptr(order, _i32p), _ptr(coef), _ptr(aic)),
                    "arima_order_search_batch")
        return order, coef, aic

    def autofit(self, series, max_p=5, max_d=2, max_q=5):
        """ARIMA.autoFit per series (see include/sparkts_arima.h). Returns dict(order N x 4 (p, d, q, intercept),
        coef N x 11, aic N, status N, n_fits N)."""
        series = np.ascontiguousarray(np.atleast_2d(series), dtype=np.float64)
        N, T = series.shape
        out = dict(order=np.empty((N, 4), dtype=np.int32), coef=np.empty((N, 11)), aic=np.empty(N),
                   status=np.empty(N, dtype=np.int32), n_fits=np.empty(N, dtype=np.int32))
        self._check(self.L.arima_autofit_batch(self.h, _ptr(series), N, T, max_p, max_d, max_q,
                                               _ptr(out["order"], _i32p), _ptr(out["coef"]), _ptr(out["aic"]),
                                               _ptr(out["status"], _i32p), _ptr(out["n_fits"], _i32p)),
                    "arima_autofit_batch")
        return out

    def autofit_device(self, d_series, n_series, T, ld, max_p, max_d, max_q, d_order, d_coef, d_aic, d_status,
                       d_n_fits=None, stream=None, blocking=True):
        """Device-pointer autoFit (ints = raw HBM addresses)."""
        self._check(self.L.arima_autofit_batch_device(self.h, d_series, n_series, T, ld, max_p, max_d, max_q, d_order,
                                                      d_coef, d_aic, d_status, d_n_fits, stream),
                    "arima_autofit_batch_device")
        if blocking:
            self.synchronize()

    def kpss(self, series):
        """TimeSeriesStatisticalTests.kpsstest(ts, "c") per series: (stat N, status N)."""
        series = np.ascontiguousarray(np.atleast_2d(series), dtype=np.float64)
        N, T = series.shape
        stat = np.empty(N)
        st = np.empty(N, dtype=np.int32)
        self._check(self.L.arima_kpss_batch(self.h, _ptr(series), N, T, _ptr(stat), _ptr(st, _i32p)),
                    "arima_kpss_batch")
        return stat, st

    def model_flags(self, coef, p, q, include_intercept):
        k = p + q + (1 if include_intercept else 0)
        coef = np.ascontiguousarray(np.asarray(coef, dtype=np.float64).reshape(-1, max(k, 1))[:, :k])
        N = coef.shape[0]
        out = np.empty(N, dtype=np.uint8)
        self._check(self.L.arima_model_flags_batch(self.h, _ptr(coef), N, p, q, int(bool(include_intercept)),
                                                   _ptr(out, _u8p)), "arima_model_flags_batch")
        return out
