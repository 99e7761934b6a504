"""The JNI shim (integration/jvm/native/sparkts_arima_jni.c) built against tests/jni_harness/'s jni.h subset and a fake
JNIEnv (no JDK in this image), then driven through ctypes as the Scala facade (ArimaMI355X.scala) would drive it:
direct NIO buffers become raw pointers. CPU tests: the shim compiles with -Werror, exports every JNI method the facade
declares `@native`, and forwards the error paths. GPU tests: fitBatch / autoFit through the shim are bit-identical to
the same ABI calls made directly (Engine), which the parity suites pin to the oracle."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tests", "jni_harness")
SO = os.path.join(HARNESS, "_build", "libjni_harness.so")
SCALA = os.path.join(ROOT, "integration", "jvm", "src", "main", "scala", "com", "cloudera", "sparkts", "models",
                     "ArimaMI355X.scala")
PREFIX = "Java_com_cloudera_sparkts_models_ArimaMI355XNative_00024_"

_vp, _i64, _i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32


def _harness():
    if not os.path.exists(SO):
        lib = os.path.join(ROOT, "spark-timeseries_amd", "libsparkts_arima.so")
        if not os.path.exists(lib):
            pytest.skip("engine library not built")
        subprocess.run(["make", "-s", "-C", HARNESS], check=True)
    L = ctypes.CDLL(SO)
    L.fake_jni_env.restype = _vp
    fn = lambda name: getattr(L, PREFIX + name)
    fn("create").restype = _i64
    fn("create").argtypes = [_vp, _vp, _i32]
    fn("destroy").argtypes = [_vp, _vp, _i64]
    fn("lastError").restype = ctypes.c_char_p
    fn("lastError").argtypes = [_vp, _vp, _i64]
    fn("setOption").argtypes = [_vp, _vp, _i64, ctypes.c_char_p, _i64]
    fn("fitBatch").argtypes = [_vp, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _i32, ctypes.c_uint8, _i32, _vp, _vp,
                               _vp, _vp, _vp, _vp, _vp]
    fn("autoFit").argtypes = [_vp, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp]
    return L, fn, L.fake_jni_env()


def _p(a):
    return None if a is None else a.ctypes.data


def test_shim_exports_every_native_method_of_the_facade():
    L, fn, env = _harness()
    with open(SCALA) as f:
        natives = set(re.findall(r"@native\s+def\s+(\w+)", f.read()))
    assert {"create", "destroy", "lastError", "setOption", "fitBatch", "forecastBatch", "orderSearch",
            "autoFit"} <= natives
    for name in natives:
        assert hasattr(L, PREFIX + name), f"JNI symbol for ArimaMI355XNative.{name} missing"


def test_shim_forwards_null_handle_errors():
    L, fn, env = _harness()
    assert fn("lastError")(env, None, 0) == b"null handle"
    assert fn("setOption")(env, None, 0, b"fit_pipeline", 1) == -1
    x = np.zeros((2, 8))
    out = np.empty(2)
    assert fn("fitBatch")(env, None, 0, _p(x), 2, 8, 1, 0, 1, 1, 0, None, _p(np.empty((2, 3))), _p(out), None, None,
                          None, None) == -1
    assert fn("autoFit")(env, None, 0, _p(x), 2, 8, 5, 2, 5, None, None, None, None, None) == -1


@pytest.mark.gpu
def test_shim_fit_and_autofit_match_direct_abi(engine):
    L, fn, env = _harness()
    h = fn("create")(env, None, 0)
    assert h != 0
    try:
        assert fn("setOption")(env, None, h, b"no_such_option", 1) != 0
        assert fn("lastError")(env, None, h)
        rng = np.random.default_rng(11)
        N, T = 300, 256
        s = np.ascontiguousarray(np.cumsum(rng.standard_normal((N, T)), axis=1))
        p, d, q = 2, 1, 2
        coef, ll = np.empty((N, 5)), np.empty(N)
        st, ne, ng = np.empty(N, np.int32), np.empty(N, np.int32), np.empty(N, np.int32)
        fl = np.empty(N, np.uint8)
        rc = fn("fitBatch")(env, None, h, _p(s), N, T, p, d, q, 1, 0, None, _p(coef), _p(ll), _p(st), _p(ne), _p(ng),
                            _p(fl))
        assert rc == 0, fn("lastError")(env, None, h)
        exp = engine.fit_batch(s, p, d, q)
        assert np.array_equal(coef.view(np.int64), exp["coef"].view(np.int64))
        assert np.array_equal(ll.view(np.int64), exp["ll"].view(np.int64))
        for a, k in ((st, "status"), (ne, "n_eval"), (ng, "n_grad"), (fl, "flags")):
            assert np.array_equal(a, exp[k]), k

        n2 = 64
        order, c11 = np.empty((n2, 4), np.int32), np.empty((n2, 11))
        aic, ast, nf = np.empty(n2), np.empty(n2, np.int32), np.empty(n2, np.int32)
        rc = fn("autoFit")(env, None, h, _p(s[:n2]), n2, T, 5, 2, 5, _p(order), _p(c11), _p(aic), _p(ast), _p(nf))
        assert rc == 0, fn("lastError")(env, None, h)
        r = engine.autofit(s[:n2], 5, 2, 5)
        assert np.array_equal(order, r["order"]) and np.array_equal(ast, r["status"])
        assert np.array_equal(nf, r["n_fits"])
        assert np.array_equal(aic.view(np.int64), np.asarray(r["aic"]).view(np.int64))
        assert np.array_equal(c11.view(np.int64), np.asarray(r["coef"]).view(np.int64))
    finally:
        assert fn("destroy")(env, None, h) == 0
