"""Powell's RESCUE in the css-bobyqa restatement (oracle/bobyqa_oracle.c bq_rescue; bobyqb label 190 of the
BOBYQA that commons BOBYQAOptimizer translates, configured by ARIMA.fitWithCSSBOBYQA, ARIMA.scala:130-160, and reached
through autoFit's fitTryBothStrategies retries, :315-319).

No JVM here, so RESCUE's bits are pinned to the restatement only; what is checked on the CPU:
  - every series of the bobyqa_rescue_* fixtures enters RESCUE, and the oracle reproduces the fixtures bit for bit;
  - each RESCUE leaves a consistent interpolation system: the Lagrange functions it rebuilds (BMAT, ZMAT) interpolate
    the new point set to rounding and the rebuilt model reproduces the values, both measured against the set's
    spread (oracle/bobyqa_rescue_check.c);
  - the autoFit rows that used to stop in RESCUE (status 13) now complete, matching autofit_rescue_c2_T1024.
The GPU side (tests/test_gpu_bobyqa.py) compares k_bobyqa_fit with these fixtures."""
import ctypes
import os

import numpy as np
import pytest

import oracle as O
from conftest import all_cases, load_case

HERE = os.path.dirname(os.path.abspath(__file__))
CHK = os.path.join(HERE, "..", "oracle", "_build", "libbobyqa_rescue_check.so")
RESCUE_CASES = all_cases("bobyqa_rescue_")


def _check_lib():
    if not os.path.exists(CHK):
        O.build()
    L = ctypes.CDLL(CHK)
    L.orc_fit.restype = ctypes.c_int
    L.orc_fit.argtypes = [O._dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                          O._dp, ctypes.c_int, O._dp, O._dp, O._ip]
    L.orc_rescue_check_lagrange.restype = ctypes.c_double
    L.orc_rescue_check_model.restype = ctypes.c_double
    L.orc_rescue_check_calls.restype = ctypes.c_int
    return L


def test_rescue_fixtures_exist():
    assert {"bobyqa_rescue_ridge_101c", "bobyqa_rescue_c2like_001c"} <= set(RESCUE_CASES)
    assert any(n.startswith("bobyqa_rescue_af_") for n in RESCUE_CASES)


@pytest.mark.parametrize("name", RESCUE_CASES)
def test_oracle_reproduces_rescue_fixture_and_enters_rescue(name):
    meta, arr = load_case(name)
    p, d, q, I = meta["p"], meta["d"], meta["q"], meta["I"]
    L = O.lib()
    L.orc_bobyqa_last_rescues.restype = ctypes.c_int
    for i, s in enumerate(arr["series"]):
        r = O.fit(s, p, d, q, I, method=1)
        assert L.orc_bobyqa_last_rescues() >= 1, (name, i)
        assert r["status"] == arr["status"][i] and r["n_eval"] == arr["n_eval"][i], (name, i)
        assert np.array_equal(r["coef"].view(np.int64), arr["coef"][i].view(np.int64)), (name, i)
        assert np.array_equal(np.float64(r["ll"]).view(np.int64), arr["ll"][i].view(np.int64)), (name, i)


@pytest.mark.parametrize("name", RESCUE_CASES)
def test_rescue_rebuilds_a_consistent_interpolation_system(name):
    meta, arr = load_case(name)
    p, d, q, I = meta["p"], meta["d"], meta["q"], meta["I"]
    L = _check_lib()
    k = p + q + I
    for i, s in enumerate(arr["series"]):
        s = np.ascontiguousarray(s)
        coef, ll, cnt = np.empty(k), ctypes.c_double(), (ctypes.c_int * 3)()
        L.orc_rescue_check_reset()
        st = L.orc_fit(s.ctypes.data_as(O._dp), len(s), p, d, q, I, 1, None, O.DEFAULT_SMEAR,
                       coef.ctypes.data_as(O._dp), ctypes.byref(ll), cnt)
        assert st == arr["status"][i] and np.array_equal(coef, arr["coef"][i]), (name, i)   # same fit, checked
        assert L.orc_rescue_check_calls() >= 1
        # errors over kappa = (r_max / r_min)^4, the set's spread (bobyqa_rescue_check.c): Lagrange conditions
        # L_j(x_i) = delta_ij hold to rounding (<= 5e-14 measured); the model's values to 1e-5 (the points RESCUE
        # reinstates keep the pre-RESCUE model's rounding; the evaluated ones are exact)
        assert L.orc_rescue_check_lagrange() < 1e-12, (name, i, L.orc_rescue_check_lagrange())
        assert L.orc_rescue_check_model() < 1e-5, (name, i, L.orc_rescue_check_model())


def test_rescued_autofit_rows_complete():
    z = np.load(os.path.join(HERE, "golden", "autofit_rescue_c2_T1024.npz"), allow_pickle=False)
    assert (z["status"] == 0).all()
    for i in range(0, len(z["series"]), 4):                      # a sample: each walk runs ~9 fits on the CPU
        r = O.autofit(z["series"][i], 5, 2, 5)
        assert r["status"] == z["status"][i] and tuple(r["order"]) == tuple(z["order"][i])
        assert r["n_fits"] == z["n_fits"][i]
        assert np.array_equal(np.asarray(r["coef"]).view(np.int64), z["coef"][i].view(np.int64))
        assert np.float64(r["aic"]).view(np.int64) == z["aic"][i].view(np.int64)
