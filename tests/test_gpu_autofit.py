"""ARIMA.autoFit over a batch on the GPU (arima_autofit_batch*, ARIMA.scala:280-375) against the CPU restatement
(oracle.autofit + orc_kpss): the KPSS choice of d, the stepwise walk's selection, coefficients, approxAIC, status and
the number of candidate fits, bit for bit."""
import numpy as np
import pytest

import oracle as O
from conftest import all_cases, load_case

pytestmark = pytest.mark.gpu


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype.kind == "f":
        return np.array_equal(a.view(np.int64), b.view(np.int64)) or np.array_equal(a, b, equal_nan=True) and \
            np.array_equal(np.signbit(a), np.signbit(b))
    return np.array_equal(a, b)


def check_autofit(res, exp, tag):
    for k in ("status", "order", "n_fits"):
        bad = np.nonzero((np.asarray(res[k]) != np.asarray(exp[k])).reshape(len(exp["status"]), -1).any(axis=1))[0]
        assert bad.size == 0, f"{tag}: {k} differs at rows {bad[:8].tolist()}: {np.asarray(res[k])[bad[:4]].tolist()} " \
                              f"vs {np.asarray(exp[k])[bad[:4]].tolist()}"
    assert _same(res["coef"], exp["coef"]), f"{tag}: coefficients differ"
    assert _same(res["aic"], exp["aic"]), f"{tag}: approxAIC differs"


@pytest.mark.parametrize("name", all_cases("autofit_"))
def test_autofit_golden(engine, name):
    meta, arr = load_case(name)
    r = engine.autofit(arr["series"], meta["max_p"], meta["max_d"], meta["max_q"])
    check_autofit(r, arr, name)


def test_kpss_matches_oracle(engine):
    rng = np.random.default_rng(7)
    for T in (2, 3, 20, 250, 1024, 4096):
        s = np.cumsum(rng.standard_normal((32, T)), axis=1) * rng.uniform(0.1, 10, (32, 1))
        s[:8] = rng.standard_normal((8, T))
        stat, st = engine.kpss(s)
        exp = [O.kpss(row, "c") for row in s]
        assert np.array_equal(st, [e[0] for e in exp]), T
        assert _same(stat, np.array([e[1] for e in exp])), T
    stat, st = engine.kpss(np.zeros((3, 1)))
    assert np.all(st == 5) and np.all(np.isnan(stat))


def test_autofit_c2_batch_matches_oracle(engine):
    # the C2 generator (BASELINE configs[1]'s series), a batch large enough that every candidate order's list is a
    # multi-wave fit; oracle on a subsample
    import torch
    N, T = 4096, 1024
    s = torch.empty((N, T), dtype=torch.float64, device="cuda")
    engine.sample_device(s.data_ptr(), N, T, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 1234, 0)
    engine.synchronize()
    host = s.cpu().numpy()
    r = engine.autofit(host, 5, 2, 5)
    idx = np.arange(0, N, 37)
    exp = [O.autofit(host[i], 5, 2, 5) for i in idx]
    sub = {k: np.asarray(v)[idx] for k, v in r.items()}
    check_autofit(sub, {k: np.array([e[k] for e in exp]) for k in ("status", "order", "n_fits", "coef", "aic")},
                  "c2_4096")
    assert (r["order"][:, 1] == 1).mean() > 0.5                       # KPSS mostly picks d = 1 for the I(1) generator


def test_autofit_device_entry_point_and_bounds(engine):
    import torch
    meta, arr = load_case("autofit_mixed_T256")
    N, T = arr["series"].shape
    d = torch.from_numpy(arr["series"]).cuda()
    out = dict(order=torch.empty((N, 4), dtype=torch.int32, device="cuda"),
               coef=torch.empty((N, 11), dtype=torch.float64, device="cuda"),
               aic=torch.empty(N, dtype=torch.float64, device="cuda"), status=torch.empty(N, dtype=torch.int32, device="cuda"),
               n_fits=torch.empty(N, dtype=torch.int32, device="cuda"))
    engine.autofit_device(d.data_ptr(), N, T, T, 5, 2, 5, out["order"].data_ptr(), out["coef"].data_ptr(),
                          out["aic"].data_ptr(), out["status"].data_ptr(), out["n_fits"].data_ptr())
    check_autofit({k: v.cpu().numpy() for k, v in out.items()}, arr, "device entry point")
    with pytest.raises(Exception):
        engine.autofit(arr["series"], 9, 2, 5)     # max_p <= 8: its css-bobyqa retries have <= 11 parameters


def test_autofit_long_series_matches_oracle(engine):
    # T = 3000: KPSS lag 12 (the register ring's longer reach), longer css-cgd fits and css-bobyqa retries on rows
    # past the express path's parallel-in-time length; mixed I(0) / I(1) / I(2) series
    rng = np.random.default_rng(2026)
    N, T = 12, 3000
    e = rng.standard_normal((N, T))
    s = e.copy()
    for t in range(1, T):
        s[:, t] = 0.6 * s[:, t - 1] + e[:, t] + 0.3 * e[:, t - 1]
    s[4:8] = np.cumsum(s[4:8], axis=1)
    s[8:] = np.cumsum(np.cumsum(s[8:], axis=1), axis=1) * 0.01
    r = engine.autofit(s, 5, 2, 5)
    exp = [O.autofit(row, 5, 2, 5) for row in s]
    check_autofit(r, {k: np.array([x[k] for x in exp]) for k in ("status", "order", "n_fits", "coef", "aic")},
                  "long_T3000")
