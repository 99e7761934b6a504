"""The runtime-order path (spark-timeseries_amd/csrc/arima_generic.hip): orders above the compiled ones (p or q > 5, up
to 20), through the same C ABI as every other fit, against the CPU restatement bit for bit (VERDICT r5 missing 1).

The reference's fitModel takes any p, q (ARIMA.scala:79-86) and autoFit any maxP and series length (ARIMA.scala:280,
TimeSeriesStatisticalTests.scala:390); the library now returns ARIMA_E_UNSUPPORTED only for orders above 20, css-bobyqa
above 11 parameters and autoFit above maxP = 8 (its css-bobyqa retries), each stated in include/sparkts_arima.h."""
import numpy as np
import pytest

import oracle as O
import sparkts_amd._lib as L
from test_gpu_parity import _same, check_fit

pytestmark = pytest.mark.gpu


def _series(seed, N, T, p, d, q, I, base):
    """Host-generated ARIMA(p, d, q) series (ARIMAModel.sample semantics through the oracle's addTimeDependentEffects)."""
    rng = np.random.default_rng(seed)
    return np.stack([O.add_time_dependent_effects(rng.standard_normal(T), p, d, q, I, base) for _ in range(N)])


def _expect(s, p, d, q, I, method=0, smear=1):
    st, coef, ll, cnt = O.fit_batch(s, p, d, q, I, method=method, smear=smear)
    return dict(status=st, coef=coef, ll=ll, n_eval=cnt[:, 0], n_grad=cnt[:, 1],
                flags=np.array([O.model_flags(coef[i], p, q, I) if st[i] == 0 else 0 for i in range(len(st))]))


GENERIC_FITS = [
    # (p, d, q, I, base coefficients)
    (7, 1, 2, 1, [0.2, 0.3, -0.1, 0.1, 0.05, -0.05, 0.04, 0.02, 0.3, 0.1]),
    (0, 1, 8, 0, [0.3, 0.1, -0.1, 0.05, 0.05, -0.02, 0.02, 0.01]),
    (9, 0, 0, 1, [1.0, 0.3, -0.1, 0.1, 0.05, -0.05, 0.04, 0.02, -0.02, 0.01]),
    (6, 0, 6, 1, [0.5, 0.2, -0.1, 0.05, 0.05, -0.02, 0.02, 0.2, 0.1, -0.05, 0.05, 0.02, 0.01]),
    (12, 2, 1, 0, [0.2, 0.1, -0.1, 0.05, 0.05, -0.02, 0.02, 0.01, 0.01, -0.01, 0.01, 0.01, 0.3]),
]


@pytest.mark.parametrize("case", GENERIC_FITS, ids=lambda c: f"{c[0]}{c[1]}{c[2]}{'c' if c[3] else ''}")
def test_generic_fit_matches_oracle(engine, case):
    p, d, q, I, base = case
    s = _series(100 + p * 7 + q, 48, 600, p, d, q, I, base)
    res = engine.fit_batch(s, p, d, q, bool(I))
    st = engine.stats()
    check_fit(res, _expect(s, p, d, q, I), f"ARIMA({p},{d},{q}){'+c' if I else ''}")
    assert st["series_done"] == 48 and st["n_eval"] == int(res["n_eval"].sum())
    assert (res["status"] == 0).any()            # (6,0,6)+c: MaxEval is common, as in the reference


def test_generic_fit_device_entry_odd_rows_and_fuse(engine):
    # the device entry point with rows at odd 8-B offsets (ld = T + 1), fused differencing on and off, and a user init
    import torch
    p, d, q, I, base = GENERIC_FITS[0]
    N, T = 96, 500
    s = _series(7, N, T, p, d, q, I, base)
    ld = T + 1
    buf = torch.full((N, ld), float("nan"), dtype=torch.float64, device="cuda")
    buf[:, :T] = torch.from_numpy(s).cuda()
    k = p + q + I
    out = {}
    try:
        for fuse in (1, 0):
            engine.set_option("fuse_diff", fuse)
            r = [torch.empty((N, k), dtype=torch.float64, device="cuda"), torch.empty(N, dtype=torch.float64, device="cuda")] + \
                [torch.empty(N, dtype=torch.int32, device="cuda") for _ in range(3)] + \
                [torch.empty(N, dtype=torch.uint8, device="cuda")]
            engine.fit_batch_device(buf.data_ptr(), N, T, ld, p, d, q, I, *[t.data_ptr() for t in r])
            out[fuse] = [t.cpu().numpy() for t in r]
    finally:
        engine.set_option("fuse_diff", 1)
    for x, y in zip(out[1], out[0]):
        assert _same(x, y)
    exp = _expect(s, p, d, q, I)
    check_fit(dict(coef=out[1][0], ll=out[1][1], status=out[1][2], n_eval=out[1][3], n_grad=out[1][4],
                   flags=out[1][5]), exp, "device odd ld")
    ui = np.full(k, 0.1)
    r = engine.fit_batch(s[:16], p, d, q, True, user_init=ui)
    e = O.fit_batch(s[:16], p, d, q, I, user_init=np.broadcast_to(ui, (16, k)))
    assert np.array_equal(r["status"], e[0]) and np.array_equal(r["n_eval"], e[3][:, 0])
    assert _same(r["coef"][e[0] == 0], e[1][e[0] == 0])


@pytest.mark.parametrize("pq", [(7, 2), (0, 8), (6, 6), (3, 9)])
@pytest.mark.parametrize("smear", [0, 1])
def test_generic_gradient_and_loglik(engine, pq, smear):
    p, q = pq
    rng = np.random.default_rng(p * 31 + q)
    y = rng.standard_normal((40, 333))
    for I in (0, 1):
        k = p + q + I
        coef = rng.uniform(-0.3, 0.3, (40, k))
        engine.set_option("smear", smear)
        try:
            g = engine.css_gradient(y, p, q, I, coef)
        finally:
            engine.set_option("smear", L.DEFAULT_SMEAR)
        exp = np.stack([O.gradient_css_arma(y[i], p, q, I, coef[i], smear) for i in range(40)])
        assert _same(g, exp), (pq, smear, I)
        ll = engine.css_loglik(y, p, 0, q, I, coef)
        assert _same(ll, np.array([O.loglik_css(y[i], p, 0, q, I, coef[i]) for i in range(40)]))


@pytest.mark.parametrize("pqi", [(7, 2, 1), (9, 0, 1), (0, 8, 0), (6, 6, 1), (20, 0, 1), (2, 20, 0)])
def test_generic_hannan_rissanen_and_flags(engine, pqi):
    p, q, I = pqi
    rng = np.random.default_rng(p + 100 * q)
    y = np.stack([O.add_time_dependent_effects(rng.standard_normal(700), 1, 0, 1, 1, [0.5, 0.4, 0.3])
                  for _ in range(32)])
    init, st = engine.hannan_rissanen(y, p, q, I)
    for i in range(32):
        est, eini = O.hannan_rissanen(y[i], p, q, I)
        assert st[i] == est
        if est == 0:
            assert _same(init[i], eini), (i, pqi)
    coef = rng.uniform(-0.35, 0.35, (200, p + q + I))
    f = engine.model_flags(coef, p, q, I)
    assert np.array_equal(f, np.array([O.model_flags(c, p, q, I) for c in coef])), pqi


@pytest.mark.parametrize("pdqi", [(7, 1, 2, 1), (0, 2, 8, 0), (9, 0, 0, 1), (6, 12, 6, 1), (2, 10, 1, 0), (1, 0, 14, 1)])
@pytest.mark.parametrize("n_future", [0, 13])
def test_generic_forecast(engine, pdqi, n_future):
    # the runtime-order forecast (k_gen_forecast) for orders above 5 and d above 8 (k_forecast's compiled range)
    p, d, q, I = pdqi
    rng = np.random.default_rng(500 + p + d + q)
    N, T = 70, 160
    s = rng.standard_normal((N, T)).cumsum(axis=1) + 3.0
    coef = rng.uniform(-0.3, 0.3, (N, p + q + I))
    out = engine.forecast(s, p, d, q, I, coef, n_future)
    exp = np.stack([O.forecast(s[i], p, d, q, I, coef[i], n_future) for i in range(N)])
    assert _same(out, exp), (pdqi, n_future)


def test_generic_css_bobyqa(engine):
    # css-bobyqa (ARIMA.scala:130-160) at ARIMA(7,1,2)+c: 10 parameters, within the dimensions css-bobyqa compiles
    p, d, q, I, base = GENERIC_FITS[0]
    s = _series(77, 24, 400, p, d, q, I, base)
    res = engine.fit_batch(s, p, d, q, True, method="css-bobyqa")
    check_fit(res, _expect(s, p, d, q, I, method=1), "css-bobyqa (7,1,2)+c")
    with pytest.raises(L.EngineError):                           # 13 parameters: beyond the compiled dimensions
        engine.fit_batch(s, 6, 1, 6, True, method="css-bobyqa")


def test_generic_bounds(engine):
    s = _series(3, 4, 200, 1, 0, 1, 1, [0.5, 0.3, 0.2])
    with pytest.raises(L.EngineError):
        engine.fit_batch(s, 21, 0, 0, True)                       # above kGenMaxOrder
    r = engine.fit_batch(s[:, :5], 7, 1, 2, True)                 # too short for the lag matrices: statuses, no error
    assert np.all(r["status"] != 0)
    e = O.fit_batch(s[:, :5], 7, 1, 2, 1)
    assert np.array_equal(r["status"], e[0])


def test_autofit_max_p_8_long_series(engine):
    # autoFit with maxP = 8 on T = 25 000: KPSS lag 36 (past the 32-entry register ring: one pass
    # per lag), walks that reach p = 6..8 (the runtime-order fits), bit for bit against oracle.autofit
    rng = np.random.default_rng(2027)
    N, T = 6, 25000
    designs = [[0.1, 0.1, 0.1, 0.1, 0.15, 0.15, 0.15, 0.1],             # near-unit-root AR(8): KPSS d = 1, p -> 8
               [0.5, -0.4, 0.3, -0.3, 0.25, -0.2, 0.2, -0.15]]           # alternating AR(8): d = 0, p -> 5
    rows = []
    for i in range(N):
        ar = designs[i % 2]
        rows.append(O.add_time_dependent_effects(rng.standard_normal(T), len(ar), 0, 0, 1, [0.2] + ar))
    s = np.stack(rows)
    r = engine.autofit(s, 8, 1, 2)
    exp = [O.autofit(row, 8, 1, 2) for row in s]
    for k in ("status", "order", "n_fits"):
        assert np.array_equal(np.asarray(r[k]), np.array([x[k] for x in exp])), (k, r[k], [x[k] for x in exp])
    assert _same(r["coef"], np.array([x["coef"] for x in exp]))
    assert _same(r["aic"], np.array([x["aic"] for x in exp]))
    assert (r["order"][:, 0] > 5).any(), r["order"]              # the walk did go past the compiled orders
    with pytest.raises(L.EngineError):
        engine.autofit(s[:1, :500], 9, 1, 2)                       # css-bobyqa retries above 11 parameters


def test_autofit_slices_are_transparent(engine):
    # option autofit_slice: the batch in consecutive slices (the bound on autoFit's workspaces) -- the same
    # selections bit for bit
    import torch
    N, T = 1500, 256
    d = torch.empty((N, T), dtype=torch.float64, device="cuda")
    engine.sample_device(d.data_ptr(), N, T, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 99, 0)
    host = d.cpu().numpy()
    whole = engine.autofit(host, 5, 2, 5)
    try:
        engine.set_option("autofit_slice", 600)   # three slices
        sliced = engine.autofit(host, 5, 2, 5)
    finally:
        engine.set_option("autofit_slice", 0)
    for k in whole:
        assert _same(whole[k], sliced[k]), k
