"""GPU parity: the HIP path (through the C ABI) against the CPU restatement, bit for bit.

Fixtures (tests/golden/*.npz) hold inputs and the oracle's outputs; larger synthetic batches are generated on the
device, copied back and checked against the oracle run here; full-size runs are checked through
size-independent properties (determinism, permutation invariance, status accounting).
Bar: integer outputs exact; floating outputs bit-identical (the kernel performs the reference's fp64 operations
in the reference's order). The north_star tolerances (coef 1e-4 abs, CSS LL 1e-6 rel) are
asserted as well so a failure report says which bar broke.
"""
import numpy as np
import pytest

import oracle as O
import sparkts_amd._lib as L
from conftest import all_cases, load_case

pytestmark = pytest.mark.gpu

COEF_ATOL = 1e-4      # north_star: fitted coefficients within 1e-4 absolute
LL_RTOL = 1e-6        # north_star: CSS log-likelihood within 1e-6 relative


def _same(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.array_equal(a.view(np.int64) if a.size else a, b.view(np.int64) if b.size else b) or \
        np.array_equal(a, b, equal_nan=True)


def check_fit(res, exp, ctx):
    st = res["status"]
    assert np.array_equal(st, exp["status"]), f"{ctx}: status {st} vs {exp['status']}"
    ok = st == 0
    assert np.array_equal(res["n_eval"], exp["n_eval"]), f"{ctx}: n_eval {res['n_eval']} vs {exp['n_eval']}"
    assert np.array_equal(res["n_grad"], exp["n_grad"]), f"{ctx}: n_grad"
    if ok.any():
        c, ce = res["coef"][ok], exp["coef"][ok]
        # a normal return can sit at a NaN point (css-bobyqa on NaN models): the north_star tolerances below apply to
        # the finite values; every value, NaN positions included, must still match exactly (_same, after them)
        fin = np.isfinite(ce)
        assert np.all(np.abs(c - ce)[fin] <= COEF_ATOL), f"{ctx}: coef tolerance"
        ll, lle = res["ll"][ok], exp["ll"][ok]
        lf = np.isfinite(lle)
        assert np.all(np.abs(ll - lle)[lf] <= LL_RTOL * np.abs(lle)[lf]), f"{ctx}: LL tolerance"
        assert _same(c, ce), f"{ctx}: coefficients not bit-identical: max diff {np.nanmax(np.abs(c - ce))}"
        assert _same(ll, lle), f"{ctx}: LL not bit-identical"
        assert np.array_equal(res["flags"][ok], exp["flags"][ok]), f"{ctx}: flags"
    assert np.all(np.isnan(res["coef"][~ok])), f"{ctx}: failed fits must report NaN coefficients"


@pytest.mark.parametrize("name", all_cases())
def test_golden_fixture(engine, name):
    meta, arr = load_case(name)
    engine.set_option("smear", meta["smear"])
    try:
        res = engine.fit_batch(arr["series"], meta["p"], meta["d"], meta["q"], meta["I"], meta["method"],
                               arr.get("user_init"))
    finally:
        engine.set_option("smear", L.DEFAULT_SMEAR)
    check_fit(res, arr, name)


def test_sqrt_div_log_are_bit_exact(engine):
    # the LL of random coefficient vectors exercises log / div; HR exercises sqrt
    rng = np.random.default_rng(7)
    s = rng.standard_normal((256, 300)).cumsum(axis=1)
    coef = np.column_stack([rng.normal(0, 1, 256), rng.uniform(-0.9, 0.9, (256, 2)), rng.uniform(-0.9, 0.9, 256)])
    ll = engine.css_loglik(s, 2, 1, 1, True, coef)
    exp = np.array([O.loglik_css(s[i], 2, 1, 1, 1, coef[i]) for i in range(256)])
    assert _same(ll, exp)


def test_difference_bit_exact(engine):
    rng = np.random.default_rng(3)
    s = rng.standard_normal((37, 123)) * 1e3
    for d in range(0, 6):
        out = engine.difference(s, d)
        exp = np.stack([O.differences_of_order_d(r, d) for r in s])
        assert np.array_equal(out, exp), d
        inv = engine.inverse_difference(out, d)
        expi = np.stack([O.inverse_differences_of_order_d(r, d) for r in exp])
        assert np.array_equal(inv, expi), d


@pytest.mark.parametrize("pqi", [(1, 1, 1), (2, 2, 1), (0, 1, 1), (3, 2, 0), (5, 5, 1), (2, 4, 1)])
@pytest.mark.parametrize("smear", [0, 1])
def test_gradient_bit_exact(engine, pqi, smear):
    p, q, I = pqi
    rng = np.random.default_rng(p * 100 + q * 10 + I)
    y = rng.standard_normal((64, 257))
    k = p + q + I
    coef = rng.uniform(-0.5, 0.5, (64, k))
    engine.set_option("smear", smear)
    try:
        g = engine.css_gradient(y, p, q, I, coef)
    finally:
        engine.set_option("smear", L.DEFAULT_SMEAR)
    exp = np.stack([O.gradient_css_arma(y[i], p, q, I, coef[i], smear) for i in range(64)])
    assert _same(g, exp)


@pytest.mark.parametrize("pqi", [(1, 1, 1), (2, 2, 1), (0, 1, 1), (3, 2, 0), (5, 5, 1), (0, 0, 1), (4, 0, 1)])
def test_hannan_rissanen_bit_exact(engine, pqi):
    p, q, I = pqi
    rng = np.random.default_rng(11 + p + q)
    y = np.stack([O.add_time_dependent_effects(rng.standard_normal(400), 1, 0, 1, 1, [0.5, 0.4, 0.3])
                  for _ in range(64)])
    init, st = engine.hannan_rissanen(y, p, q, I)
    for i in range(64):
        est, eini = O.hannan_rissanen(y[i], p, q, I)
        assert st[i] == est
        if est == 0:
            assert _same(init[i], eini), (i, init[i], eini)


def test_model_flags_match_oracle(engine):
    rng = np.random.default_rng(5)
    for p, q in [(1, 0), (0, 1), (2, 2), (5, 5), (3, 1)]:
        coef = rng.uniform(-1.5, 1.5, (200, 1 + p + q))
        f = engine.model_flags(coef, p, q, True)
        exp = np.array([O.model_flags(c, p, q, 1) for c in coef])
        assert np.array_equal(f, exp), (p, q)


def _device_sample(engine, N, T, p, d, q, I, base, jitter, seed, first=0):
    import torch
    buf = torch.empty((N, T), dtype=torch.float64, device="cuda")
    engine.sample_device(buf.data_ptr(), N, T, T, p, d, q, I, base, jitter, seed, first)
    return buf


def test_c2_batch_vs_oracle(engine):
    # C2 workload (ARIMA(2,1,2)+c, T=1024) on 2048 device-generated series, every series checked vs the oracle
    N, T = 2048, 1024
    s = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 20261015).cpu().numpy()
    res = engine.fit_batch(s, 2, 1, 2, True)
    st, coef, ll, cnt = O.fit_batch(s, 2, 1, 2, 1)
    exp = dict(status=st, coef=coef, ll=ll, n_eval=cnt[:, 0], n_grad=cnt[:, 1],
               flags=np.array([O.model_flags(coef[i], 2, 2, 1) if st[i] == 0 else 0 for i in range(N)]))
    check_fit(res, exp, "c2_2048")


def test_c1_batch_vs_oracle(engine):
    N, T = 2048, 500
    s = _device_sample(engine, N, T, 1, 0, 1, 1, [3.5, 0.3, 0.7], 0.05, 20261015).cpu().numpy()
    res = engine.fit_batch(s, 1, 0, 1, True)
    st, coef, ll, cnt = O.fit_batch(s, 1, 0, 1, 1)
    exp = dict(status=st, coef=coef, ll=ll, n_eval=cnt[:, 0], n_grad=cnt[:, 1],
               flags=np.array([O.model_flags(coef[i], 1, 1, 1) if st[i] == 0 else 0 for i in range(N)]))
    check_fit(res, exp, "c1_2048")


def test_sampler_is_shard_invariant(engine):
    a = _device_sample(engine, 300, 64, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 99).cpu().numpy()
    b = _device_sample(engine, 100, 64, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 99, first=200).cpu().numpy()
    assert np.array_equal(a[200:], b)
    assert np.all(np.isfinite(a))


def test_full_size_properties(engine):
    """65536 series x 1024 (C2): determinism, permutation invariance, counters and statuses consistent."""
    import torch
    N, T = 65536, 1024
    dev = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 20261015)
    host = dev.cpu().numpy()
    r1 = engine.fit_batch(host, 2, 1, 2, True)
    stats = engine.stats()
    r2 = engine.fit_batch(host, 2, 1, 2, True)
    for k in r1:
        assert np.array_equal(r1[k], r2[k], equal_nan=True), k
    perm = np.random.default_rng(0).permutation(N)
    r3 = engine.fit_batch(host[perm], 2, 1, 2, True)
    for k in r1:
        assert np.array_equal(r1[k][perm], r3[k], equal_nan=True), k
    assert stats["n_eval"] == int(r1["n_eval"].sum()) and stats["n_grad"] == int(r1["n_grad"].sum())
    assert stats["series_done"] == N
    ok = r1["status"] == 0
    assert ok.mean() > 0.99
    assert np.all(np.isfinite(r1["ll"][ok]))
    # spot-check 256 random series against the oracle
    idx = np.random.default_rng(1).choice(N, 256, replace=False)
    st, coef, ll, cnt = O.fit_batch(host[idx], 2, 1, 2, 1)
    assert np.array_equal(st, r1["status"][idx])
    assert np.array_equal(coef[st == 0], r1["coef"][idx][st == 0])
    del dev
    torch.cuda.empty_cache()


def test_python_mirror_api(engine):
    from sparkts_amd.models import ARIMA
    meta, arr = load_case("kat_ds1_101")
    m = ARIMA.fit_model(1, 0, 1, arr["series"][0])
    assert np.array_equal(m.coefficients, arr["coef"][0])
    assert m.log_likelihood_css(arr["series"][0]) == arr["ll"][0]
    assert m.is_stationary() and m.is_invertible()
    assert m.approx_aic(arr["series"][0]) == -2 * arr["ll"][0] + 2 * 3
    with pytest.raises(ARIMA.UnsupportedOperationException):
        ARIMA.fit_model(1, 0, 1, arr["series"][0], method="css-newton")
    mb = ARIMA.fit_model(1, 0, 1, arr["series"][0], method="css-bobyqa")
    eb = O.fit(arr["series"][0], 1, 0, 1, method=1)
    assert np.array_equal(mb.coefficients, eb["coef"])
    with pytest.raises(ARIMA.TooManyEvaluationsException):
        ARIMA.fit_model(1, 0, 1, np.full(50, np.nan))
    # ARIMAModel.sample: the device sampler with this model's coefficients (jitter 0), deterministic per seed
    s1, s2 = m.sample(300, seed=5), m.sample(300, seed=5)
    assert s1.shape == (300,) and np.array_equal(s1, s2) and np.all(np.isfinite(s1))
    assert not np.array_equal(s1, m.sample(300, seed=6)) and m.sample(0).shape == (0,)
    refit = ARIMA.fit_model(1, 0, 1, m.sample(5000, seed=11))
    d = np.abs(refit.coefficients - m.coefficients)                      # a refit, ARIMASuite.scala:58-74 style:
    assert d[0] < 1.0 and np.all(d[1:] < 0.1)                           # intercept within 1, the rest within 0.1
    from sparkts_amd import fit_arima_partition
    recs = [("a", arr["series"][0]), ("b", arr["series"][0][:200]), ("c", arr["series"][0])]
    out = list(fit_arima_partition(recs, 1, 0, 1))
    assert [k for k, _ in out] == ["a", "b", "c"]
    assert np.array_equal(out[0][1], arr["coef"][0]) and np.array_equal(out[2][1], arr["coef"][0])


# ---- ARIMAModel.forecast (ARIMA.scala:696-764): bit-identical to the oracle on every order the build compiles ----
FORECAST_CASES = [(0, 0, 0, 1), (1, 0, 1, 1), (2, 1, 2, 1), (2, 1, 2, 0), (1, 2, 0, 1), (0, 1, 3, 1), (3, 3, 1, 0),
                  (5, 1, 5, 1), (4, 2, 2, 1), (0, 2, 0, 1), (1, 8, 1, 1)]


@pytest.mark.parametrize("pdqi", FORECAST_CASES)
@pytest.mark.parametrize("n_future", [0, 1, 17])
def test_forecast_bit_exact(engine, pdqi, n_future):
    p, d, q, I = pdqi
    rng = np.random.default_rng(1000 + 97 * p + 13 * d + q + I + n_future)
    N, T = 96, 211
    s = rng.standard_normal((N, T)).cumsum(axis=1) * 3.0 + 5.0
    coef = rng.uniform(-0.6, 0.6, (N, p + q + I))
    out = engine.forecast(s, p, d, q, I, coef, n_future)
    exp = np.stack([O.forecast(s[i], p, d, q, I, coef[i], n_future) for i in range(N)])
    assert out.shape == (N, T + n_future)
    assert _same(out, exp), (pdqi, n_future, np.nanmax(np.abs(out - exp)))


@pytest.mark.parametrize("pdqi", [(0, 4, 0, 1), (2, 5, 1, 0), (1, 6, 4, 1), (5, 7, 3, 1), (4, 0, 5, 0), (3, 1, 0, 1)])
@pytest.mark.parametrize("N", [1, 65])
def test_forecast_tiles_ragged(engine, pdqi, N):
    # k_forecast works on 64-series x 16-step LDS tiles (one instantiation per (d, max(p, q))): partial waves,
    # a length that is no multiple of the tile, d up to 7 (output lag d inside the LDS ring), and strided rows
    # (ld > T) through the device entry point
    import torch
    p, d, q, I = pdqi
    rng = np.random.default_rng(77 + 11 * d + p + N)
    T, nf, ld, ldo = 37, 9, 45, 50
    s = rng.standard_normal((N, T)).cumsum(axis=1) + 2.0
    coef = rng.uniform(-0.5, 0.5, (N, p + q + I))
    exp = np.stack([O.forecast(s[i], p, d, q, I, coef[i], nf) for i in range(N)])
    assert _same(engine.forecast(s, p, d, q, I, coef, nf), exp)
    sd = torch.zeros((N, ld), dtype=torch.float64, device="cuda")
    sd[:, :T] = torch.from_numpy(s).cuda()
    cd = torch.from_numpy(coef).cuda().contiguous()
    od = torch.full((N, ldo), -7.0, dtype=torch.float64, device="cuda")
    engine.forecast_device(sd.data_ptr(), N, T, ld, p, d, q, I, cd.data_ptr(), nf, od.data_ptr(), ldo)
    torch.cuda.synchronize()
    o = od.cpu().numpy()
    assert _same(o[:, :T + nf], exp)
    assert np.all(o[:, T + nf:] == -7.0)                     # nothing written past T + nFuture


@pytest.mark.parametrize("T", [2, 3, 4, 6])
def test_forecast_short_series(engine, T):
    # series barely longer than d and shorter than max(p, q): the prefix/diag regions overlap (C-9 edge cases)
    rng = np.random.default_rng(T)
    for p, d, q, I in [(2, 2, 3, 1), (5, 1, 5, 0), (1, 2, 1, 1)]:
        if T < d:
            continue
        s = rng.standard_normal((8, T))
        coef = rng.uniform(-0.5, 0.5, (8, p + q + I))
        out = engine.forecast(s, p, d, q, I, coef, 5)
        exp = np.stack([O.forecast(s[i], p, d, q, I, coef[i], 5) for i in range(8)])
        assert _same(out, exp), (T, p, d, q, I)


def test_forecast_of_fitted_model(engine):
    # fit -> forecast on the C2 workload, and the ARIMA(0,0,0) mean KAT (ARIMASuite.scala:122-132) through the GPU
    N, T = 512, 1024
    s = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 20261015).cpu().numpy()
    res = engine.fit_batch(s, 2, 1, 2, True)
    ok = res["status"] == 0
    f = engine.forecast(s[ok], 2, 1, 2, True, res["coef"][ok], 30)
    exp = np.stack([O.forecast(s[ok][i], 2, 1, 2, 1, res["coef"][ok][i], 30) for i in range(int(ok.sum()))])
    assert np.all(np.abs(f - exp) <= 1e-6 * np.abs(exp))      # north_star: forecasts within 1e-6 relative
    assert _same(f, exp)
    from sparkts_amd.models import ARIMA
    meta, arr = load_case("kat_ds1_101")
    m = ARIMA.fit_model(0, 0, 0, arr["series"][0])
    fc = m.forecast(arr["series"][0], 10)
    mean = arr["series"][0].sum() / arr["series"][0].size
    assert np.all(np.abs(np.ravel(fc)[-10:] - mean) < 1e-4)


# ---- order search: same selection as the oracle's grid, bit for bit ----
@pytest.mark.parametrize("grid", [(5, 2, 5, 2), (2, 1, 2, 1), (3, 0, 1, 0)])
def test_order_search_matches_oracle(engine, grid):
    max_p, max_d, max_q, imode = grid
    N, T = 24, 300
    s = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 77).cpu().numpy()
    s[::5] = O.add_time_dependent_effects(np.random.default_rng(2).standard_normal(T), 1, 0, 1, 1, [3.5, 0.3, 0.7])
    order, coef, aic = engine.order_search(s, max_p, max_d, max_q, imode)
    eo, ec, ea = O.order_search(s, max_p, max_d, max_q, imode)
    assert np.array_equal(order, eo), (order, eo)
    assert _same(aic, ea)
    assert _same(coef, ec)
    if grid == (5, 2, 5, 2):
        assert np.all(order[:, 0] >= 0)      # the full C5 grid finds a qualifying model for every series
    else:
        assert np.any(order[:, 0] >= 0) or max_d == 0


def _near_unit_root_coefs(eps_list):
    """ARIMA(2,0,2)+c coefficient rows whose AR and MA polynomials have roots at radius 1 +- eps (real pairs and
    complex pairs), the boundary that isStationary / isInvertible decide (ARIMA.scala:777-815)."""
    rows = []
    for eps in eps_list:
        for r in (1.0 + eps, 1.0 - eps):
            for w in (0.0, 0.7, 2.1):
                if w == 0.0:                     # real roots r and 3: (1 - x/r)(1 - x/3)
                    a1, a2 = 1.0 / r + 1.0 / 3.0, -1.0 / (3.0 * r)
                else:                            # complex pair r e^{+-iw}
                    a1, a2 = 2.0 * np.cos(w) / r, -1.0 / (r * r)
                rows.append([0.5, a1, a2, 0.2, 0.1])       # AR side on the boundary, MA well inside
                rows.append([0.5, 0.2, 0.1, -a1, -a2])     # MA side on the boundary (1 + th1 x + th2 x^2)
    return np.array(rows)


def test_model_flags_near_unit_circle(engine):
    # the GPU uses a Schur-Cohn step-down, the reference companion-matrix eigenvalues. Both must agree
    # for roots 1e-12 .. 1e-6 away from |z| = 1 (beyond that the answer is below the eigen-solver's own rounding
    # and the reference itself is implementation-defined: DESIGN.md 5.2).
    coef = _near_unit_root_coefs([1e-6, 1e-9, 1e-12])
    f = engine.model_flags(coef, 2, 2, True)
    exp = np.array([O.model_flags(c, 2, 2, 1) for c in coef])
    assert np.array_equal(f, exp), np.nonzero(f != exp)


# ---- generator parity: ARIMAModel.sample / addTimeDependentEffects (ARIMA.scala:629-678) on identical noise ----
_M32 = 0xFFFFFFFF


def _philox4x32_10(ctr, k0, k1):
    c = list(ctr)
    for _ in range(10):
        p0, p1 = 0xD2511F53 * c[0], 0xCD9E8D57 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & _M32, p1 & _M32, ((p0 >> 32) ^ c[3] ^ k1) & _M32, p0 & _M32]
        k0, k1 = (k0 + 0x9E3779B9) & _M32, (k1 + 0xBB67AE85) & _M32
    return c


def _u01_53(a, b):
    return (float(a >> 5) * 67108864.0 + float(b >> 6)) * (1.0 / 9007199254740992.0)


def _roots_ok(poly):                       # the sampler's Schur-Cohn test, same operations (arima_kernels.hip)
    a = list(poly)
    for mm in range(len(a) - 1, 0, -1):
        kk = a[mm]
        if not abs(kk) < 1.0:
            return False
        den = 1.0 - kk * kk
        a = [(a[i] - kk * a[mm - i]) / den for i in range(mm)] + a[mm:]
    return True


def _sampler_coef(gsid, seed, p, q, I, base, jitter):
    """Restates k_sample's per-series coefficient draw (Philox4x32-10, redraw until stationary and invertible)."""
    K = I + p + q
    k0, k1 = seed & _M32, seed >> 32
    for attempt in range(16):
        trial = [0.0] * K
        for j in range(0, K, 2):
            o = _philox4x32_10([j, gsid & _M32, gsid >> 32, 0x5A17 + attempt], k0 ^ 0x3C6EF372, k1 ^ 0xA54FF53A)
            trial[j] = base[j] + jitter * (2.0 * _u01_53(o[0], o[1]) - 1.0)
            if j + 1 < K:
                trial[j + 1] = base[j + 1] + jitter * (2.0 * _u01_53(o[2], o[3]) - 1.0)
        if _roots_ok([1.0] + [-1.0 * x for x in trial[I:I + p]]) and _roots_ok([1.0] + trial[I + p:]):
            return np.array(trial)
    return np.array(base, dtype=np.float64)


@pytest.mark.parametrize("pdqi", [(2, 1, 2, 1), (1, 0, 1, 1), (3, 2, 1, 0), (5, 1, 5, 1)])
def test_sampler_filter_matches_oracle_on_identical_noise(engine, pdqi):
    # the device generator = Philox noise -> addTimeDependentEffects (ARIMA.scala:629-646) -> inverse differencing;
    # with (0,0,0) and no intercept it returns the noise itself, which lets the oracle filter the SAME noise
    p, d, q, I = pdqi
    N, T, seed, first = 48, 333, 4242, 1000
    base = [0.5, 0.3, -0.2, 0.1, 0.05, -0.05, 0.2, 0.1, -0.1, 0.05, 0.05][: I + p + q]
    noise = _device_sample(engine, N, T, 0, 0, 0, 0, [0.0], 0.0, seed, first).cpu().numpy()
    out = _device_sample(engine, N, T, p, d, q, I, base, 0.02, seed, first).cpu().numpy()
    for i in range(N):
        c = _sampler_coef(first + i, seed, p, q, I, base, 0.02)
        exp = O.add_time_dependent_effects(noise[i], p, d, q, I, c)
        assert _same(out[i], exp), (i, np.max(np.abs(out[i] - exp)))


@pytest.mark.parametrize("xblocks", [0, 4])
def test_express_path_is_transparent(engine, xblocks):
    # k_cg_fit hands long-running series to express workgroups (wave-per-series, row in LDS): results
    # and counters must be identical with and without them, and identical to the oracle
    N, T = 1024, 1024
    s = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 777).cpu().numpy()
    engine.set_option("express_blocks", xblocks)
    try:
        res = engine.fit_batch(s, 2, 1, 2, True)
        st = engine.stats()
    finally:
        engine.set_option("express_blocks", -1)
    if xblocks:
        assert st["express_blocks"] == xblocks
    st_o, coef, ll, cnt = O.fit_batch(s, 2, 1, 2, 1)
    exp = dict(status=st_o, coef=coef, ll=ll, n_eval=cnt[:, 0], n_grad=cnt[:, 1],
               flags=np.array([O.model_flags(coef[i], 2, 2, 1) if st_o[i] == 0 else 0 for i in range(N)]))
    check_fit(res, exp, f"express_blocks={xblocks}")


def test_long_fits_through_express(engine):
    # ARIMA(5,1,5)+c (C4's model) at T=512: many fits run thousands of evaluations (MaxEval failures included),
    # so most of them are donated to the express path
    meta, arr = load_case("c4_515_T512")
    res = engine.fit_batch(arr["series"], 5, 1, 5, True)
    st = engine.stats()
    check_fit(res, arr, "c4_515_T512")
    assert st["express_series"] > 0, st


@pytest.mark.parametrize("name", ["c4_515_T512", "c1_101_T500", "c2_212_T1024_shift", "grid_p5d0q5i1", "grid_p1d2q4i0",
                                  "grid_p0d1q3i1", "grid_p3d0q1i0", "edge_nan_101", "kat_ds1_101_userinit"])
def test_express_objective_passes_parallel_in_time(engine, name):
    # express waves evaluate objective requests with all 64 lanes on one series (css_pit_lds: blocks of the time
    # axis swept until every block's inputs equal its left neighbour's outputs, then the sum of squares folded in
    # order): bit-identical to the oracle's serial recursion. A small batch drains the work counter at once, so
    # fits longer than 32 evaluations are donated to the express path.
    meta, arr = load_case(name)
    engine.set_option("smear", meta["smear"])
    try:
        res = engine.fit_batch(arr["series"], meta["p"], meta["d"], meta["q"], meta["I"], meta["method"],
                               arr.get("user_init"))
        st = engine.stats()
    finally:
        engine.set_option("smear", L.DEFAULT_SMEAR)
    check_fit(res, arr, name)
    if name == "c4_515_T512":
        assert st["express_pit_passes"] > 0, st
        assert st["express_pit_sweeps"] >= 2 * st["express_pit_passes"], st


def test_host_path_chunks_match_oracle(engine):
    # arima_fit_batch cut into 7 chunks over 3 fit contexts (uploads overlapping earlier chunks' fits): every
    # series bit-identical to the oracle, and the counters summed over the chunks
    N, T = 2048, 1024
    s = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 777).cpu().numpy()
    engine.set_option("host_chunk", 300)
    engine.set_option("host_pipeline", 3)
    try:
        res = engine.fit_batch(s, 2, 1, 2, True)
        st_g = engine.stats()
    finally:
        engine.set_option("host_chunk", 1 << 18)
    st, coef, ll, cnt = O.fit_batch(s, 2, 1, 2, 1)
    exp = dict(status=st, coef=coef, ll=ll, n_eval=cnt[:, 0], n_grad=cnt[:, 1],
               flags=np.array([O.model_flags(coef[i], 2, 2, 1) if st[i] == 0 else 0 for i in range(N)]))
    check_fit(res, exp, "host_chunks")
    assert st_g["n_series"] == N and st_g["n_eval"] == int(cnt[:, 0].sum()), st_g


@pytest.mark.parametrize("pipeline", [2, 3])
def test_pipelined_device_fits_match_serial(engine, pipeline):
    # fit_pipeline = P: consecutive arima_fit_batch_device calls rotate over P contexts and run concurrently; each
    # call's outputs must equal the serial run's bit for bit (different orders too, so the contexts differ in shape)
    import torch
    N, T = 1 << 16, 1024
    s = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 99)
    orders = [(2, 1, 2, 1), (1, 1, 1, 1), (2, 1, 2, 1), (3, 1, 2, 0), (2, 1, 2, 1)]

    prev = engine.get_option("fit_pipeline")

    def run(P):
        engine.set_option("fit_pipeline", P)
        outs = []
        try:
            for (p, d, q, I) in orders:
                k = p + q + I
                r = [torch.empty((N, k), dtype=torch.float64, device=s.device),
                     torch.empty(N, dtype=torch.float64, device=s.device)] + \
                    [torch.empty(N, dtype=torch.int32, device=s.device) for _ in range(3)] + \
                    [torch.empty(N, dtype=torch.uint8, device=s.device)]
                engine.fit_batch_device(s.data_ptr(), N, T, T, p, d, q, I, *[t.data_ptr() for t in r],
                                        blocking=False)
                outs.append(r)
            engine.synchronize()
        finally:
            engine.set_option("fit_pipeline", prev)
        return [[t.cpu().numpy() for t in r] for r in outs]

    a, b = run(1), run(pipeline)
    for i, (ra, rb) in enumerate(zip(a, b)):
        for x, y in zip(ra, rb):
            assert _same(x, y), (pipeline, orders[i])


def test_pipelined_fits_that_share_buffers_stay_ordered(engine):
    # fit_pipeline > 1 (the default is 3): a call that reads an in-flight call's outputs (read after write), writes
    # what one reads (write after read) or writes the same outputs (write after write) waits for it, so chained and
    # buffer-reusing asynchronous calls give the serial (fit_pipeline 1) results bit for bit
    import torch
    N, T = 1 << 15, 1024
    s1 = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 71)
    s2 = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 72)
    dev = s1.device

    def outs(k=5):
        return [torch.empty((N, k), dtype=torch.float64, device=dev), torch.empty(N, dtype=torch.float64, device=dev)] + \
            [torch.empty(N, dtype=torch.int32, device=dev) for _ in range(3)] + \
            [torch.empty(N, dtype=torch.uint8, device=dev)]

    def fit(series, o, init=None):
        engine.fit_batch_device(series.data_ptr(), N, T, T, 2, 1, 2, 1, *[t.data_ptr() for t in o],
                                d_user_init=None if init is None else init.data_ptr(), blocking=False)

    def scenario():
        a, b, c = outs(), outs(), outs()
        z = s2.clone()
        fit(s1, a)
        fit(s2, b, init=a[0])          # RAW: b starts from a's coefficients
        fit(z, c)                      # c reads z ...
        zl = outs()
        zl[1] = z[:, 0]                # ... while the next call writes its ll into z's first column: WAR
        fit(s1, zl)
        fit(s1, b)                     # WAW: b's buffers rewritten by a fit of s1
        engine.synchronize()
        return [[t.cpu().numpy() for t in r] for r in (a, b, c)]

    prev = engine.get_option("fit_pipeline")
    try:
        engine.set_option("fit_pipeline", 1)
        serial = scenario()
        engine.set_option("fit_pipeline", 3)
        piped = scenario()
    finally:
        engine.set_option("fit_pipeline", prev)
    for ra, rb in zip(serial, piped):
        for x, y in zip(ra, rb):
            assert _same(x, y)
    assert _same(piped[1][0], piped[0][0])      # the WAW's final contents: s1's fit, as the first call's


@pytest.mark.parametrize("xblocks", [-1, 0])
def test_drain_merge_is_transparent(engine, xblocks):
    # k_cg_fit's drain merge (option merge_live): once the work counter has run out, a wave with few live slots
    # hands them to the merge pool and leaves, and waves still running take them into free slots. Only where a
    # series is fitted changes: outputs bit-identical with the merge off, at the default and at 64 (every drained
    # wave offers its slots: the protocol's worst case), with and without express waves; every series written,
    # no watchdog fault; a subsample against the oracle.
    import torch
    N, T = 1 << 18, 1024
    s = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 4242)
    outs = {}
    dflt = engine.get_option("merge_live")
    engine.set_option("express_blocks", xblocks)
    try:
        for ml in (0, 16, 64):
            engine.set_option("merge_live", ml)
            r = [torch.empty((N, 5), dtype=torch.float64, device=s.device),
                 torch.empty(N, dtype=torch.float64, device=s.device)] + \
                [torch.empty(N, dtype=torch.int32, device=s.device) for _ in range(3)] + \
                [torch.empty(N, dtype=torch.uint8, device=s.device)]
            engine.fit_batch_device(s.data_ptr(), N, T, T, 2, 1, 2, True, *[t.data_ptr() for t in r])
            st = engine.stats()
            outs[ml] = ([t.cpu().numpy() for t in r], st)
    finally:
        engine.set_option("merge_live", dflt)
        engine.set_option("express_blocks", -1)
    base, st0 = outs[0]
    assert st0["merge_series"] == 0 and st0["merge_waves"] == 0, st0
    for ml in (16, 64):
        o, st = outs[ml]
        for x, y in zip(base, o):
            assert _same(x, y), ml
        assert st["series_done"] == N and st["fault"] == 0, st
        assert st["merge_waves"] > 0 and st["merge_series"] > 0, st
        assert st["n_eval"] == st0["n_eval"] and st["n_grad"] == st0["n_grad"], (st, st0)
    rows = np.arange(0, N, N // 256)
    sh = s[torch.as_tensor(rows, device=s.device)].cpu().numpy()
    st_o, coef, ll, cnt = O.fit_batch(sh, 2, 1, 2, 1)
    o = outs[64][0]
    exp = dict(status=st_o, coef=coef, ll=ll, n_eval=cnt[:, 0], n_grad=cnt[:, 1],
               flags=np.array([O.model_flags(coef[i], 2, 2, 1) if st_o[i] == 0 else 0 for i in range(len(rows))]))
    res = dict(coef=o[0][rows], ll=o[1][rows], status=o[2][rows], n_eval=o[3][rows], n_grad=o[4][rows],
               flags=o[5][rows])
    check_fit(res, exp, f"merge64 xblocks={xblocks}")


def test_c4_T4096_vs_oracle(engine):
    # C4 at its own length (BASELINE.json configs[3]): ARIMA(5,1,5)+c, T = 4096, 48 device-generated series checked
    # against the oracle -- status (MaxEval / bracket failures included), n_eval, n_grad, coefficients, LL, flags
    # the benched workload: SURVEY 8(d)'s +-0.05 jitter, as bench.py --config c4 samples it
    N, T = 48, 4096
    base = [0.1, 0.4, -0.2, 0.1, 0.05, -0.05, 0.3, 0.2, -0.1, 0.05, 0.05]
    s = _device_sample(engine, N, T, 5, 1, 5, 1, base, 0.05, 20261015).cpu().numpy()
    res = engine.fit_batch(s, 5, 1, 5, True)
    st, coef, ll, cnt = O.fit_batch(s, 5, 1, 5, 1)
    exp = dict(status=st, coef=coef, ll=ll, n_eval=cnt[:, 0], n_grad=cnt[:, 1],
               flags=np.array([O.model_flags(coef[i], 5, 5, 1) if st[i] == 0 else 0 for i in range(N)]))
    check_fit(res, exp, "c4_T4096")


def test_express_ring_under_pressure_matches_bulk(engine):
    # a small batch of mostly-MaxEval fits: every bulk wave drains early and turns express, so nearly every group of
    # every wave holds a ticket while bulk waves still donate -- the hand-off ring's worst case (a fill must never
    # overwrite an entry before its ticket holder has read it). Results must equal the express-free run bit for bit.
    import torch
    N, T = 1 << 16, 1024
    s = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 20261015)
    outs = {}
    prev = engine.get_option("fit_pipeline")
    engine.set_option("fit_pipeline", 1)      # drained bulk waves turn express only when no other fit may follow
    for xb in (0, -1):
        engine.set_option("express_blocks", xb)
        try:
            r = [torch.empty((N, 6), dtype=torch.float64, device=s.device),
                 torch.empty(N, dtype=torch.float64, device=s.device)] + \
                [torch.empty(N, dtype=torch.int32, device=s.device) for _ in range(3)] + \
                [torch.empty(N, dtype=torch.uint8, device=s.device)]
            engine.fit_batch_device(s.data_ptr(), N, T, T, 3, 1, 2, True, *[t.data_ptr() for t in r])
            st = engine.stats()
        finally:
            engine.set_option("express_blocks", -1)
        outs[xb] = ([t.cpu().numpy() for t in r], st)
    engine.set_option("fit_pipeline", prev)
    (a, _), (b, st) = outs[0], outs[-1]
    assert st["express_series"] > 1000, st
    for x, y in zip(a, b):
        assert _same(x, y)


def test_order_search_T1024_matches_oracle(engine):
    # C5 at its own length: the full (d <= 2, p <= 5, q <= 5, +-c) grid on 16 C2-shaped series of T = 1024, fits of
    # consecutive grid points running concurrently on the search's lanes; order, coefficients and AIC bit-exact
    s = _device_sample(engine, 16, 1024, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 4711).cpu().numpy()
    order, coef, aic = engine.order_search(s, 5, 2, 5, 2)
    eo, ec, ea = O.order_search(s, 5, 2, 5, 2)
    assert np.array_equal(order, eo), (order, eo)
    assert _same(coef, ec)
    assert _same(aic, ea)


def test_order_search_lane_count_is_transparent(engine):
    # every lane keeps its own best per series and candidates compare by (approxAIC, grid position), so the outcome
    # cannot depend on how many lanes run the grid or in which order their fits finish: 1, 8 (default), 32 lanes
    s = _device_sample(engine, 4096, 512, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 99).cpu().numpy()
    res = {}
    for lanes in (1, 8, 32):
        engine.set_option("search_lanes", lanes)
        try:
            assert engine.get_option("search_lanes") == lanes
            res[lanes] = engine.order_search(s, 3, 2, 3, 2)
        finally:
            engine.set_option("search_lanes", 8)
    for lanes in (1, 32):
        for x, y in zip(res[8], res[lanes]):
            assert _same(np.asarray(x), np.asarray(y)), lanes
    assert np.all(res[8][0][:, 0] >= 0)


def test_order_search_express_and_hr_grid_are_transparent(engine):
    # round-4 defaults that only move work: the search's concurrent fits without express waves (search_express_blocks
    # 0) vs with them (-1: as a single fit), and the HR init as capped grids of single-wave workgroups (hr_grid) vs a
    # lane per series -- selections, approxAIC and coefficients bit-identical
    s = _device_sample(engine, 4096, 512, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 7).cpu().numpy()
    res = {}
    try:
        for sx, hg in ((0, -1), (-1, -1), (0, 256), (0, 0)):
            engine.set_option("search_express_blocks", sx)
            engine.set_option("hr_grid", hg)
            res[(sx, hg)] = engine.order_search(s, 3, 2, 3, 2)
    finally:
        engine.set_option("search_express_blocks", 0)
        engine.set_option("hr_grid", -1)
    base = res[(0, -1)]
    for key, r in res.items():
        for x, y in zip(base, r):
            assert _same(np.asarray(x), np.asarray(y)), key
    assert np.all(base[0][:, 0] >= 0)


@pytest.mark.parametrize("hr_grid", [0, 256, 1024])
def test_hr_grid_is_transparent(engine, hr_grid):
    # k_hr_init with a lane per series (0) or a capped grid of single-wave workgroups striding over the series: the
    # same Householder per lane, so the inits -- and the fits from them -- are bit-identical to the oracle either way
    N, T = 2048, 1024
    s = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 31).cpu().numpy()
    engine.set_option("hr_grid", hr_grid)
    try:
        res = engine.fit_batch(s, 2, 1, 2, True)
    finally:
        engine.set_option("hr_grid", -1)
    st, coef, ll, cnt = O.fit_batch(s, 2, 1, 2, 1)
    exp = dict(status=st, coef=coef, ll=ll, n_eval=cnt[:, 0], n_grad=cnt[:, 1],
               flags=np.array([O.model_flags(coef[i], 2, 2, 1) if st[i] == 0 else 0 for i in range(N)]))
    check_fit(res, exp, f"hr_grid={hr_grid}")


def test_wire_format_partition_fit_matches_oracle(engine):
    # records in the JVM <-> Python wire format (PythonConnector.scala:59-88) through fit_arima_records: the
    # coefficients that come back, decoded, equal the oracle's (NaN for failed fits); two series lengths in one
    # partition exercise the bucketing
    from sparkts_amd.timeseriesrdd import bytes_to_key_series, fit_arima_records, key_series_to_bytes
    rng = np.random.default_rng(31)
    recs, exp = [], {}
    for i in range(40):
        T = 300 if i % 3 else 257
        y = O.add_time_dependent_effects(rng.standard_normal(T), 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1])
        y = np.cumsum(y)
        recs.append(key_series_to_bytes(f"s{i}", y))
        e = O.fit(y, 2, 1, 2)
        exp[f"s{i}"] = e["coef"] if e["status"] == 0 else np.full(5, np.nan)
    out = [bytes_to_key_series(b) for b in fit_arima_records(recs, 2, 1, 2)]
    assert [k for k, _ in out] == [f"s{i}" for i in range(40)]
    for k, c in out:
        assert _same(c, exp[k]), k


@pytest.mark.parametrize("pipeline,N", [(1, 5000), (3, 5000), (3, 70000)])
def test_sliced_device_fit_matches_unsliced(engine, pipeline, N):
    # arima_fit_batch_device over more series than one slice (option fit_slice_bytes: 1024 series of T = 1024 here)
    # runs slice by slice over the fit contexts -- the path that bounds C3's 8M-series workspaces on one GPU. Results
    # must equal the one-slice fit bit for bit, and the stats must sum over every slice. N = 70000 is 69 slices: more
    # than the 64 slice slots, so slots are reused within one call and their stats must still be counted once each
    # (ADVICE r3).
    import torch
    T = 1024
    s = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 4242)

    def run():
        r = [torch.empty((N, 5), dtype=torch.float64, device=s.device),
             torch.empty(N, dtype=torch.float64, device=s.device)] + \
            [torch.empty(N, dtype=torch.int32, device=s.device) for _ in range(3)] + \
            [torch.empty(N, dtype=torch.uint8, device=s.device)]
        engine.fit_batch_device(s.data_ptr(), N, T, T, 2, 1, 2, True, *[t.data_ptr() for t in r])
        return [t.cpu().numpy() for t in r], engine.stats()

    prev = engine.get_option("fit_pipeline")
    whole, st_whole = run()
    engine.set_option("fit_slice_bytes", 1024 * 1024 * 8)
    engine.set_option("fit_pipeline", pipeline)
    try:
        sliced, st = run()
    finally:
        engine.set_option("fit_slice_bytes", 0)
        engine.set_option("fit_pipeline", prev)
    for x, y in zip(whole, sliced):
        assert _same(x, y)
    assert st["n_series"] == N and st["n_eval"] == int(whole[3].sum()) and st["n_grad"] == int(whole[4].sum()), st
    assert st["n_eval"] == st_whole["n_eval"] and st["ms_cg_fit"] > 0
    assert st["series_done"] == N, st


def test_express_ring_cap_is_transparent(engine):
    # the express hand-off ring holds a fixed number of entries per launch (32768); tickets beyond it are never
    # filled and their series stay on the bulk path. A 4-entry ring reaches that cap at once on the pressure
    # workload: results must still equal the express-free run bit for bit.
    import torch
    N, T = 1 << 15, 1024
    s = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 20261015)
    outs = {}
    for xb, ring in ((0, 0), (-1, 4)):
        engine.set_option("express_blocks", xb)
        engine.set_option("express_ring", ring)
        try:
            r = [torch.empty((N, 6), dtype=torch.float64, device=s.device),
                 torch.empty(N, dtype=torch.float64, device=s.device)] + \
                [torch.empty(N, dtype=torch.int32, device=s.device) for _ in range(3)] + \
                [torch.empty(N, dtype=torch.uint8, device=s.device)]
            engine.fit_batch_device(s.data_ptr(), N, T, T, 3, 1, 2, True, *[t.data_ptr() for t in r])
            st = engine.stats()
        finally:
            engine.set_option("express_blocks", -1)
            engine.set_option("express_ring", 0)
        outs[ring] = ([t.cpu().numpy() for t in r], st)
    (a, _), (b, st) = outs[0], outs[4]
    assert 0 < st["express_series"] <= 4, st
    assert st["fault"] == 0
    for x, y in zip(a, b):
        assert _same(x, y)


def test_row_pad_is_transparent(engine):
    # option row_pad widens the differenced rows' stride (whole 128-B lines) so that the rows of concurrently
    # streamed series stop sharing the low address bits; results must not move by a bit, on the fit path and on the
    # order search (which keeps one differenced copy per d)
    import torch
    N, T = 8192, 1024
    s = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 7)
    host = s.cpu().numpy()[:512]
    outs = {}
    for pad in (0, 40):
        engine.set_option("row_pad", pad)
        try:
            assert engine.get_option("row_pad") == (48 if pad else 0)
            r = [torch.empty((N, 5), dtype=torch.float64, device=s.device),
                 torch.empty(N, dtype=torch.float64, device=s.device)] + \
                [torch.empty(N, dtype=torch.int32, device=s.device) for _ in range(3)] + \
                [torch.empty(N, dtype=torch.uint8, device=s.device)]
            engine.fit_batch_device(s.data_ptr(), N, T, T, 2, 1, 2, True, *[t.data_ptr() for t in r])
            st = engine.stats()
            srch = engine.order_search(host, 2, 1, 2, 2)
        finally:
            engine.set_option("row_pad", 0)
        outs[pad] = ([t.cpu().numpy() for t in r], st, srch)
    (a, sa, qa), (b, sb, qb) = outs[0], outs[40]
    assert sb["series_done"] == N and sb["fault"] == 0 and sa["n_eval"] == sb["n_eval"]
    for x, y in zip(a, b):
        assert _same(x, y)
    for x, y in zip(qa, qb):
        assert _same(np.asarray(x), np.asarray(y))


@pytest.mark.parametrize("pdqi", [(2, 1, 2, 1), (1, 0, 1, 1), (3, 1, 0, 1), (5, 1, 5, 1), (0, 1, 1, 0)])
@pytest.mark.parametrize("layout", ["aligned", "odd_ld"])
def test_fused_differencing_is_transparent(engine, pdqi, layout):
    # round 6: device fits of d <= 1 read the caller's rows and difference them inside every pass (HR streams, AR-only
    # OLS, bulk objective / gradient passes, express staging) instead of a k_difference workspace. Option fuse_diff:
    # 2 fuses at every order, 1 (default) where it pays (p + q <= 6), 0 never; results must not move by a bit, for
    # 128-B aligned rows and for rows at any 8-B offset (ld = T + 3 and a base one element into the allocation), and
    # must equal the oracle.
    import torch
    p, d, q, I = pdqi
    N, T = 3000, 700
    base = [0.5, 0.3, -0.2, 0.1, 0.05, -0.05, 0.2, 0.1, -0.1, 0.05, 0.05][: I + p + q]
    s = _device_sample(engine, N, T, p, d, q, I, base, 0.05, 555 + p + q)
    if layout == "odd_ld":
        ld = T + 3
        buf = torch.full((N + 1, ld), float("nan"), dtype=torch.float64, device=s.device)
        flat = buf.view(-1)[1:1 + N * ld].view(N, ld)       # rows start at odd 8-B offsets
        flat[:, :T] = s
        ptr = flat.data_ptr()
    else:
        ld, ptr = T, s.data_ptr()
    k = p + q + I
    outs = {}
    try:
        for fuse in (2, 1, 0):
            engine.set_option("fuse_diff", fuse)
            r = [torch.empty((N, k), dtype=torch.float64, device=s.device),
                 torch.empty(N, dtype=torch.float64, device=s.device)] + \
                [torch.empty(N, dtype=torch.int32, device=s.device) for _ in range(3)] + \
                [torch.empty(N, dtype=torch.uint8, device=s.device)]
            engine.fit_batch_device(ptr, N, T, ld, p, d, q, I, *[t.data_ptr() for t in r])
            st = engine.stats()
            outs[fuse] = ([t.cpu().numpy() for t in r], st)
    finally:
        engine.set_option("fuse_diff", 1)
    (a, sa), (b, sb), (c, sc) = outs[2], outs[0], outs[1]
    for x, y, z in zip(a, b, c):
        assert _same(x, y) and _same(x, z), pdqi
    assert sa["series_done"] == N and sa["n_eval"] == sb["n_eval"] == sc["n_eval"]
    rows = np.arange(0, N, 25)
    host = s.cpu().numpy()[rows]
    st_o, coef, ll, cnt = O.fit_batch(host, p, d, q, I)
    exp = dict(status=st_o, coef=coef, ll=ll, n_eval=cnt[:, 0], n_grad=cnt[:, 1],
               flags=np.array([O.model_flags(coef[i], p, q, I) if st_o[i] == 0 else 0 for i in range(len(rows))]))
    res = dict(coef=a[0][rows], ll=a[1][rows], status=a[2][rows], n_eval=a[3][rows], n_grad=a[4][rows], flags=a[5][rows])
    check_fit(res, exp, f"fused {pdqi} {layout}")


def test_lowering_fit_pipeline_keeps_chained_fits_ordered(engine):
    # fits issued at fit_pipeline 3 may still run on contexts 1 and 2 when the caller lowers the option to 1
    # and chains the next fit on them (no synchronize in between). The library must order that call after the fits
    # whose buffers it touches, whatever the current setting: same results as a fully serial run.
    import torch
    N, T = 1 << 15, 1024
    s1 = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 81)
    s2 = _device_sample(engine, N, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 82)
    dev = s1.device

    def outs():
        return [torch.empty((N, 5), dtype=torch.float64, device=dev), torch.empty(N, dtype=torch.float64, device=dev)] + \
            [torch.empty(N, dtype=torch.int32, device=dev) for _ in range(3)] + \
            [torch.empty(N, dtype=torch.uint8, device=dev)]

    def fit(series, o, init=None):
        engine.fit_batch_device(series.data_ptr(), N, T, T, 2, 1, 2, 1, *[t.data_ptr() for t in o],
                                d_user_init=None if init is None else init.data_ptr(), blocking=False)

    def scenario(first_p):
        a, b, c, e = outs(), outs(), outs(), outs()
        engine.set_option("fit_pipeline", first_p)
        fit(s1, a)                     # context 0
        fit(s2, b)                     # context 1 (at 3)
        fit(s1, c)                     # context 2 (at 3)
        engine.set_option("fit_pipeline", 1)
        fit(s2, e, init=c[0])          # RAW on c, which may still run on context 2
        fit(s1, b)                     # WAW on b, which may still run on context 1
        engine.synchronize()
        return [[t.cpu().numpy() for t in r] for r in (a, b, c, e)]

    prev = engine.get_option("fit_pipeline")
    try:
        serial = scenario(1)
        piped = scenario(3)
    finally:
        engine.set_option("fit_pipeline", prev)
    for ra, rb in zip(serial, piped):
        for x, y in zip(ra, rb):
            assert _same(x, y)
