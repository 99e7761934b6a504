"""css-bobyqa on the GPU (k_bobyqa_fit: ARIMA.fitWithCSSBOBYQA, ARIMA.scala:130-160, commons BOBYQAOptimizer as it
configures it) against the CPU restatement (oracle/bobyqa_oracle.c): status, evaluation count, coefficients, CSS
log-likelihood and flags bit for bit. The golden bobyqa_* fixtures run through test_gpu_parity.test_golden_fixture."""
import numpy as np
import pytest

import oracle as O
from conftest import GOLDEN, all_cases, load_case
from test_gpu_parity import check_fit

pytestmark = pytest.mark.gpu


def _expected(s, p, d, q, I, user_init=None):
    st, coef, ll, cnt = O.fit_batch(s, p, d, q, I, method=1, user_init=user_init)
    flags = np.array([O.model_flags(coef[i], p, q, I) if st[i] == 0 else 0 for i in range(len(st))], dtype=np.uint8)
    return dict(status=st, coef=coef, ll=ll, n_eval=cnt[:, 0], n_grad=cnt[:, 1], flags=flags)


def test_bobyqa_c2_batch_matches_oracle(engine):
    import torch
    N, T = 256, 1024
    s = torch.empty((N, T), dtype=torch.float64, device="cuda")
    engine.sample_device(s.data_ptr(), N, T, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 777, 0)
    engine.synchronize()
    host = s.cpu().numpy()
    check_fit(engine.fit_batch(host, 2, 1, 2, True, 1), _expected(host, 2, 1, 2, 1), "bobyqa_c2_256")


@pytest.mark.parametrize("pqi", [(1, 1, 0), (2, 1, 1), (3, 2, 1), (0, 2, 0), (5, 5, 1), (4, 0, 1), (0, 1, 1)])
def test_bobyqa_orders_match_oracle(engine, pqi):
    p, q, I = pqi
    rng = np.random.default_rng(31 + p * 7 + q)
    T = 300
    s = np.cumsum(rng.standard_normal((24, T)), axis=1) * 0.3 + rng.standard_normal((24, T))
    check_fit(engine.fit_batch(s, p, 1, q, bool(I), 1), _expected(s, p, 1, q, I), f"bobyqa_{pqi}")


def test_bobyqa_user_init_and_device_entry_point(engine):
    import torch
    ds1 = np.loadtxt(f"{GOLDEN}/ds1.csv")
    ui = np.array([[0.0, 0.2, 1.0]])
    check_fit(engine.fit_batch(ds1[None, :], 1, 0, 1, True, 1, ui), _expected(ds1[None, :], 1, 0, 1, 1, ui),
              "bobyqa_userinit")
    N, T = 64, 500
    s = torch.empty((N, T), dtype=torch.float64, device="cuda")
    engine.sample_device(s.data_ptr(), N, T, T, 1, 0, 1, 1, [3.5, 0.3, 0.7], 0.05, 99, 0)
    o = {k: torch.empty(N * (3 if k == "coef" else 1), dtype=t, device="cuda")
         for k, t in [("coef", torch.float64), ("ll", torch.float64), ("status", torch.int32), ("n_eval", torch.int32),
                      ("n_grad", torch.int32), ("flags", torch.uint8)]}
    engine.fit_batch_device(s.data_ptr(), N, T, T, 1, 0, 1, 1, o["coef"].data_ptr(), o["ll"].data_ptr(),
                            o["status"].data_ptr(), o["n_eval"].data_ptr(), o["n_grad"].data_ptr(), o["flags"].data_ptr(),
                            method=1, blocking=True)
    res = {k: v.cpu().numpy() for k, v in o.items()}
    res["coef"] = res["coef"].reshape(N, 3)
    check_fit(res, _expected(s.cpu().numpy(), 1, 0, 1, 1), "bobyqa_device")


def test_bobyqa_layouts_are_transparent(engine):
    # the lane-per-series and wave-per-series kernels (option bobyqa_wave 0 / 1; the default picks by batch size and
    # uses the wave layout for autoFit's retries) run the same operations: outputs bit-identical, for direct fits of
    # several dimensions and for autoFit's retries; a subsample against the oracle
    import torch
    from test_gpu_autofit import check_autofit
    N, T = 512, 1024
    s = torch.empty((N, T), dtype=torch.float64, device="cuda")
    engine.sample_device(s.data_ptr(), N, T, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 4711, 0)
    engine.synchronize()
    host = s.cpu().numpy()
    prev = engine.get_option("bobyqa_wave")
    try:
        for (p, q, I) in ((2, 2, 1), (1, 1, 0), (4, 2, 1)):
            res = {}
            for wave in (0, 1):
                engine.set_option("bobyqa_wave", wave)
                res[wave] = engine.fit_batch(host, p, 1, q, bool(I), 1)
            check_fit(res[1], res[0], f"layouts_{p}{q}{I}")
        idx = np.arange(0, N, 61)
        check_fit({k: v[idx] for k, v in res[1].items()}, _expected(host[idx], 4, 1, 2, 1), "layouts_oracle")
        af = {}
        for wave in (0, 1):
            engine.set_option("bobyqa_wave", wave)
            af[wave] = engine.autofit(host[:128], 5, 2, 5)
        check_autofit(af[1], af[0], "autofit_layouts")
    finally:
        engine.set_option("bobyqa_wave", prev)


@pytest.mark.parametrize("name", all_cases("bobyqa_rescue_"))
def test_bobyqa_rescue_both_layouts_match_oracle(engine, name):
    # Powell's RESCUE (bobyqb label 190; oracle bq_rescue, device bq_rescue_setup / _point / _fold): every series of
    # these fixtures enters it (tests/test_oracle_rescue.py); both kernels bit for bit against the fixture
    meta, arr = load_case(name)
    prev = engine.get_option("bobyqa_wave")
    try:
        for wave in (0, 1):
            engine.set_option("bobyqa_wave", wave)
            res = engine.fit_batch(arr["series"], meta["p"], meta["d"], meta["q"], bool(meta["I"]), 1)
            check_fit(res, arr, f"{name}_wave{wave}")
    finally:
        engine.set_option("bobyqa_wave", prev)


def test_autofit_rows_that_reach_rescue(engine):
    # the 15 C2-generator rows whose walk retries a candidate with css-bobyqa into RESCUE (status 13 before round 6),
    # both retry layouts, against oracle.autofit (fixture autofit_rescue_c2_T1024)
    from test_gpu_autofit import check_autofit
    z = np.load(f"{GOLDEN}/autofit_rescue_c2_T1024.npz", allow_pickle=False)
    exp = {k: z[k] for k in ("order", "coef", "aic", "status", "n_fits")}
    prev = engine.get_option("bobyqa_wave")
    try:
        for wave in (0, 1):
            engine.set_option("bobyqa_wave", wave)
            check_autofit(engine.autofit(z["series"], 5, 2, 5), exp, f"autofit_rescue_wave{wave}")
    finally:
        engine.set_option("bobyqa_wave", prev)
