"""bench.py's parity helpers (the `parity` block of the bench line) on fabricated CPU data: a row
counts as matching only when every output is bit-identical -- NaN payloads and signed zeros compared by bits, not by
value -- and a failed fit matches the oracle only with NaN coefficients."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

torch = pytest.importorskip("torch")


@pytest.fixture
def bench():
    # imported inside the tests: bench.py sets GPU_MAX_HW_QUEUES at import, which must not leak into a GPU test run
    # that merely collects this file
    sys.path.insert(0, ROOT)
    import bench as b
    return b


def _outs(n=6, k=5, seed=0):
    g = torch.Generator().manual_seed(seed)
    return dict(coef=torch.randn((n, k), generator=g, dtype=torch.float64),
                ll=torch.randn(n, generator=g, dtype=torch.float64),
                status=torch.zeros(n, dtype=torch.int32), n_eval=torch.full((n,), 40, dtype=torch.int32),
                n_grad=torch.full((n,), 5, dtype=torch.int32), flags=torch.zeros(n, dtype=torch.uint8))


def test_outputs_match_is_bitwise(bench):
    a = _outs()
    b = {k: v.clone() for k, v in a.items()}
    assert bench.outputs_match(a, b).all()
    b["coef"][1, 2] = -0.0 if a["coef"][1, 2] == 0.0 else np.nextafter(a["coef"][1, 2].item(), np.inf)
    b["ll"][3] = float("nan")
    a["ll"][4] = float("nan")
    b["ll"][4] = float("nan")                   # same NaN bits: still a match
    b["n_eval"][5] += 1
    m = bench.outputs_match(a, b)
    assert m.tolist() == [True, False, True, False, True, False]


def test_same_bits_distinguishes_signed_zero(bench):
    a = torch.tensor([0.0, 1.0], dtype=torch.float64)
    b = torch.tensor([-0.0, 1.0], dtype=torch.float64)
    assert bench.same_bits(a, b).tolist() == [False, True]


def test_oracle_row_parity_counts_rows(bench):
    n, (p, q, I) = 4, (2, 2, 1)
    rng = np.random.default_rng(1)
    coef = rng.uniform(-0.3, 0.3, size=(n, I + p + q))
    exp = dict(status=np.array([0, 0, 1, 0], dtype=np.int32), n_eval=np.array([30, 31, 10000, 40], dtype=np.int32),
               n_grad=np.array([4, 4, 90, 5], dtype=np.int32), coef=coef.copy(), ll=rng.normal(size=n), pqi=(p, q, I))
    exp["coef"][2] = np.nan
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    flags = np.array([O.model_flags(exp["coef"][i], p, q, I) if exp["status"][i] == 0 else 0 for i in range(n)],
                     dtype=np.uint8)
    res = dict(status=exp["status"].copy(), n_eval=exp["n_eval"].copy(), n_grad=exp["n_grad"].copy(),
               coef=exp["coef"].copy(), ll=exp["ll"].copy(), flags=flags)
    assert bench.oracle_row_parity(res, exp) == n
    res["coef"][0, 0] = np.nextafter(res["coef"][0, 0], np.inf)    # one ulp off: row 0 no longer matches
    res["coef"][2, 1] = 0.0                                          # a failed fit must report NaN coefficients
    res["n_grad"][3] += 1
    assert bench.oracle_row_parity(res, exp) == 1
