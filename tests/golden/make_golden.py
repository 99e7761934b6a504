"""Generates the committed golden fixtures (tests/golden/*.npz) — run from the repo root:

    python tests/golden/make_golden.py

Inputs: the reference's own data files (R_ARIMA_DataSet1/2.csv, copied as data into ds1.csv / ds2.csv), series
sampled exactly as the reference's Scala tests sample them (commons MersenneTwister(seed) + nextGaussian through
ARIMAModel.sample, tests/jvm_random.py), and seeded numpy noise through ARIMAModel.sample for batches.
Expected outputs: the CPU restatement in oracle/ (pinned to the reference's known-answer tests by
tests/test_oracle_kats.py). The reference itself cannot run here (no JVM), so these vectors pin
the GPU path to the restatement bit for bit, and the restatement to the reference at the reference's own
tolerances.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as O  # noqa: E402
from jvm_random import MersenneTwister  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def jitter_coef(rng, base, p, q, I, jitter):
    for _ in range(100):
        c = np.asarray(base, float) + rng.uniform(-jitter, jitter, len(base))
        if O.is_stationary(c, p, q, I) and O.is_invertible(c, p, q, I):
            return c
    return np.asarray(base, float)


def sample_batch(rng, N, T, p, d, q, I, base, jitter):
    out = np.empty((N, T))
    for i in range(N):
        c = jitter_coef(rng, base, p, q, I, jitter)
        out[i] = O.add_time_dependent_effects(rng.standard_normal(T), p, d, q, I, c)
    return out


def run_case(name, series, p, d, q, I, method=0, user_init=None, smear=O.DEFAULT_SMEAR):
    series = np.ascontiguousarray(np.atleast_2d(series), dtype=np.float64)
    N = series.shape[0]
    k = p + q + I
    ui = None if user_init is None else np.ascontiguousarray(np.broadcast_to(np.asarray(user_init, float), (N, k)))
    st, coef, ll, cnt = O.fit_batch(series, p, d, q, I, method, ui, smear)
    flags = np.array([O.model_flags(coef[i], p, q, I) if st[i] == 0 else 0 for i in range(N)], dtype=np.uint8)
    arrays = dict(series=series, status=st, coef=coef, ll=ll, n_eval=cnt[:, 0], n_grad=cnt[:, 1], n_iter=cnt[:, 2],
                  flags=flags)
    if ui is not None:
        arrays["user_init"] = ui
    meta = dict(name=name, p=p, d=d, q=q, I=I, method=method, smear=smear, user_init=ui is not None)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), meta=json.dumps(meta), **arrays)
    print(f"{name:28s} N={N:4d} T={series.shape[1]:5d} status={np.bincount(st, minlength=11)[:11].tolist()} "
          f"evals(mean)={cnt[:, 0].mean():.1f}")


def main():
    ds1 = np.loadtxt(os.path.join(HERE, "ds1.csv"))
    ds2 = np.loadtxt(os.path.join(HERE, "ds2.csv"))
    # --- the reference's own test inputs ----------------------------------------------------------------
    run_case("kat_ds1_101", ds1, 1, 0, 1, 1)                                   # ARIMASuite.scala:27-41
    run_case("kat_ds1_101_userinit", ds1, 1, 0, 1, 1, user_init=[0.0, 0.2, 1.0])   # test_ARIMA.py:27-32
    run_case("kat_ds2_031", ds2, 0, 3, 1, 1)                                   # ARIMASuite.scala:134-156
    mt = lambda seed, n: np.array(MersenneTwister(seed).gaussians(n))
    s212 = O.add_time_dependent_effects(mt(10, 1000), 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1])
    run_case("kat_mt10_212", s212, 2, 1, 2, 1)                                 # ARIMASuite.scala:43-56
    run_case("kat_mt10_212_shift", s212, 2, 1, 2, 1, smear=0)            # the other Breeze reading
    s112 = O.add_time_dependent_effects(mt(10, 1000), 1, 1, 2, 0, [0.3, 0.7, 0.1])
    run_case("kat_mt10_112_noint", s112, 1, 1, 2, 0)                           # ARIMASuite.scala:76-97
    run_case("kat_mt10_102_on_diff", O.differences_of_order_d(s112, 1)[1:], 1, 0, 2, 0)
    run_case("kat_mt10_000", mt(10, 100), 0, 0, 0, 1)                          # ARIMASuite.scala:114-132
    s200 = O.add_time_dependent_effects(mt(10, 250), 2, 0, 0, 1, [2.5, 0.4, 0.3])
    run_case("kat_mt10_200_ar_only", s200, 2, 0, 0, 1)                         # AR shortcut, ARIMA.scala:90-96
    # --- seeded synthetic batches (configs of BASELINE.json at test size) --------------------------------
    rng = np.random.default_rng(20261015)
    run_case("c1_101_T500", sample_batch(rng, 64, 500, 1, 0, 1, 1, [3.5, 0.3, 0.7], 0.05), 1, 0, 1, 1)
    c2 = sample_batch(rng, 64, 1024, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05)
    run_case("c2_212_T1024", c2, 2, 1, 2, 1)
    run_case("c2_212_T1024_shift", c2[:16], 2, 1, 2, 1, smear=0)
    c4b = [0.1, 0.4, -0.2, 0.1, 0.05, -0.05, 0.3, 0.2, -0.1, 0.05, 0.05]
    run_case("c4_515_T512", sample_batch(rng, 16, 512, 5, 1, 5, 1, c4b, 0.02), 5, 1, 5, 1)
    # order grid at small size: every (p, d, q, intercept) the C5 search visits, 6 series each
    grid = []
    base = sample_batch(rng, 6, 160, 1, 1, 1, 1, [0.5, 0.4, 0.3], 0.05)
    for p in range(0, 6):
        for q in range(0, 6):
            for d in range(0, 3):
                for I in (0, 1):
                    grid.append((p, d, q, I))
    for (p, d, q, I) in grid:
        run_case(f"grid_p{p}d{d}q{q}i{I}", base, p, d, q, I)
    # --- edge cases --------------------------------------------------------------------------------------
    short = rng.standard_normal((2, 16)).cumsum(axis=1)
    for T in range(0, 16):                                   # negative lag-matrix sizes, empty / tiny OLS
        run_case(f"edge_T{T}_212", short[:, :T], 2, 1, 2, 1)
        run_case(f"edge_T{T}_101_noint", short[:, :T], 1, 0, 1, 0)
        run_case(f"edge_T{T}_300", short[:, :T], 3, 0, 0, 1)
        run_case(f"edge_T{T}_000_noint", short[:, :T], 0, 0, 0, 0)
    const = np.full((2, 50), 3.0)
    run_case("edge_constant_111", const, 1, 1, 1, 1)                           # singular AR(m) regression
    run_case("edge_constant_101", const, 1, 0, 1, 1)
    nanser = sample_batch(rng, 3, 120, 1, 0, 1, 1, [1.0, 0.3, 0.4], 0.0)
    nanser[0, 50] = np.nan
    nanser[1, 0] = np.nan
    nanser[2, :] = np.inf
    run_case("edge_nan_101", nanser, 1, 0, 1, 1)
    run_case("edge_unsupported_method", ds1, 1, 0, 1, 1, method=99)             # an unknown method string
    run_case("edge_userinit_nonfinite", ds1, 1, 0, 1, 1, user_init=[np.nan, 0.2, 1.0])
    run_case("edge_userinit_wild", ds1, 1, 0, 1, 1, user_init=[0.0, 3.0, -4.0])


if __name__ == "__main__":
    main()
