"""Generates the autoFit golden fixtures (tests/golden/autofit_*.npz) -- run from the repo root:

    python tests/golden/make_golden_autofit.py

Inputs: the series of ARIMASuite's autoFit test (ARIMASuite.scala:181-211: ARIMAModel(2,0,0,[2.5,0.4,0.3]).sample(250,
MersenneTwister(10)) and its 5-fold integration), and seeded numpy noise through ARIMAModel.sample for mixed batches
(stationary AR/ARMA, the C2 generator, twice-integrated walks, white noise, a NaN and a constant series).
Expected outputs: oracle.autofit (the CPU restatement of ARIMA.autoFit + kpsstest, pinned by the reference's KATs in
tests/test_oracle_kats.py).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import oracle as O  # noqa: E402
from jvm_random import MersenneTwister  # noqa: E402
from make_golden import sample_batch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def run_case(name, series, max_p, max_d, max_q):
    series = np.ascontiguousarray(np.atleast_2d(series), dtype=np.float64)
    N = series.shape[0]
    rs = [O.autofit(series[i], max_p, max_d, max_q) for i in range(N)]
    arrays = dict(series=series, status=np.array([r["status"] for r in rs], dtype=np.int32),
                  order=np.array([r["order"] for r in rs], dtype=np.int32),
                  coef=np.stack([r["coef"] for r in rs]), aic=np.array([r["aic"] for r in rs]),
                  n_fits=np.array([r["n_fits"] for r in rs], dtype=np.int32))
    meta = dict(name=name, max_p=max_p, max_d=max_d, max_q=max_q)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), meta=json.dumps(meta), **arrays)
    print(f"{name:24s} N={N:4d} T={series.shape[1]:5d} status={np.bincount(arrays['status'], minlength=14).tolist()} "
          f"fits(mean)={arrays['n_fits'].mean():.1f}")


def main():
    noise = np.array(MersenneTwister(10).gaussians(250))
    sampled = O.add_time_dependent_effects(noise, 2, 0, 0, 1, [2.5, 0.4, 0.3])
    high_i = O.inverse_differences_of_order_d(sampled, 5)
    run_case("autofit_kat_maxd2", np.stack([sampled, high_i]), 5, 2, 5)
    run_case("autofit_kat_maxd10", np.stack([sampled, high_i]), 5, 10, 5)
    rng = np.random.default_rng(20261018)
    T = 256
    parts = [
        sample_batch(rng, 12, T, 2, 0, 0, 1, [2.5, 0.4, 0.3], 0.05),                  # the KAT's AR(2)+c
        sample_batch(rng, 12, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05),        # the C2 generator
        sample_batch(rng, 8, T, 1, 0, 1, 1, [3.5, 0.3, 0.7], 0.05),                   # C1's ARMA(1,1)+c
        sample_batch(rng, 8, T, 1, 2, 1, 0, [0.5, 0.3], 0.05),                        # twice integrated
        sample_batch(rng, 6, T, 0, 0, 0, 1, [1.0], 0.0),                              # white noise + c
        sample_batch(rng, 6, T, 0, 1, 1, 0, [0.9], 0.02),                             # near-cancelling MA
    ]
    extra = np.stack([np.full(T, np.nan), np.full(T, 3.0), np.concatenate([np.zeros(T - 1), [1.0]])])
    mixed = np.concatenate(parts + [extra])
    run_case("autofit_mixed_T256", mixed, 5, 2, 5)
    run_case("autofit_mixed_T256_p2q1", mixed[:24], 2, 2, 1)
    c2 = sample_batch(rng, 16, 1024, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05)
    run_case("autofit_c2_T1024", c2, 5, 2, 5)


if __name__ == "__main__":
    main()
