"""Generates the css-bobyqa golden fixtures (tests/golden/bobyqa_*.npz) -- run from the repo root:

    python tests/golden/make_golden_bobyqa.py

ARIMA.fitModel(..., method = "css-bobyqa") (ARIMA.scala:106, fitWithCSSBOBYQA :130-160) on the series of ARIMASuite's
BOBYQA test (ARIMASuite.scala:58-74), the reference's R data set 1, seeded batches of the benchmark generators and
edge cases (a 1-parameter model, a user init, NaN and constant series). Expected outputs: the CPU restatement
(oracle/bobyqa_oracle.c via oracle.fit(method=1)); the file layout is make_golden.py's."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import oracle as O  # noqa: E402
from jvm_random import MersenneTwister  # noqa: E402
from make_golden import run_case, sample_batch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    kat = O.add_time_dependent_effects(np.array(MersenneTwister(10).gaussians(1000)), 2, 1, 2, 1,
                                       [8.2, 0.2, 0.5, 0.3, 0.1])
    run_case("bobyqa_kat_mt10_212", kat, 2, 1, 2, 1, method=1)
    ds1 = np.loadtxt(os.path.join(HERE, "ds1.csv"))
    run_case("bobyqa_ds1_101", ds1, 1, 0, 1, 1, method=1)
    run_case("bobyqa_ds1_101_userinit", ds1, 1, 0, 1, 1, method=1, user_init=[0.0, 0.2, 1.0])
    run_case("bobyqa_ds1_001_noint", ds1, 0, 0, 1, 0, method=1)                  # k = 1: NumberIsTooSmall
    rng = np.random.default_rng(20261019)
    run_case("bobyqa_c2_212_T1024", sample_batch(rng, 32, 1024, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05), 2, 1, 2,
             1, method=1)
    run_case("bobyqa_c1_101_T500", sample_batch(rng, 32, 500, 1, 0, 1, 1, [3.5, 0.3, 0.7], 0.05), 1, 0, 1, 1, method=1)
    run_case("bobyqa_c4_515_T512", sample_batch(rng, 12, 512, 5, 1, 5, 1,
                                                [0.1, 0.4, -0.2, 0.1, 0.05, -0.05, 0.3, 0.2, -0.1, 0.05, 0.05], 0.05),
             5, 1, 5, 1, method=1)
    run_case("bobyqa_ma_011_T256", sample_batch(rng, 16, 256, 0, 1, 1, 1, [0.1, 0.5], 0.05), 0, 1, 1, 1, method=1)
    edge = np.stack([np.full(120, np.nan), np.full(120, 3.0), sample_batch(rng, 1, 120, 1, 0, 1, 1, [1.0, 0.3, 0.4],
                                                                            0.0)[0]])
    run_case("bobyqa_edge_101", edge, 1, 0, 1, 1, method=1)
    run_case("edge_unsupported_method", ds1, 1, 0, 1, 1, method=99)


if __name__ == "__main__":
    main()
