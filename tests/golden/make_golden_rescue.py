"""Generates the fixtures of css-bobyqa fits that run Powell's RESCUE (bobyqa_oracle.c bq_rescue) -- run from the
repo root after `make -C oracle`:

    python tests/golden/make_golden_rescue.py

Inputs:
  - tests/golden/inputs/rescue_autofit_rows.npz: the 15 series of the C2 generator (ARIMAModel.sample semantics, the
    device sampler) whose autoFit walk met a css-bobyqa retry that reaches RESCUE -- row 54 793 of the 65 536-series
    probe batch (seed 1234) and 14 rows of the 1 048 576-series bench batch (seed 20261015), found on the GPU by
    tools/rescue_hunt.py (before round 6 those rows reported status 13);
  - a constructed family: white noise at level 30 / 100 / 300 fitted as ARMA(1,1)+c, whose CSS objective has a ridge
    along c = level * (1 - phi) -- the intercept and the AR coefficient move together, the interpolation set stretches
    along the ridge and the UPDATE denominators lose their digits (the seeds below are those whose fit enters RESCUE);
  - one C2-like twice-sampled series fitted as ARMA(0,1)+c on its first differences (found by a CPU search).
Outputs (the CPU restatement, oracle.fit(method=1) / oracle.autofit):
  - autofit_rescue_c2_T1024: autoFit of the 15 rows (make_golden_autofit's layout);
  - bobyqa_rescue_*: the retries themselves (css-bobyqa on the walk's differenced series, d = 0, grouped by order),
    the ridge family and the C2-like case (make_golden's layout). Every series of a bobyqa_rescue_* fixture enters
    RESCUE at least once (asserted here and in tests/test_oracle_rescue.py)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import oracle as O  # noqa: E402
import make_golden  # noqa: E402
import make_golden_autofit  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
RIDGE = {30: [33, 71, 94, 98, 101, 155, 166, 208], 100: [6, 21, 40, 42, 53, 57, 62, 99, 108, 129, 131, 170],
         300: [31, 52, 144, 225, 275]}


def rescues(series, p, d, q, I):
    """RESCUE calls of each series' css-bobyqa fit (one thread: the counter is thread-local)."""
    L = O.lib()
    L.orc_bobyqa_last_rescues.restype = ctypes.c_int
    out = []
    for s in series:
        O.fit(s, p, d, q, I, method=1)
        out.append(L.orc_bobyqa_last_rescues())
    return np.array(out)


def ridge_series():
    return np.stack([lvl + np.random.default_rng([seed, lvl]).standard_normal(500)
                     for lvl, seeds in RIDGE.items() for seed in seeds])


def c2_like_series():
    rng = np.random.default_rng([11, 392])
    c = np.array([8.2, 0.2, 0.5, 0.3, 0.1]) + rng.uniform(-0.05, 0.05, 5)
    ts = np.cumsum(O.add_time_dependent_effects(rng.standard_normal(1024), 2, 1, 2, 1, c))
    return O.differences_of_order_d(ts, 1)[None, :]


def main():
    O.set_threads(1)
    rows = np.load(os.path.join(HERE, "inputs", "rescue_autofit_rows.npz"))["rows"]
    make_golden_autofit.run_case("autofit_rescue_c2_T1024", rows, 5, 2, 5)
    # the walk's retries that reach RESCUE, found by replaying each walk with the oracle's RESCUE counter
    L = O.lib()
    L.orc_bobyqa_last_rescues.restype = ctypes.c_int
    groups = {}
    fit0 = O.fit
    for row in rows:
        st, d = O.autofit_select_d(row, 2)
        diffed = O.differences_of_order_d(row, d)

        def fit(ts, p, d_, q, intercept=True, method=0, **kw):
            r = fit0(ts, p, d_, q, intercept, method=method, **kw)
            if method == 1 and L.orc_bobyqa_last_rescues() > 0:
                groups.setdefault((p, q, int(intercept)), []).append(np.array(diffed))
            return r
        O.fit = fit
        try:
            O.autofit(row, 5, 2, 5)
        finally:
            O.fit = fit0
    for (p, q, I), ss in sorted(groups.items()):
        name = f"bobyqa_rescue_af_{p}0{q}{'c' if I else ''}"
        ser = np.stack(ss)
        assert (rescues(ser, p, 0, q, I) > 0).all(), name
        make_golden.run_case(name, ser, p, 0, q, I, method=1)
    ridge = ridge_series()
    assert (rescues(ridge, 1, 0, 1, 1) > 0).all()
    make_golden.run_case("bobyqa_rescue_ridge_101c", ridge, 1, 0, 1, 1, method=1)
    c2 = c2_like_series()
    assert (rescues(c2, 0, 0, 1, 1) > 0).all()
    make_golden.run_case("bobyqa_rescue_c2like_001c", c2, 0, 0, 1, 1, method=1)


if __name__ == "__main__":
    main()
