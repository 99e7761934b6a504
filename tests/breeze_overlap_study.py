"""How much the Breeze overlap semantics at ARIMA.scala:526 matters on the C2 workload.

Fits the same synthetic ARIMA(2,1,2)+c series (T = 1024, ARIMASuite's model +-0.05, seeded numpy noise through
ARIMAModel.sample) with the oracle under both readings of `dEdTheta(1 to -1, ::) := dEdTheta(0 to -2, ::)`:
smear (element-wise ascending copy, the default) and shift (memmove-like). Writes profiles/r02/breeze_overlap.json.
Test infrastructure (it runs the CPU restatement only): python tests/breeze_overlap_study.py [N]
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(HERE, "golden"))
import oracle as O  # noqa: E402
from make_golden import sample_batch  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    rng = np.random.default_rng(20261015)
    s = sample_batch(rng, N, 1024, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05)
    out = {}
    res = {}
    for name, sm in (("smear", 1), ("shift", 0)):
        st, coef, ll, cnt = O.fit_batch(s, 2, 1, 2, 1, smear=sm)
        res[name] = (st, coef, ll, cnt)
        out[name] = dict(converged=float((st == 0).mean()), mean_n_eval=float(cnt[:, 0].mean()),
                         mean_n_grad=float(cnt[:, 1].mean()), mean_n_iter=float(cnt[:, 2].mean()))
    ok = (res["smear"][0] == 0) & (res["shift"][0] == 0)
    dc = np.max(np.abs(res["smear"][1][ok] - res["shift"][1][ok]), axis=1)
    dll = np.abs(res["smear"][2][ok] - res["shift"][2][ok]) / np.abs(res["shift"][2][ok])
    out["series"] = N
    out["both_converged"] = int(ok.sum())
    out["frac_coef_diff_gt_1e-4"] = float((dc > 1e-4).mean())
    out["coef_maxabs_diff"] = dict(median=float(np.median(dc)), p90=float(np.quantile(dc, 0.9)), max=float(dc.max()))
    out["frac_ll_reldiff_gt_1e-6"] = float((dll > 1e-6).mean())
    print(json.dumps(out, indent=1))
    with open(os.path.join(ROOT, "profiles", "r02", "breeze_overlap.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
