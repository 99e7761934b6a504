"""Pass throughput at full occupancy (dev probe): one objective pass (k_css_loglik) and one gradient pass
(k_css_grad) over every row of an N x T batch, lane per series, no optimizer state. Run under
`rocprofv3 --kernel-trace --stats` and read the kernels' average durations: bytes = N * 8 * (T - d) per launch.

usage: python tools/pass_rate.py [N] [T]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "spark-timeseries_amd"))
import sparkts_amd._lib as L  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
T = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
eng = L.Engine.get(0)
rng = np.random.default_rng(1)
x = np.cumsum(rng.standard_normal((N, T)), axis=1)
dx = np.diff(x, axis=1)
coef = [0.1, 0.2, 0.1, 0.3, 0.1]
for _ in range(3):
    ll = eng.css_loglik(x, 2, 1, 2, True, coef)
    g = eng.css_gradient(dx, 2, 2, True, coef)
print("ok", float(np.nanmean(ll)), float(np.nanmean(g)))
