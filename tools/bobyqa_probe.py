"""Probe: the cost of the css-bobyqa device fit (k_bobyqa_fit) and of autoFit at growing batch sizes on the C2
series generator. Prints one JSON line per measurement (run on the GPU box: python tools/bobyqa_probe.py [N ...]).
PROBE_WHAT=bobyqa runs only the css-bobyqa fits (for counter passes)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import sparkts_amd._lib as L  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [1024, 4096, 16384]
    eng = L.Engine.get(0)
    T = 1024
    for N in sizes:
        s = torch.empty((N, T), dtype=torch.float64, device="cuda")
        eng.sample_device(s.data_ptr(), N, T, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 1234, 0)
        eng.synchronize()
        coef = torch.empty((N, 5), dtype=torch.float64, device="cuda")
        ll = torch.empty(N, dtype=torch.float64, device="cuda")
        st = torch.empty(N, dtype=torch.int32, device="cuda")
        ne = torch.empty(N, dtype=torch.int32, device="cuda")
        only = os.environ.get("PROBE_WHAT", "")
        for method, name in ((L.METHOD_CSS_CGD, "css-cgd"), (1, "css-bobyqa")):
            if only and only not in name:
                continue
            t0 = time.perf_counter()
            eng.fit_batch_device(s.data_ptr(), N, T, T, 2, 1, 2, True, coef.data_ptr(), ll.data_ptr(), st.data_ptr(),
                                 d_n_eval=ne.data_ptr(), method=method)
            dt = time.perf_counter() - t0
            n_eval = ne.cpu().numpy()
            print(json.dumps({"what": f"fit {name}", "N": N, "s": dt, "series_per_s": N / dt,
                              "n_eval_mean": float(n_eval.mean()), "n_eval_p99": float(np.percentile(n_eval, 99)),
                              "n_eval_max": int(n_eval.max()),
                              "status": {str(k): int(v) for k, v in zip(*np.unique(st.cpu().numpy(),
                                                                                  return_counts=True))}}), flush=True)
        if only:
            continue
        t0 = time.perf_counter()
        r = eng.autofit(s.cpu().numpy(), 5, 2, 5)
        dt = time.perf_counter() - t0
        print(json.dumps({"what": "autofit", "N": N, "s": dt, "series_per_s": N / dt,
                          "fits_per_series": float(r["n_fits"].mean()),
                          "status": {str(k): int(v) for k, v in zip(*np.unique(r["status"], return_counts=True))}}),
              flush=True)


if __name__ == "__main__":
    main()
