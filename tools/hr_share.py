"""Dev tool: the Hannan-Rissanen init's share of a pipelined C2 step.

Runs the bench's C2 workload (1M x 1024, ARIMA(2,1,2)+c, fit_pipeline 6) twice on one engine: as the bench does
(each step: difference -> HR init -> fit), and with the HR inits precomputed once and passed as the user init
(each step: difference -> fit). Both fits start from the same bit-identical points, so their outputs must match;
the throughput difference is what the HR kernel costs inside the pipelined step. Not a bench line: the second
configuration skips work the step must do.

usage: python tools/hr_share.py [--config c2|c4] [--series N] [--steps K]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--pipeline", type=int, default=0, help="fit contexts (0: 6 for c2, 4 for c4, as bench.py)")
    ap.add_argument("--config", default="c2", choices=["c2", "c4"])
    a = ap.parse_args()
    import numpy as np
    import torch
    import sparkts_amd._lib as L
    eng = L.Engine.get(0)
    if a.config == "c2":
        N, T, (p, d, q, I), base, jit = a.series, 1024, (2, 1, 2, 1), [8.2, 0.2, 0.5, 0.3, 0.1], 0.05
    else:
        N, T, (p, d, q, I), jit = a.series, 4096, (5, 1, 5, 1), 0.02
        base = [0.1, 0.4, -0.2, 0.1, 0.05, -0.05, 0.3, 0.2, -0.1, 0.05, 0.05]
    a.pipeline = a.pipeline or (6 if a.config == "c2" else 4)
    k = p + q + I
    dev = torch.device("cuda", 0)
    s = torch.empty((N, T), dtype=torch.float64, device=dev)
    eng.sample_device(s.data_ptr(), N, T, T, p, d, q, I, base, jit, 20261015)
    diffed = np.diff(s.cpu().numpy(), axis=1)            # d = 1 (k_difference is bit-exact to this)
    init_h, hr_st = eng.hannan_rissanen(diffed, p, q, True)
    init = torch.from_numpy(np.ascontiguousarray(init_h, dtype=np.float64)).to(dev)
    del diffed
    eng.set_option("fit_pipeline", a.pipeline)
    outs = [[torch.empty((N, k), dtype=torch.float64, device=dev), torch.empty(N, dtype=torch.float64, device=dev)]
            + [torch.empty(N, dtype=torch.int32, device=dev) for _ in range(3)]
            + [torch.empty(N, dtype=torch.uint8, device=dev)] for _ in range(a.pipeline)]
    res = {}
    for mode in ("hr", "user_init", "hr", "user_init"):
        calls = [0]

        def step():
            o = outs[calls[0] % len(outs)]
            calls[0] += 1
            eng.fit_batch_device(s.data_ptr(), N, T, T, p, d, q, I, *[t.data_ptr() for t in o],
                                 d_user_init=init.data_ptr() if mode == "user_init" else None, blocking=False)
        for _ in range(3):
            step()
        eng.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        eng.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        res.setdefault(mode, []).append(N / dt)
        last = [t.clone() for t in outs[(calls[0] - 1) % len(outs)]]
        res.setdefault(mode + "_out", last)
    same = all(torch.equal(x.view(torch.uint8), y.view(torch.uint8)) for x, y in zip(res["hr_out"], res["user_init_out"]))
    print(json.dumps({"config": a.config, "series": N, "pipeline": a.pipeline, "series_per_s_with_hr": res["hr"],
                      "series_per_s_user_init": res["user_init"], "outputs_identical": same,
                      "hr_failed": int((hr_st != 0).sum())}), flush=True)


if __name__ == "__main__":
    main()
