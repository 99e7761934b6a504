"""Child process of tests/test_gpu_pipeline.py (test infrastructure, not product code).

Runs the configuration bench.py times -- `fit_pipeline` P fit contexts on GPU_MAX_HW_QUEUES hardware queues (the
parent sets the variable before this process starts HIP) -- over one device-generated C2 batch: a serial fit first
(fit_pipeline 1), then `--fits` consecutive pipelined fits rotating over P output sets, and compares every output
set with the serial fit bit for bit. Writes the mismatch counts and the serial result's first rows to --out.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=65536)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--pipeline", type=int, default=6)
    ap.add_argument("--fits", type=int, default=8)
    ap.add_argument("--rows", type=int, default=256)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import numpy as np
    import torch
    import sparkts_amd._lib as L

    p, d, q, I = 2, 1, 2, 1
    k = p + q + I
    dev = torch.device("cuda", 0)
    eng = L.Engine(0)
    N, T = a.N, a.T
    series = torch.empty((N, T), dtype=torch.float64, device=dev)
    eng.sample_device(series.data_ptr(), N, T, T, p, d, q, I, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 20261015)

    def new_out():
        return dict(coef=torch.empty((N, k), dtype=torch.float64, device=dev),
                    ll=torch.empty(N, dtype=torch.float64, device=dev),
                    status=torch.empty(N, dtype=torch.int32, device=dev),
                    n_eval=torch.empty(N, dtype=torch.int32, device=dev),
                    n_grad=torch.empty(N, dtype=torch.int32, device=dev),
                    flags=torch.empty(N, dtype=torch.uint8, device=dev))

    def fit(o, blocking):
        eng.fit_batch_device(series.data_ptr(), N, T, T, p, d, q, I, o["coef"].data_ptr(), o["ll"].data_ptr(),
                             o["status"].data_ptr(), o["n_eval"].data_ptr(), o["n_grad"].data_ptr(),
                             o["flags"].data_ptr(), blocking=blocking)

    eng.set_option("fit_pipeline", 1)
    ref = new_out()
    fit(ref, True)
    serial_done = eng.stats()["series_done"]
    eng.set_option("fit_pipeline", a.pipeline)
    outs = [new_out() for _ in range(a.pipeline)]
    for i in range(a.fits):
        fit(outs[i % a.pipeline], False)
    eng.synchronize()
    last_done = eng.stats()["series_done"]

    def row_mismatch(x, y):
        bad = torch.zeros(N, dtype=torch.bool, device=dev)
        for key in x:
            u, v = x[key], y[key]
            if u.dtype == torch.float64:
                u, v = u.view(torch.int64), v.view(torch.int64)
            ne = u != v
            bad |= ne.reshape(N, -1).any(dim=1) if ne.dim() > 1 else ne
        return int(bad.sum().item())

    mism = [row_mismatch(ref, o) for o in outs]
    r = a.rows
    np.savez(a.out, series=series[:r].cpu().numpy(), **{key: v[:r].cpu().numpy() for key, v in ref.items()},
             meta=json.dumps({"mismatch_per_set": mism, "serial_done": serial_done, "last_done": last_done,
                              "N": N, "pipeline": a.pipeline, "fits": a.fits,
                              "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}))
    print(json.dumps({"mismatch_per_set": mism, "serial_done": serial_done, "last_done": last_done}), flush=True)


if __name__ == "__main__":
    main()
