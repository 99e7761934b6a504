"""Measure the SURVEY.md 8(f) rows built this round on one GPU (device-resident inputs):
  forecast      ARIMAModel.forecast (k_forecast) on N x 1024 C2 series, nFuture=30, fitted coefficients
  order_search  C5 grid p,q in [0,5], d in [0,2], +-intercept (216 fits/series) on N x 1024 C2 series
Prints one JSON line. Also checks the device-pointer forecast against the host-buffer entry point on 64 rows.
usage: python tools/bench_next.py [--fc-series N] [--os-series N]
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
    ap.add_argument("--fc-series", type=int, default=1 << 20)
    ap.add_argument("--os-series", type=int, default=1 << 16)
    ap.add_argument("--n-future", type=int, default=30)
    a = ap.parse_args()
    import numpy as np
    import torch
    import sparkts_amd._lib as L
    eng = L.Engine.get(0)
    T, base = 1024, [8.2, 0.2, 0.5, 0.3, 0.1]
    dev = torch.device("cuda:0")
    out = {"gpu": torch.cuda.get_device_name(0)}

    # forecast: fit first (coefficients resident in HBM), then time the forecast kernel alone
    N = a.fc_series
    s = torch.empty((N, T), dtype=torch.float64, device=dev)
    eng.sample_device(s.data_ptr(), N, T, T, 2, 1, 2, True, base, 0.05, 20261015)
    coef = torch.empty((N, 5), dtype=torch.float64, device=dev)
    ll = torch.empty(N, dtype=torch.float64, device=dev)
    st = torch.empty(N, dtype=torch.int32, device=dev)
    eng.fit_batch_device(s.data_ptr(), N, T, T, 2, 1, 2, True, coef.data_ptr(), ll.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    L_ = T + a.n_future
    LD = (L_ + 15) // 16 * 16            # 128-B aligned output rows: k_forecast's flushes are whole lines
    fo = torch.empty((N, LD), dtype=torch.float64, device=dev)
    eng.forecast_device(s.data_ptr(), N, T, T, 2, 1, 2, True, coef.data_ptr(), a.n_future, fo.data_ptr(), LD)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.forecast_device(s.data_ptr(), N, T, T, 2, 1, 2, True, coef.data_ptr(), a.n_future, fo.data_ptr(), LD)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    host = eng.forecast(s[:64].cpu().numpy(), 2, 1, 2, True, coef[:64].cpu().numpy(), a.n_future)
    same = bool(np.array_equal(host, fo[:64, :L_].cpu().numpy()))
    bytes_ = N * (T * 8 + 5 * 8 + L_ * 8)
    out["forecast"] = {"series": N, "T": T, "n_future": a.n_future, "ms": dt * 1e3, "series_per_s": N / dt,
                       "algorithmic_GBps": bytes_ / dt / 1e9, "device_vs_host_api_identical": same}
    del s, coef, ll, st, fo
    torch.cuda.empty_cache()

    # order search (C5 grid)
    N = a.os_series
    if N <= 0:
        print(json.dumps(out))
        return
    s = torch.empty((N, T), dtype=torch.float64, device=dev)
    eng.sample_device(s.data_ptr(), N, T, T, 2, 1, 2, True, base, 0.05, 20261015)
    order = torch.empty((N, 4), dtype=torch.int32, device=dev)
    cbest = torch.empty((N, 11), dtype=torch.float64, device=dev)
    aic = torch.empty(N, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.order_search_device(s.data_ptr(), N, T, T, 5, 2, 5, 2, order.data_ptr(), cbest.data_ptr(), aic.data_ptr())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    o = order.cpu().numpy()
    sel = {}
    for r in o:
        key = f"({r[0]},{r[1]},{r[2]}){'+c' if r[3] == 1 else ''}" if r[0] >= 0 else "none"
        sel[key] = sel.get(key, 0) + 1
    top = dict(sorted(sel.items(), key=lambda kv: -kv[1])[:6])
    out["order_search"] = {"series": N, "T": T, "grid_fits_per_series": 216, "s": dt, "series_per_s": N / dt,
                           "fits_per_s": N * 216 / dt, "selected_orders_top": top}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
