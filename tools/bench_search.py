"""C5 order-search throughput on one GPU (tools; device-resident inputs): the full (d <= 2, p <= 5, q <= 5,
+-intercept) min-approxAIC grid (ARIMA.scala:826-830, 342) over N synthetic C2-shaped series, with the search's
concurrent fit lanes set by --lanes (1 = one grid point at a time). Prints a progress line every 15 s while the
search runs, then one JSON line.
usage: python tools/bench_search.py [--series N] [--lanes L] [--T 1024]
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
    ap.add_argument("--series", type=int, default=1 << 18)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--lanes", type=int, default=8)
    a = ap.parse_args()
    import torch
    import sparkts_amd._lib as L
    eng = L.Engine.get(0)
    eng.set_option("search_lanes", a.lanes)
    N, T = a.series, a.T
    dev = torch.device("cuda:0")
    s = torch.empty((N, T), dtype=torch.float64, device=dev)
    eng.sample_device(s.data_ptr(), N, T, T, 2, 1, 2, True, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 20261015)
    order = torch.empty((N, 4), dtype=torch.int32, device=dev)
    cbest = torch.empty((N, 11), dtype=torch.float64, device=dev)
    aic = torch.empty(N, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    t0 = time.perf_counter()
    eng.order_search_device(s.data_ptr(), N, T, T, 5, 2, 5, 2, order.data_ptr(), cbest.data_ptr(), aic.data_ptr(),
                            stream=stream.cuda_stream, blocking=False)
    ev = torch.cuda.Event()
    ev.record(stream)
    last = t0
    while not ev.query():
        time.sleep(0.05)
        if time.perf_counter() - last > 15:
            last = time.perf_counter()
            print(f"# searching ... {last - t0:.0f} s", file=sys.stderr, flush=True)
    eng.synchronize()
    dt = time.perf_counter() - t0
    o = order.cpu().numpy()
    sel = {}
    for r in o:
        key = f"({r[0]},{r[1]},{r[2]}){'+c' if r[3] == 1 else ''}" if r[0] >= 0 else "none"
        sel[key] = sel.get(key, 0) + 1
    top = dict(sorted(sel.items(), key=lambda kv: -kv[1])[:6])
    print(json.dumps({"workload": "C5 order search", "series": N, "T": T, "lanes": a.lanes, "grid_fits_per_series": 216,
                      "s": dt, "series_per_s": N / dt, "fits_per_s": N * 216 / dt, "selected_orders_top": top}),
          flush=True)


if __name__ == "__main__":
    main()
