"""Per-order cost of the C5 order-search grid (tools; not part of the product): every (p, d, q, intercept) point
of the grid fitted on its own through arima_fit_batch_device on N synthetic C2-shaped series, with the fit kernel's
time, evaluation counts and status mix. Prints one JSON line per order plus a summary line.
usage: python tools/grid_profile.py [--series N] [--T 1024] [--max-p 5] [--max-d 2] [--max-q 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=1 << 16)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--max-p", type=int, default=5)
    ap.add_argument("--max-d", type=int, default=2)
    ap.add_argument("--max-q", type=int, default=5)
    ap.add_argument("--orders", default="", help="only these p,d,q,I orders (';'-separated)")
    ap.add_argument("--express-blocks", type=int, default=-1)
    a = ap.parse_args()
    import torch
    import sparkts_amd._lib as L
    eng = L.Engine.get(0)
    eng.set_option("express_blocks", a.express_blocks)
    N, T = a.series, a.T
    dev = torch.device("cuda:0")
    s = torch.empty((N, T), dtype=torch.float64, device=dev)
    eng.sample_device(s.data_ptr(), N, T, T, 2, 1, 2, True, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 20261015)
    coef = torch.empty((N, 11), dtype=torch.float64, device=dev)
    ll = torch.empty(N, dtype=torch.float64, device=dev)
    st = torch.empty(N, dtype=torch.int32, device=dev)
    ne = torch.empty(N, dtype=torch.int32, device=dev)
    ng = torch.empty(N, dtype=torch.int32, device=dev)
    fl = torch.empty(N, dtype=torch.uint8, device=dev)
    tot_ms, tot_eval, rows = 0.0, 0, []
    if a.orders:
        grid = [tuple(map(int, o.split(","))) for o in a.orders.split(";")]
    else:
        grid = [(p, d, q, I) for d in range(a.max_d + 1) for p in range(a.max_p + 1) for q in range(a.max_q + 1)
                for I in (0, 1)]
    for (p, d, q, I) in grid:
        print("fit", p, d, q, I, file=sys.stderr, flush=True)
        try:
            eng.fit_batch_device(s.data_ptr(), N, T, T, p, d, q, I, coef.data_ptr(), ll.data_ptr(), st.data_ptr(),
                                 ne.data_ptr(), ng.data_ptr(), fl.data_ptr())
        except RuntimeError as e:
            print(json.dumps(dict(order=[p, d, q, I], error=str(e), stats=eng.stats())), flush=True)
            continue
        x = eng.stats()
        stc = torch.bincount(st.long(), minlength=11).cpu().tolist()
        r = dict(order=[p, d, q, I], ms_total=round(x["ms_total"], 2), ms_fit=round(x["ms_cg_fit"], 2),
                 mean_eval=round(float(ne.double().mean()), 1), max_eval=int(ne.max()),
                 mean_grad=round(float(ng.double().mean()), 2), maxeval_frac=round(stc[1] / N, 4),
                 passes_per_series=round((x["f_passes"] + x["g_passes"] + x["express_f_passes"] +
                                          x["express_g_passes"]) / N, 2),
                 flops=x["flops"], tflops=round(x["flops"] / max(x["ms_total"], 1e-9) / 1e9, 3),
                 express_series=x["express_series"], status={k: v for k, v in enumerate(stc) if v})
        rows.append(r)
        tot_ms += x["ms_total"]
        tot_eval += int(ne.long().sum())
        print(json.dumps(r), flush=True)
    rows.sort(key=lambda r: -r["ms_total"])
    print(json.dumps(dict(summary=True, series=N, T=T, fits=len(rows), serial_ms=tot_ms,
                          fits_per_s_serial=N * len(rows) / (tot_ms * 1e-3), mean_eval_per_fit=tot_eval / (N * len(rows)),
                          slowest=[(r["order"], r["ms_total"]) for r in rows[:10]])), flush=True)


if __name__ == "__main__":
    main()
