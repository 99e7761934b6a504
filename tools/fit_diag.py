"""Diagnostics run of the fit kernel (tools; not part of the product): one C2-shaped batch through
arima_fit_batch_device, printing the kernel's counters. With a -DSTS_TIMING build (make dev ... DEVFLAGS=-DSTS_TIMING,
selected with SPARKTS_ARIMA_LIB) it also prints where the waves spend their cycles."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=1 << 20)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--order", default="2,1,2,1")
    ap.add_argument("--smear", type=int, default=1)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--express-blocks", type=int, default=-1)
    a = ap.parse_args()
    import torch
    import sparkts_amd._lib as L
    p, d, q, I = map(int, a.order.split(","))
    base = {(2, 1, 2, 1): [8.2, 0.2, 0.5, 0.3, 0.1], (1, 0, 1, 1): [3.5, 0.3, 0.7],
            (5, 1, 5, 1): [0.1, 0.4, -0.2, 0.1, 0.05, -0.05, 0.3, 0.2, -0.1, 0.05, 0.05]}[(p, d, q, I)]
    eng = L.Engine.get(0)
    eng.set_option("smear", a.smear)
    eng.set_option("express_blocks", a.express_blocks)
    N, T, k = a.series, a.T, p + q + I
    s = torch.empty((N, T), dtype=torch.float64, device="cuda")
    eng.sample_device(s.data_ptr(), N, T, T, p, d, q, I, base, 0.05 if k < 11 else 0.02, 20261015)
    outs = [torch.empty((N, k), dtype=torch.float64, device="cuda"), torch.empty(N, dtype=torch.float64, device="cuda"),
            torch.empty(N, dtype=torch.int32, device="cuda"), torch.empty(N, dtype=torch.int32, device="cuda"),
            torch.empty(N, dtype=torch.int32, device="cuda"), torch.empty(N, dtype=torch.uint8, device="cuda")]
    for r in range(a.reps):
        eng.fit_batch_device(s.data_ptr(), N, T, T, p, d, q, I, *[t.data_ptr() for t in outs])
        st = eng.stats()
    dg = st["diag"]
    out = dict(st)
    if dg[4] > 0:
        clk = dg[4] / (st["ms_cg_fit"] * 1e-3)          # shader cycles per second over the kernel span
        waves = st["grid_blocks"] * 4
        tot = dg[0] + dg[1] + dg[2] + dg[3]
        out["timing"] = dict(clock_GHz=clk / 1e9, span_ms=dg[4] / clk * 1e3,
                             mean_wave_busy_ms=tot / waves / clk * 1e3,
                             frac_f=dg[0] / tot, frac_g=dg[1] / tot, frac_adv=dg[2] / tot, frac_sel=dg[3] / tot,
                             mean_after_drain_ms=dg[5] / waves / clk * 1e3)
    nev = outs[3].cpu()
    out["n_eval_max"] = int(nev.max())
    if dg[0] > 0:            # STS_TIMING build: ll = finish time (100 MHz counter), flags = 1 bulk / 2 express
        import numpy as np
        fin = outs[1].cpu().numpy()
        path = outs[5].cpu().numpy()
        ne = nev.numpy()
        ng = outs[4].cpu().numpy()
        cf = outs[0].cpu().numpy()
        ok = outs[2].cpu().numpy() >= 0
        t_st, t_dn = cf[:, 0], cf[:, 1]
        t0 = t_st.min()
        ms = (fin - t0) / 1e5
        st_ms = (t_st - t0) / 1e5
        dn_ms = np.where(t_dn > 0, (t_dn - t0) / 1e5, -1.0)

        def rec(i):
            return dict(n_eval=int(ne[i]), n_grad=int(ng[i]), start_ms=round(float(st_ms[i]), 2),
                        donate_ms=round(float(dn_ms[i]), 2), finish_ms=round(float(ms[i]), 2), path=int(path[i]))
        order = np.argsort(-ne)[:20]
        out["slowest_series"] = [rec(i) for i in order]
        out["latest_finishers"] = [rec(i) for i in np.argsort(-ms)[:20]]
        top = np.argsort(-ne)[:max(1, N // 1000)]
        dur = ms - st_ms
        out["top_0p1pct"] = dict(count=int(len(top)), n_eval_min=int(ne[top].min()),
                                 start_ms_q=[float(np.quantile(st_ms[top], x)) for x in (0.1, 0.5, 0.9)],
                                 dur_ms_q=[float(np.quantile(dur[top], x)) for x in (0.1, 0.5, 0.9, 1.0)],
                                 dur_per_eval_us=float(np.median(dur[top] / ne[top]) * 1e3),
                                 express_frac=float((path[top] == 2).mean()))
        out["duration_ms_quantiles"] = {str(qq): float(np.quantile(dur, qq)) for qq in (0.5, 0.9, 0.99, 0.999, 1.0)}
        out["finish_ms_quantiles"] = {str(qq): float(np.quantile(ms, qq)) for qq in (0.5, 0.9, 0.99, 0.999, 1.0)}
        out["express_count"] = int((path == 2).sum())
    out["n_eval_p999"] = float(nev.double().quantile(0.999)) if N <= 1 << 24 else None
    print(json.dumps(out))


if __name__ == "__main__":
    main()
