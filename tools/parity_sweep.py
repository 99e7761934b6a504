"""Parity sweep (evidence, run on the GPU box): device fits vs the CPU restatement, bit for bit, over a spread of
orders -- the order-specialised kernels (p, q <= 5, fused and unfused differencing), the runtime-order path
(p or q in 6..20) and css-bobyqa -- on seeded host-generated series. One JSON line per case and a summary line;
every field the fit returns is compared (status, n_eval, n_grad, coefficients, CSS LL, flags).

usage: python tools/parity_sweep.py [--series 1024] [--T 400] [--threads 16] [--out gpurun_out/parity_sweep.jsonl]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# (p, d, q, intercept, method): 0 = css-cgd, 1 = css-bobyqa
CASES = [(1, 0, 1, 1, 0), (2, 1, 2, 1, 0), (0, 1, 1, 0, 0), (3, 0, 0, 1, 0), (5, 1, 5, 1, 0), (4, 2, 3, 1, 0),
         (0, 2, 2, 0, 0), (5, 0, 1, 0, 0), (2, 1, 4, 1, 0), (6, 1, 0, 1, 0), (7, 1, 2, 1, 0), (0, 1, 8, 0, 0),
         (9, 0, 0, 1, 0), (6, 0, 6, 1, 0), (3, 1, 10, 0, 0), (12, 0, 2, 1, 0), (20, 0, 0, 1, 0), (2, 1, 2, 1, 1),
         (1, 0, 1, 1, 1), (5, 1, 5, 1, 1), (3, 0, 2, 0, 1), (7, 1, 2, 1, 1)]


def same(a, b):
    import numpy as np
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return a.shape == b.shape and (np.array_equal(a.view(np.int64), b.view(np.int64)) or
                                   np.array_equal(a, b, equal_nan=True))


def series_for(rng, N, T, d):
    import numpy as np
    x = rng.standard_normal((N, T))
    level = rng.uniform(-5, 5, (N, 1))
    ar = rng.uniform(-0.6, 0.6, (N, 1))
    y = np.empty_like(x)
    y[:, 0] = x[:, 0]
    for t in range(1, T):                                  # AR(1)-ish rows with per-series levels
        y[:, t] = ar[:, 0] * y[:, t - 1] + x[:, t]
    y = y + level
    for _ in range(d):
        y = np.cumsum(y, axis=1) * 0.5
    return np.ascontiguousarray(y)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=1024)
    ap.add_argument("--T", type=int, default=400)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "parity_sweep.jsonl"))
    a = ap.parse_args()
    import numpy as np
    import oracle as O
    import sparkts_amd._lib as L
    O.set_threads(a.threads)
    eng = L.Engine.get(0)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    tot, ok_cases, rows_ok, rows = 0, 0, 0, 0
    with open(a.out, "w") as out:
        for ci, (p, d, q, I, method) in enumerate(CASES):
            rng = np.random.default_rng([20261018, ci])
            s = series_for(rng, a.series, a.T, d)
            fuse_modes = (2, 0) if method == 0 and d <= 1 and max(p, q) <= 5 else (1,)
            t0 = time.time()
            st, coef, ll, cnt = O.fit_batch(s, p, d, q, I, method)
            flags = np.array([O.model_flags(coef[i], p, q, I) if st[i] == 0 else 0 for i in range(len(st))],
                             dtype=np.uint8)
            t_cpu = time.time() - t0
            for fm in fuse_modes:
                eng.set_option("fuse_diff", fm)
                r = eng.fit_batch(s, p, d, q, bool(I), method)
                good = ((r["status"] == st) & (r["n_eval"] == cnt[:, 0]) & (r["n_grad"] == cnt[:, 1]) &
                        (r["flags"] == flags))
                good &= np.array([same(r["coef"][i], coef[i]) and same(r["ll"][i], ll[i]) for i in range(len(st))])
                rec = {"p": p, "d": d, "q": q, "intercept": I, "method": ["css-cgd", "css-bobyqa"][method],
                       "fuse_diff": fm, "series": int(len(st)), "T": a.T, "bit_identical": int(good.sum()),
                       "converged": int((st == 0).sum()), "oracle_seconds": round(t_cpu, 2)}
                out.write(json.dumps(rec) + "\n")
                print(json.dumps(rec), flush=True)
                tot += 1
                ok_cases += int(good.all())
                rows_ok += int(good.sum())
                rows += len(st)
            eng.set_option("fuse_diff", 1)
        summary = {"summary": True, "cases": tot, "cases_bit_identical": ok_cases, "rows": rows,
                   "rows_bit_identical": rows_ok}
        out.write(json.dumps(summary) + "\n")
        print(json.dumps(summary), flush=True)
    sys.exit(0 if ok_cases == tot else 1)


if __name__ == "__main__":
    main()
