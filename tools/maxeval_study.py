"""CPU study: do the MaxEval fits of C4 that never turn NaN enter an exactly repeating state?

For every C4-shaped series (ARIMA(5,1,5)+c, T = 4096, SURVEY 8(d)'s coefficients with +-0.05 jitter, host-generated
noise through the oracle's addTimeDependentEffects) the oracle's CG fit records the optimizer state at the top of each
iteration (tools: orc_fit_state_trace): point, searchDirection, delta, the previous objective. The optimizer is a
deterministic function of that state and of the iteration counter modulo k (the Fletcher-Reeves restart,
`iter % n == 0`), so if two iterations i < j have bitwise the same state and (j - i) % k == 0, every later iteration
repeats with period j - i -- and the fit could be fast-forwarded to MaxEval exactly, as the NaN-absorbing state is
(cg_lane.hpp kNanIterEvals). The study reports, over the MaxEval fits with a finite point: how many become periodic,
where, with which period, and how many evaluations a fast-forward would skip.

usage: python tools/maxeval_study.py [--series 1000] [--threads 8] [--out profiles/r06/maxeval_study.json]
"""
import argparse
import ctypes
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

P, D, Q, I, T = 5, 1, 5, 1, 4096
BASE = [0.1, 0.4, -0.2, 0.1, 0.05, -0.05, 0.3, 0.2, -0.1, 0.05, 0.05]
K = I + P + Q
W = 2 * K + 3
CAP = 6000


def _roots_ok(poly):
    a = list(poly)
    for mm in range(len(a) - 1, 0, -1):
        kk = a[mm]
        if not abs(kk) < 1.0:
            return False
        den = 1.0 - kk * kk
        a = [(a[i] - kk * a[mm - i]) / den for i in range(mm)] + a[mm:]
    return True


def make_series(i, seed):
    rng = np.random.default_rng([seed, i])
    for _ in range(16):
        c = np.array(BASE) + rng.uniform(-0.05, 0.05, K)
        if _roots_ok([1.0] + list(-c[I:I + P])) and _roots_ok([1.0] + list(c[I + P:])):
            break
    return O.add_time_dependent_effects(rng.standard_normal(T), P, D, Q, I, c)


def trace(ts):
    L = O.lib()
    buf = np.empty(CAP * W)
    n = ctypes.c_int(0)
    cnt = (ctypes.c_int * 3)()
    ts = np.ascontiguousarray(ts, dtype=np.float64)
    st = L.orc_fit_state_trace(ts.ctypes.data_as(O._dp), T, P, D, Q, I, 1, buf.ctypes.data_as(O._dp), CAP,
                               ctypes.byref(n), cnt)
    return st, buf[: n.value * W].reshape(n.value, W), list(cnt)


def analyse(i, seed):
    ts = make_series(i, seed)
    st, states, cnt = trace(ts)
    out = {"i": i, "status": int(st), "n_eval": cnt[0], "n_grad": cnt[1], "n_iter": cnt[2]}
    if st != 1 or len(states) == 0:
        return out
    last_pt = states[-1, :K]
    out["finite"] = bool(np.all(np.isfinite(last_pt)))
    fin_rows = np.all(np.isfinite(states[:, :K]), axis=1)
    first_nan = int(np.argmin(fin_rows)) if not fin_rows.all() else len(states)
    # evaluations the reference spends while the point is still finite (the part no NaN fast-forward can skip)
    out["evals_finite_prefix"] = int(states[first_nan, 2 * K + 2]) if first_nan < len(states) else cnt[0]
    out["iters_finite_prefix"] = first_nan
    states = states[:first_nan]                                      # look for a repeating state before the NaN
    if len(states) == 0:
        out["periodic"] = False
        return out
    key_bits = states[:, : 2 * K + 2].copy().view(np.int64)          # point, dir, delta, previous objective
    seen = {}
    for it in range(len(states)):
        key = (key_bits[it].tobytes(), (it + 1) % K)                 # iteration it + 1 (1-based), its restart phase
        if key in seen:
            j0 = seen[key]
            out["periodic"] = True
            out["period_start_iter"] = j0 + 1
            out["period"] = it - j0
            out["evals_at_start"] = int(states[j0, 2 * K + 2])
            out["evals_per_period"] = int(states[it, 2 * K + 2] - states[j0, 2 * K + 2])
            out["evals_skippable"] = cnt[0] - int(states[it, 2 * K + 2])
            return out
        seen[key] = it
    out["periodic"] = False
    # the closest approach: the smallest number of distinct state words between nearby iterations (how far from exact)
    best = None
    for lag in range(K, min(8 * K, len(states)) + 1, K):
        diff = (key_bits[lag:] != key_bits[:-lag]).sum(axis=1)
        m = int(diff.min()) if diff.size else None
        if m is not None and (best is None or m < best[0]):
            best = (m, lag)
    out["min_differing_words"] = best
    # does the point still move at all at the end? (relative change over the last 100 iterations)
    tail = states[-min(100, len(states)):, :K]
    with np.errstate(all="ignore"):
        out["tail_rel_move"] = float(np.max(np.abs(tail[-1] - tail[0]) / np.maximum(np.abs(tail[0]), 1e-300)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=1000)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06", "maxeval_study.json"))
    a = ap.parse_args()
    O.lib()
    O.set_threads(1)
    t0 = time.time()
    with ThreadPoolExecutor(a.threads) as ex:                         # ctypes releases the GIL during each fit
        res = list(ex.map(lambda i: analyse(i, a.seed), range(a.series)))
    dt = time.time() - t0
    st = np.array([r["status"] for r in res])
    me = [r for r in res if r["status"] == 1]
    fin = [r for r in me if r.get("finite")]
    per = [r for r in me if r.get("periodic")]
    pref = np.array([r["evals_finite_prefix"] for r in me]) if me else np.zeros(1)
    summary = {
        "workload": f"ARIMA({P},{D},{Q})+c css-cgd, T = {T}, {a.series} series (C4-shaped: SURVEY 8(d) coefficients "
                    f"+-0.05, numpy noise through the oracle's addTimeDependentEffects, seed {a.seed})",
        "seconds": dt,
        "status_counts": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
        "maxeval_fits": len(me), "maxeval_nan_point": len(me) - len(fin), "maxeval_finite_point": len(fin),
        "maxeval_evals_finite_prefix": {"median": float(np.median(pref)), "p90": float(np.percentile(pref, 90)),
                                        "max": int(pref.max()), "mean": float(pref.mean()),
                                        "over_1000": int((pref > 1000).sum()), "over_4000": int((pref > 4000).sum())},
        "periodic": len(per),
        "periods": sorted({r["period"] for r in per}),
        "period_start_iter_median": float(np.median([r["period_start_iter"] for r in per])) if per else None,
        "evals_skippable_mean": float(np.mean([r["evals_skippable"] for r in per])) if per else None,
        "evals_skippable_fraction_of_maxeval_evals": (sum(r["evals_skippable"] for r in per) /
                                                      max(1, sum(r["n_eval"] for r in me))),
        "non_periodic_min_differing_words": [r.get("min_differing_words") for r in me
                                             if not r.get("periodic") and r.get("min_differing_words")][:40],
        "method": "state = (point, searchDirection, delta, previous objective) bits at the top of each CG iteration and "
                  "the restart phase iter mod k; periodic = a state seen twice (the optimizer is a function of it)",
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"summary": summary, "fits": res}, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
