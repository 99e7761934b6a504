"""Dev tool: time one build of the library (SPARKTS_ARIMA_LIB=...) on the C2 workload and print one JSON line with
kernel times, pass counters, timing diagnostics and a digest of the outputs, so variants can be compared for
speed and for bit-identical results in one GPU call.

usage: SPARKTS_ARIMA_LIB=spark-timeseries_amd/libsparkts_arima_dev_X.so python tools/variant_run.py [--series N]
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--config", default="2,1,2,1,1024")
    ap.add_argument("--opt", action="append", default=[])
    args = ap.parse_args()
    import torch
    import sparkts_amd._lib as L
    eng = L.Engine.get(0)
    for o in args.opt:
        n, v = o.split("=")
        eng.set_option(n, int(v))
    p, d, q, I, T = map(int, args.config.split(","))
    base = {(2, 1, 2, 1): [8.2, 0.2, 0.5, 0.3, 0.1], (1, 0, 1, 1): [3.5, 0.3, 0.7]}.get(
        (p, d, q, I), [0.1] + [0.05] * (p + q))
    N = args.series
    k = p + q + I
    dev = torch.device("cuda", 0)
    series = torch.empty((N, T), dtype=torch.float64, device=dev)
    eng.sample_device(series.data_ptr(), N, T, T, p, d, q, I, base, 0.05, 20261015, 0)
    outs = [torch.empty((N, k), dtype=torch.float64, device=dev), torch.empty(N, dtype=torch.float64, device=dev),
            torch.empty(N, dtype=torch.int32, device=dev), torch.empty(N, dtype=torch.int32, device=dev),
            torch.empty(N, dtype=torch.int32, device=dev), torch.empty(N, dtype=torch.uint8, device=dev)]
    best = None
    for _ in range(args.reps):
        eng.fit_batch_device(series.data_ptr(), N, T, T, p, d, q, I, *[t.data_ptr() for t in outs])
        s = eng.stats()
        if best is None or s["ms_cg_fit"] < best["ms_cg_fit"]:
            best = s
    h = hashlib.md5()
    for t in outs:
        h.update(t.cpu().numpy().tobytes())
    diag = best["diag"]
    S = T - d - max(p, q)
    waves = best["grid_blocks"] * 4
    print(json.dumps({"lib": os.path.basename(L.LIB_PATH), "series": N, "ms_cg": round(best["ms_cg_fit"], 2),
                      "ms_hr": round(best["ms_hr_init"], 2), "ms_diff": round(best["ms_difference"], 2),
                      "series_per_s_total": round(N / best["ms_total"] * 1e3),
                      "wave_f": best["wave_f_passes"], "wave_g": best["wave_g_passes"],
                      "wave_multi": best["wave_multi_passes"], "lane_f": best["f_passes"], "lane_g": best["g_passes"],
                      "spec_hits": best["spec_hits"], "n_eval": best["n_eval"], "grid": best["grid_blocks"],
                      "adv_frac": diag[0] / diag[2] if diag[2] else None,
                      "pass_frac": diag[1] / diag[2] if diag[2] else None,
                      "mcycles_per_wave": diag[2] / waves / 1e6 if diag[2] else None,
                      "cyc_per_step_g": diag[3] / best["wave_g_passes"] / S if diag[3] else None,
                      "cyc_per_step_m": diag[4] / best["wave_multi_passes"] / S if diag[4] else None,
                      "cyc_per_step_f": (diag[1] - diag[3] - diag[4]) / best["wave_f_passes"] / S if diag[1] else None,
                      "digest": h.hexdigest()}), flush=True)


if __name__ == "__main__":
    main()
