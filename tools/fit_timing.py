"""Dev tool: where the fit kernel's waves spend their cycles, for one library build and fit kernel variant.

Needs a -DSTS_TIMING build (make -C spark-timeseries_amd/csrc dev TAG=timing DEVFLAGS=-DSTS_TIMING), selected with
SPARKTS_ARIMA_LIB. Runs one isolated C2-shaped device fit per --fit-kernel value and prints one JSON line each:
launch ms, wave passes, lane utilisation, and shader cycles per wave pass by phase (objective pass, gradient pass,
optimizer steps + refill + hand-off, pass selection) -- the phase sums come from the kernel's s_memtime counters.

usage: SPARKTS_ARIMA_LIB=... python tools/fit_timing.py [--series N] [--fit-kernel 0 3] [--order 2,1,2,1 --T 1024]
"""
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
    ap.add_argument("--fit-kernel", type=int, nargs="+", default=[0, 3])
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--express-blocks", type=int, default=-1)
    a = ap.parse_args()
    import torch
    import sparkts_amd._lib as L
    p, d, q, I = map(int, a.order.split(","))
    base = {(2, 1, 2, 1): [8.2, 0.2, 0.5, 0.3, 0.1], (1, 0, 1, 1): [3.5, 0.3, 0.7],
            (5, 1, 5, 1): [0.1, 0.4, -0.2, 0.1, 0.05, -0.05, 0.3, 0.2, -0.1, 0.05, 0.05]}[(p, d, q, I)]
    eng = L.Engine.get(0)
    eng.set_option("express_blocks", a.express_blocks)
    N, T, k = a.series, a.T, p + q + I
    S = T - d - max(p, q)
    s = torch.empty((N, T), dtype=torch.float64, device="cuda")
    eng.sample_device(s.data_ptr(), N, T, T, p, d, q, I, base, 0.05 if k < 11 else 0.02, 20261015)
    outs = [torch.empty((N, k), dtype=torch.float64, device="cuda"), torch.empty(N, dtype=torch.float64, device="cuda"),
            torch.empty(N, dtype=torch.int32, device="cuda"), torch.empty(N, dtype=torch.int32, device="cuda"),
            torch.empty(N, dtype=torch.int32, device="cuda"), torch.empty(N, dtype=torch.uint8, device="cuda")]
    for fk in a.fit_kernel:
        eng.set_option("fit_kernel", fk)
        best = None
        for _ in range(a.reps):
            eng.fit_batch_device(s.data_ptr(), N, T, T, p, d, q, I, *[t.data_ptr() for t in outs])
            st = eng.stats()
            if best is None or st["ms_cg_fit"] < best["ms_cg_fit"]:
                best = st
        st = best
        dg = st["diag"]
        wf, wm, wg = st["wave_f_passes"], st["wave_multi_passes"], st["wave_g_passes"]
        wp = wf + wm + wg
        tot = dg[0] + dg[1] + dg[2] + dg[3]
        print(json.dumps({
            "lib": os.path.basename(L.LIB_PATH), "fit_kernel": fk, "series": N, "ms_cg": round(st["ms_cg_fit"], 2),
            "wave_passes": {"f": wf, "multi": wm, "g": wg}, "lane_util": (st["f_passes"] + st["g_passes"]) / 64.0 / wp,
            "express_series": st["express_series"], "span_Mcyc": dg[4] / 1e6,
            "phase_frac": {"f": dg[0] / tot, "g": dg[1] / tot, "adv": dg[2] / tot, "sel": dg[3] / tot} if tot else None,
            "cyc_per_step_f_any": dg[0] / max(wf + wm, 1) / S, "cyc_per_step_g": dg[1] / max(wg, 1) / S,
            "cyc_adv_per_pass": dg[2] / max(wp, 1), "cyc_sel_per_pass": dg[3] / max(wp, 1),
            "cyc_step_per_pass": st.get("diag_step_cycles", 0) / max(wp, 1),
            "cyc_refill_per_pass": st.get("diag_refill_cycles", 0) / max(wp, 1),
            "objective_chain_use": st["spec_chains"] / st["wave_chains"] if st.get("wave_chains") else None,
            "low_util_passes": st.get("low_util_passes"),
            "drained_Mcyc_per_wave": dg[5] / max(st["grid_blocks"], 1) / 1e6,
            "n_eval": st["n_eval"], "series_done": st["series_done"]}), flush=True)


if __name__ == "__main__":
    main()
