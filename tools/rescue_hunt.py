"""Dev tool: find the autoFit series whose css-bobyqa retry reaches Powell's RESCUE (status 13 in builds before RESCUE
was restated) in the C2-shaped generators the bench and the probes use, and save those rows for the fixtures.

For every (seed, N) below: ARIMAModel.sample-semantics series on the device (the bench's af generator), autoFit on the
device, and the rows whose status is 13 (or, once RESCUE is restated, whose walk reached it: not observable here, so
the rows are kept by status) are written to gpurun_out/rescue/rows_<seed>.npz with their indices.
usage: python tools/rescue_hunt.py [seed:N ...]     (default 1234:65536 20261015:1048576)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))


def main():
    import numpy as np
    import torch
    import sparkts_amd._lib as L
    jobs = [tuple(int(v) for v in a.split(":")) for a in sys.argv[1:]] or [(1234, 65536), (20261015, 1 << 20)]
    eng = L.Engine.get(0)
    T = 1024
    out_dir = os.path.join(ROOT, "gpurun_out", "rescue")
    os.makedirs(out_dir, exist_ok=True)
    for seed, N in jobs:
        s = torch.empty((N, T), dtype=torch.float64, device="cuda")
        eng.sample_device(s.data_ptr(), N, T, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, seed, 0)
        o = dict(order=torch.empty((N, 4), dtype=torch.int32, device="cuda"),
                 coef=torch.empty((N, 11), dtype=torch.float64, device="cuda"),
                 aic=torch.empty(N, dtype=torch.float64, device="cuda"),
                 status=torch.empty(N, dtype=torch.int32, device="cuda"),
                 n_fits=torch.empty(N, dtype=torch.int32, device="cuda"))
        eng.autofit_device(s.data_ptr(), N, T, T, 5, 2, 5, o["order"].data_ptr(), o["coef"].data_ptr(),
                           o["aic"].data_ptr(), o["status"].data_ptr(), o["n_fits"].data_ptr())
        st = o["status"].cpu().numpy()
        idx = np.nonzero(st == 13)[0]
        rows = s[torch.from_numpy(idx).to("cuda").long()].cpu().numpy() if idx.size else np.zeros((0, T))
        np.savez(os.path.join(out_dir, f"rows_{seed}.npz"), idx=idx, rows=rows, status=st[idx])
        print(json.dumps({"seed": seed, "N": N, "status_counts": {str(k): int(v) for k, v in
                                                                  zip(*np.unique(st, return_counts=True))},
                          "rescue_rows": idx.tolist()}), flush=True)
        del s, o
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
