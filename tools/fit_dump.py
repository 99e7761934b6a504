"""Fit a device-generated C2 batch and save every output (tools; A/B of library variants must be bit-identical):
SPARKTS_ARIMA_LIB=... python tools/fit_dump.py out.npz [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))


def main():
    import numpy as np
    import torch
    import sparkts_amd._lib as L
    out, N, T = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 18, 1024
    eng = L.Engine.get(0)
    s = torch.empty((N, T), dtype=torch.float64, device="cuda")
    eng.sample_device(s.data_ptr(), N, T, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 20261015)
    r = [torch.empty((N, 5), dtype=torch.float64, device="cuda"), torch.empty(N, dtype=torch.float64, device="cuda")] + \
        [torch.empty(N, dtype=torch.int32, device="cuda") for _ in range(3)] + [torch.empty(N, dtype=torch.uint8, device="cuda")]
    eng.fit_batch_device(s.data_ptr(), N, T, T, 2, 1, 2, 1, *[t.data_ptr() for t in r])
    eng.synchronize()
    st = eng.stats()
    assert st["series_done"] == N and st["fault"] == 0, st
    np.savez(out, coef=r[0].cpu().numpy(), ll=r[1].cpu().numpy(), status=r[2].cpu().numpy(),
             n_eval=r[3].cpu().numpy(), n_grad=r[4].cpu().numpy(), flags=r[5].cpu().numpy())
    print("saved", out, N)


if __name__ == "__main__":
    main()
