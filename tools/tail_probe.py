"""Tail probe (tools; not part of the product): how much of the fit kernel's time is the critical path of its
slowest series? Fits the C2 batch, then refits the same batch without the series above an n_eval cut."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))


def main():
    import torch
    import sparkts_amd._lib as L
    eng = L.Engine.get(0)
    N, T, p, d, q, I = 1 << 20, 1024, 2, 1, 2, 1
    s = torch.empty((N, T), dtype=torch.float64, device="cuda")
    eng.sample_device(s.data_ptr(), N, T, T, p, d, q, I, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 20261015)

    def fit(x):
        n = x.shape[0]
        outs = [torch.empty((n, 5), dtype=torch.float64, device="cuda"), torch.empty(n, dtype=torch.float64, device="cuda"),
                torch.empty(n, dtype=torch.int32, device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda"),
                torch.empty(n, dtype=torch.int32, device="cuda"), torch.empty(n, dtype=torch.uint8, device="cuda")]
        eng.fit_batch_device(x.data_ptr(), n, T, T, p, d, q, I, *[t.data_ptr() for t in outs])
        eng.fit_batch_device(x.data_ptr(), n, T, T, p, d, q, I, *[t.data_ptr() for t in outs])
        return eng.stats(), outs[3]
    st, nev = fit(s)
    res = {"all": {"ms_cg_fit": st["ms_cg_fit"], "n": N, "max_eval": int(nev.max())}}
    for cut in (2000, 1000, 600, 400, 250):
        keep = nev <= cut
        x = s[keep].contiguous()
        st2, nev2 = fit(x)
        res[f"n_eval<={cut}"] = {"ms_cg_fit": st2["ms_cg_fit"], "n": int(keep.sum()), "dropped": int((~keep).sum()),
                                 "f_passes": st2["f_passes"], "g_passes": st2["g_passes"]}
        del x
    print(json.dumps(res))


if __name__ == "__main__":
    main()
