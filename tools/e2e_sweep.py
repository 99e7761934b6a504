"""Dev tool: arima_fit_batch end to end from pageable host memory (the JNI facade's path) over chunk sizes, fit
contexts and upload threads, on the C2 workload (1M x 1024). One JSON line per setting; results checked bit-identical
to the first setting's.
usage: python tools/e2e_sweep.py [--series 1048576]
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
    ap.add_argument("--series", type=int, default=1 << 20)
    ap.add_argument("--settings", default="262144:3:8,131072:3:8,131072:4:8,65536:4:8,65536:6:8,131072:4:0")
    a = ap.parse_args()
    import numpy as np
    import torch
    import sparkts_amd._lib as L
    eng = L.Engine.get(0)
    N, T = a.series, 1024
    d = torch.empty((N, T), dtype=torch.float64, device="cuda")
    eng.sample_device(d.data_ptr(), N, T, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 20261015, 0)
    host = d.cpu().numpy()
    del d
    torch.cuda.empty_cache()
    ref = None
    for st in a.settings.split(","):
        chunk, pipe, thr = (int(x) for x in st.split(":"))
        eng.set_option("host_chunk", chunk)
        eng.set_option("host_pipeline", pipe)
        eng.set_option("host_copy_threads", thr)
        eng.fit_batch(host[:chunk], 2, 1, 2, True)          # sizes the staging of this setting
        best = 1e9
        for _ in range(2):
            t0 = time.perf_counter()
            r = eng.fit_batch(host, 2, 1, 2, True)
            best = min(best, time.perf_counter() - t0)
        same = None
        if ref is None:
            ref = r
        else:
            same = all(np.array_equal(np.asarray(r[k]).view(np.uint8), np.asarray(ref[k]).view(np.uint8)) for k in r)
        print(json.dumps({"host_chunk": chunk, "host_pipeline": pipe, "host_copy_threads": thr, "seconds": best,
                          "series_per_s": N / best, "GBps_in": host.nbytes / best / 1e9, "same_as_first": same}),
              flush=True)


if __name__ == "__main__":
    main()
