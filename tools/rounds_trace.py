"""Round-by-round request counts of a rounds fit (fit_kernel 2) at C2 size (dev probe): one device fit of N
device-generated C2 series, then the round-control words (lists G, F+2, F+1, F+0 per round) as JSON lines.

usage: python tools/rounds_trace.py [N] [rounds_max] [rounds_tail]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "spark-timeseries_amd"))
import sparkts_amd._lib as L  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
R = int(sys.argv[2]) if len(sys.argv) > 2 else 96
TA = int(sys.argv[3]) if len(sys.argv) > 3 else -1
T, k = 1024, 5
eng = L.Engine.get(0)
eng.set_option("fit_kernel", 2)
eng.set_option("rounds_max", R)
eng.set_option("rounds_tail", TA)
dev = torch.device("cuda", 0)
s = torch.empty((N, T), dtype=torch.float64, device=dev)
eng.sample_device(s.data_ptr(), N, T, T, 2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05, 20261015, 0)
o = {n: torch.empty(N * (k if n == "coef" else 1), dtype=t, device=dev)
     for n, t in [("coef", torch.float64), ("ll", torch.float64), ("status", torch.int32), ("n_eval", torch.int32),
                  ("n_grad", torch.int32), ("flags", torch.uint8)]}
for _ in range(2):
    eng.fit_batch_device(s.data_ptr(), N, T, T, 2, 1, 2, 1, o["coef"].data_ptr(), o["ll"].data_ptr(),
                         o["status"].data_ptr(), o["n_eval"].data_ptr(), o["n_grad"].data_ptr(), o["flags"].data_ptr(),
                         blocking=True)
rc, tail = eng.rounds_trace()
st = eng.stats()
print(json.dumps({"N": N, "rounds_max": R, "tail": tail, "ms_cg_fit": st["ms_cg_fit"]}))
for r in range(R):
    print(json.dumps({"r": r, "G": int(rc[r, 0]), "F2": int(rc[r, 1]), "F1": int(rc[r, 2]), "F0": int(rc[r, 3]),
                      "tiles": int(rc[r, 4])}))
