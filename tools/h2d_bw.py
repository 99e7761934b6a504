"""Dev tool: host -> device copy bandwidth on the box (what bounds arima_fit_batch's end-to-end leg).

Times, for 4 GiB in 256-MiB blocks: pageable -> device (one stream), pinned -> device on 1, 2 and 4 streams at once,
and a parallel host memcpy pageable -> pinned with 1..16 threads. One JSON line on stdout.
usage: python tools/h2d_bw.py
"""
import ctypes
import json
import os
import threading
import time

import numpy as np
import torch

GiB = 1 << 30
BLOCK = 256 << 20
TOTAL = 4 * GiB


def timed(fn, reps=2):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    dev = torch.device("cuda", 0)
    nb = TOTAL // BLOCK
    d = torch.empty(TOTAL // 8, dtype=torch.float64, device=dev)
    pageable = np.random.default_rng(0).standard_normal(TOTAL // 8)
    pin = torch.empty(TOTAL // 8, dtype=torch.float64).pin_memory()
    pin.numpy()[:] = pageable
    out = {}
    src_t = torch.from_numpy(pageable)
    out["pageable_1stream_GBps"] = TOTAL / timed(lambda: d.copy_(src_t)) / 1e9
    for ns in (1, 2, 4, 8):
        streams = [torch.cuda.Stream(dev) for _ in range(ns)]
        per = BLOCK // 8

        def go():
            for b in range(nb):
                with torch.cuda.stream(streams[b % ns]):
                    d[b * per:(b + 1) * per].copy_(pin[b * per:(b + 1) * per], non_blocking=True)
        out[f"pinned_{ns}streams_GBps"] = TOTAL / timed(go) / 1e9
    libc = ctypes.CDLL("libc.so.6")
    libc.memcpy.restype = ctypes.c_void_p
    libc.memcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    src = pageable.ctypes.data
    dst = pin.data_ptr()
    for nt in (1, 2, 4, 8, 16):
        part = TOTAL // nt

        def cp():
            ths = [threading.Thread(target=libc.memcpy, args=(dst + i * part, src + i * part, part)) for i in range(nt)]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
        t = min(timed(cp) for _ in range(2))
        out[f"host_memcpy_{nt}threads_GBps"] = TOTAL / t / 1e9
    out["affinity_cpus"] = len(os.sched_getaffinity(0))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
