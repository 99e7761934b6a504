"""One rank of a series-sharded batch fit: the MI355X replacement of `TimeSeriesRDD.mapSeries(ARIMA.fitModel)`
(TimeSeriesRDD.scala:249-251) over one node, one process per GPU.

Each rank owns the contiguous range `shard_range(total, rank, world)` of the batch, generates exactly those series on
its device (the sampler is shard-invariant: series i depends only on (seed, i)), fits them through the C ABI
(`arima_fit_batch_device`) and hands its results to rank 0 with a gloo gather -- the host-side result gathering the
north_star allows; there is no collective on the data path.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node=N --master-addr 127.0.0.1 --master-port P \\
        -m sparkts_amd.shard_fit --total 65536 --T 1024 --out shards.npz [--device 0]

Without a torch.distributed environment it runs as a single rank. `--device D` (or SPARKTS_DEVICE) binds every rank
to GPU D instead of LOCAL_RANK's, so the sharded path can be exercised with several ranks on a single GPU.
"""
import argparse
import json
import os
import sys
import time

ORDERS = {"c2": (2, 1, 2, 1, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05)}


def rank_device(local_rank):
    """GPU of this rank: SPARKTS_DEVICE / --device override, else LOCAL_RANK's."""
    ov = os.environ.get("SPARKTS_DEVICE", "")
    return int(ov) if ov != "" else int(local_rank)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--total", type=int, default=65536)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--config", default="c2", choices=sorted(ORDERS))
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--device", type=int, default=None)
    ap.add_argument("--out", required=True)
    args = ap.parse_args(argv)
    if args.device is not None:
        os.environ["SPARKTS_DEVICE"] = str(args.device)

    import numpy as np
    import torch
    import torch.distributed as dist

    from . import _lib as L
    from .sharding import gather_results, max_over_ranks, shard_range

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dev_id = rank_device(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")          # results gather + timing only; the fits never leave the device
    p, d, q, I, base, jitter = ORDERS[args.config]
    k = p + q + I
    b, e = shard_range(args.total, rank, world)
    n = e - b
    torch.cuda.set_device(dev_id)
    dev = torch.device("cuda", dev_id)
    eng = L.Engine.get(dev_id)
    series = torch.empty((max(n, 1), args.T), dtype=torch.float64, device=dev)
    out = dict(coef=torch.empty((max(n, 1), k), dtype=torch.float64, device=dev),
               ll=torch.empty(max(n, 1), dtype=torch.float64, device=dev),
               status=torch.empty(max(n, 1), dtype=torch.int32, device=dev),
               n_eval=torch.empty(max(n, 1), dtype=torch.int32, device=dev),
               n_grad=torch.empty(max(n, 1), dtype=torch.int32, device=dev),
               flags=torch.empty(max(n, 1), dtype=torch.uint8, device=dev))
    if n:
        eng.sample_device(series.data_ptr(), n, args.T, args.T, p, d, q, I, base, jitter, args.seed, b)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if n:
        eng.fit_batch_device(series.data_ptr(), n, args.T, args.T, p, d, q, I, out["coef"].data_ptr(),
                             out["ll"].data_ptr(), out["status"].data_ptr(), out["n_eval"].data_ptr(),
                             out["n_grad"].data_ptr(), out["flags"].data_ptr())
    elapsed = max_over_ranks(time.perf_counter() - t0, dist if world > 1 else None)
    keys = ["coef", "ll", "status", "n_eval", "n_grad", "flags"]
    local = [out[key][:n].cpu().numpy() for key in keys]
    allr = gather_results(local, dist if world > 1 else None)
    if rank == 0:
        meta = {"world": world, "total": args.total, "T": args.T, "config": args.config, "seed": args.seed,
                "devices": "override " + os.environ["SPARKTS_DEVICE"] if os.environ.get("SPARKTS_DEVICE") else
                "LOCAL_RANK", "seconds": elapsed}
        np.savez(args.out, meta=json.dumps(meta), **dict(zip(keys, allr)))
        print(json.dumps(meta), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
