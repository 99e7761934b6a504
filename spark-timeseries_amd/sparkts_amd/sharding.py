"""Series sharding across GPUs: one process per GPU, contiguous series ranges, no collective on
the data path. The only cross-rank traffic is the timing barrier and a max-reduction of elapsed time (and, if a
caller wants them on one host, a gather of the per-series results)."""


def shard_range(n_total, rank, world):
    """Contiguous [begin, end) of `n_total` series for `rank` of `world` (sizes differ by at most one)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(n_total, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def weak_scaling_range(n_per_rank, rank):
    """Weak scaling (bench.py): every rank owns n_per_rank series, rank r the r-th block."""
    return rank * n_per_rank, (rank + 1) * n_per_rank


def max_over_ranks(value, dist=None):
    """Max of a float over all ranks (gloo/CPU tensor: no GPU involvement)."""
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_results(local_arrays, dist=None):
    """Gather per-rank result arrays (numpy) to every rank, concatenated in rank order."""
    import numpy as np
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [np.asarray(a) for a in local_arrays]
    out = []
    for a in local_arrays:
        objs = [None] * dist.get_world_size()
        dist.all_gather_object(objs, np.asarray(a))
        out.append(np.concatenate(objs))
    return out
