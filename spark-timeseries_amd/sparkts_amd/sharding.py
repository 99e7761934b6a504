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


def _active(dist):
    return dist is not None and dist.is_initialized() and dist.get_world_size() > 1


def reduce_over_ranks(value, op="max", dist=None):
    """Max / min / sum of a float over all ranks (gloo/CPU tensor: no GPU involvement)."""
    import torch
    if not _active(dist):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op={"max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN, "sum": dist.ReduceOp.SUM}[op])
    return float(t.item())


def max_over_ranks(value, dist=None):
    """Max of a float over all ranks."""
    return reduce_over_ranks(value, "max", dist)


def parity_over_ranks(matching_rows, checked_rows, dist=None):
    """Every rank checked `checked_rows` of its own series against the oracle and found `matching_rows` bit-identical.
    Returns the node-wide verdict: rows checked and matching over all ranks, the smallest per-rank matching fraction
    and whether every rank matched every row it checked (min over ranks of the per-rank verdict)."""
    ok = 1.0 if checked_rows > 0 and matching_rows == checked_rows else 0.0
    frac = matching_rows / checked_rows if checked_rows else 0.0
    return {"ranks": dist.get_world_size() if _active(dist) else 1,
            "oracle_rows": int(reduce_over_ranks(checked_rows, "sum", dist)),
            "bit_identical": int(reduce_over_ranks(matching_rows, "sum", dist)),
            "min_rank_fraction": reduce_over_ranks(frac, "min", dist),
            "every_rank_bit_identical": reduce_over_ranks(ok, "min", dist) == 1.0}


def gather_results(local_arrays, dist=None):
    """Gather per-rank result arrays (numpy, equal trailing shape on every rank) to every rank, concatenated in rank
    order. Fixed-size tensor collectives (no pickling): the row counts first, then every array's bytes padded to the
    largest rank's."""
    import numpy as np
    import torch
    if not _active(dist):
        return [np.asarray(a) for a in local_arrays]
    world = dist.get_world_size()
    out = []
    for a in local_arrays:
        a = np.ascontiguousarray(a)
        rows = torch.tensor([a.shape[0] if a.ndim else 1], dtype=torch.int64)
        all_rows = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(all_rows, rows)
        row_bytes = a.dtype.itemsize * int(np.prod(a.shape[1:], dtype=np.int64)) if a.ndim > 1 else a.dtype.itemsize
        counts = [int(r.item()) for r in all_rows]
        cap = max(counts) * row_bytes
        buf = torch.zeros(max(cap, 1), dtype=torch.uint8)
        raw = np.frombuffer(a.tobytes(), dtype=np.uint8)
        buf[: raw.size] = torch.from_numpy(raw.copy())
        parts = [torch.zeros(max(cap, 1), dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(parts, buf)
        chunks = [np.frombuffer(parts[r].numpy()[: counts[r] * row_bytes].tobytes(), dtype=a.dtype)
                  .reshape((counts[r],) + a.shape[1:]) for r in range(world)]
        out.append(np.concatenate(chunks))
    return out
