"""World-size-2 gloo tests of the multi-GPU path's host logic (sharding, timing reduction, gather).

The data path has no collective: each rank fits its own contiguous series range. These tests
run the exact sharding/reduction code of bench.py in two CPU processes and check that the union of the shards'
results equals a single-process run (the per-series compute here is the CPU oracle, used as a stand-in checker
workload because there is no GPU in this container)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT


def test_shard_ranges_partition():
    from sparkts_amd.sharding import shard_range, weak_scaling_range
    for n in [0, 1, 7, 64, 1000, 1 << 20]:
        for w in [1, 2, 3, 4, 8]:
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            sizes = [e - b for b, e in rs]
            assert max(sizes) - min(sizes) <= 1
    assert weak_scaling_range(1 << 20, 3) == (3 << 20, 4 << 20)


WORKER = r"""
import os, sys, numpy as np, torch.distributed as dist
sys.path[:0] = [os.environ["ROOT"], os.path.join(os.environ["ROOT"], "spark-timeseries_amd"),
                os.path.join(os.environ["ROOT"], "oracle")]
from sparkts_amd.sharding import shard_range, max_over_ranks, gather_results, parity_over_ranks
import oracle as O
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
rng = np.random.default_rng(0)
N, T = 25, 200
allser = np.stack([O.add_time_dependent_effects(rng.standard_normal(T), 1, 0, 1, 1, [1.0, 0.4, 0.3]) for _ in range(N)])
b, e = shard_range(N, rank, world)
st, coef, ll, cnt = O.fit_batch(allser[b:e], 1, 0, 1, 1)
t = max_over_ranks(float(rank + 1), dist)
st_all, coef_all, cnt_all = gather_results([st, coef, cnt], dist)
# bench.py's per-rank oracle parity: every rank checks its own rows, the verdicts meet in gloo sum / min reductions
st_b, coef_b, _, cnt_b = O.fit_batch(allser[b:e], 1, 0, 1, 1)
ok = int(((st_b == st) & (coef_b.view(np.int64) == coef.view(np.int64)).all(axis=1)).sum())
par = parity_over_ranks(ok, e - b, dist)
bad = parity_over_ranks(ok - (1 if rank == 1 else 0), e - b, dist)     # one rank reports a mismatching row
if rank == 0:
    st1, coef1, _, cnt1 = O.fit_batch(allser, 1, 0, 1, 1)
    assert t == float(world), t
    assert np.array_equal(st_all, st1) and np.array_equal(coef_all, coef1) and np.array_equal(cnt_all, cnt1)
    assert coef_all.shape == (N, 3) and cnt_all.dtype == cnt1.dtype
    assert par == {"ranks": world, "oracle_rows": N, "bit_identical": N, "min_rank_fraction": 1.0,
                   "every_rank_bit_identical": True}, par
    assert bad["ranks"] == world and bad["bit_identical"] == N - 1 and not bad["every_rank_bit_identical"]
    assert bad["min_rank_fraction"] < 1.0
    print("MULTIRANK_OK", flush=True)
dist.barrier()
dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2])
def test_gloo_world2_shards_match_single_process(tmp_path, world):
    script = tmp_path / "worker.py"
    script.write_text(WORKER)
    env = dict(os.environ, ROOT=ROOT, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(script)]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert "MULTIRANK_OK" in out.stdout


def _bench(*extra):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"] + list(extra)
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    import json
    return json.loads(lines[0])


def test_bench_launcher_starts_n_ranks_weak():
    # `bench.py --gpus 2` without a torch.distributed environment starts 2 ranks itself (bench.py:launch_ranks);
    # rank 0 reports the real world size and every rank owns its own 1M-series block (weak scaling)
    r = _bench("--gpus", "2")
    assert r["n_gpus"] == 2 and r["scaling"] == "weak" and r["total_series"] == 2 << 20
    assert [tuple(s) for s in r["shards"]] == [(0, 1 << 20), (1 << 20, 2 << 20)]


def test_bench_launcher_strong_scaling_partitions_total():
    # configs[2]: a fixed total (8M) split into contiguous ranges, one per rank
    r = _bench("--gpus", "2", "--total-series", str(8 << 20))
    assert r["n_gpus"] == 2 and r["scaling"] == "strong" and r["total_series"] == 8 << 20
    shards = [tuple(s) for s in r["shards"]]
    assert shards[0][0] == 0 and shards[-1][1] == 8 << 20 and shards[0][1] == shards[1][0]


def test_bench_single_rank_dry_run():
    r = _bench()
    assert r["n_gpus"] == 1 and [tuple(s) for s in r["shards"]] == [(0, 1 << 20)]
