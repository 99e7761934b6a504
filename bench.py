"""Headline benchmark: series fitted/sec, ARIMA(2,1,2) CSS-CGD, 1M x 1024 pts per GPU (BASELINE.json configs[1];
configs[2] is the same workload over N GPUs).

A step = one arima_fit_batch_device call (the drop-in for ARIMA.fitModel over one partition) over this rank's
device-resident synthetic series: differencing + Hannan-Rissanen init + the full CSS-CGD fit of every series.
Inputs are generated on the device before timing (ARIMAModel.sample semantics, Philox + Box-Muller, seed
20261015, per-series jitter +-0.05 around ARIMASuite's [8.2, 0.2, 0.5, 0.3, 0.1]).

Launch: python bench.py [--gpus N --steps K --warmup W]. With N > 1 and no torch.distributed environment, this
process starts `torch.distributed.run` with N ranks (one per GPU) as a child before touching any GPU and exits
with its status; under torch.distributed.run each rank fits its own contiguous series range (no data-path
collective; gloo carries only the timing barrier and the max-over-ranks reduction).
  --series S        series per GPU (weak scaling, default 1M: configs[1], and configs[2] read per GPU)
  --total-series S  fixed total over all GPUs (strong scaling: configs[2] = 8M series sharded over N GPUs)
  --smear 0|1       Breeze overlap reading at ARIMA.scala:526 (default 1)
  --pipeline P      fit contexts in rotation (arima_set_option "fit_pipeline", default 6; 4 for c4): step i+1's differencing,
                    init and bulk fit run while step i's slowest series finish; every step is still a
                    complete fit of every series, into its own output buffers (one set per context)
  --e2e 0|1         also time one arima_fit_batch call from pageable host memory (default 1)
  --config c5       BASELINE.json configs[4]: a step = the full (d <= 2, p <= 5, q <= 5, +-c) min-approxAIC order search
                    over this rank's shard (strong scaling over --total-series, default 1M); unit series searched/sec
  --config c1       BASELINE.json configs[0]: ARIMA(1,0,1)+c on 10 000 series x 500 pts (the reference's CPU config)
  --config c4       BASELINE.json configs[3]: ARIMA(5,1,5)+c on 1M series x 4096 pts (the long-series path)
  --config af       ARIMA.autoFit (ARIMA.scala:280-375) over C2-shaped series: KPSS choice of d, then the stepwise walk of
                    css-cgd fits (arima_autofit_batch_device); unit series auto-fitted/sec, weak scaling
  --default-leg 0|1 c2, one GPU: also time the drop-in exactly as a caller gets it -- arima_fit_batch_device with the
                    ABI's default options, in a child process that keeps the box's GPU_MAX_HW_QUEUES (default 1)
  --device D        bind every rank to GPU D (also SPARKTS_DEVICE) instead of LOCAL_RANK's: several ranks on one GPU
  --dry-run         no GPU: ranks compute their shards and report (tests/test_multirank.py)
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

# Each fit context (and each order-search lane) is its own HIP stream. HIP maps a process's streams onto
# GPU_MAX_HW_QUEUES hardware queues (default 4), and kernels of streams that share a queue run one after the other:
# 6 contexts + the handle's stream need 8 queues to overlap (C2: 8.65 M series/s with 4 queues and 3 contexts,
# 9.5-9.7 with 8-16 queues and 6-8 contexts; C5's 8 search lanes: 4638 -> 5497 series/s; profiles/r03/j_hwq/{a,b}).
# The C5 order search runs 12 search lanes (round 4; 16 in round 3), which need lanes + 2 queues (round 3: 8 lanes on
# 8 queues 10 654 series/s at 262 144 x 1024, 16 lanes on 24 queues 12 976, profiles/r03/q_lanes); 24 queues kept.
# Set before anything initialises HIP (the GPU boxes export 4); a larger setting in the environment is kept.
_C5 = any(a == "--config=c5" for a in sys.argv) or any(
    a == "--config" and i + 1 < len(sys.argv) and sys.argv[i + 1] == "c5" for i, a in enumerate(sys.argv))
_QUEUES = 24 if _C5 else 8
_BOX_QUEUES = os.environ.get("GPU_MAX_HW_QUEUES")            # the box's own setting (the default-config leg keeps it)
if not os.environ.get("SPARKTS_BENCH_DEFAULT_LEG") and int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or "4") < _QUEUES:
    os.environ["GPU_MAX_HW_QUEUES"] = str(_QUEUES)

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))

CONFIGS = {
    # name: (p, d, q, intercept, T, base coefficients, jitter); c5 searches over C2-shaped series
    "c5": (2, 1, 2, 1, 1024, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05),
    "af": (2, 1, 2, 1, 1024, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05),
    "c2": (2, 1, 2, 1, 1024, [8.2, 0.2, 0.5, 0.3, 0.1], 0.05),
    "c1": (1, 0, 1, 1, 500, [3.5, 0.3, 0.7], 0.05),
    "c4": (5, 1, 5, 1, 4096, [0.1, 0.4, -0.2, 0.1, 0.05, -0.05, 0.3, 0.2, -0.1, 0.05, 0.05], 0.05),
}
# configs[0]: 10k series; every other config 1M per GPU (autoFit too since round 6: each of its ~7 rounds waits for
# its slowest css-bobyqa retry, which a 1M batch amortises -- 34.7k series/s at 1M vs 7.7k at 64k, profiles/r06/e_split)
DEFAULT_SERIES = {"c1": 10000}
METRICS = {
    "c2": "series fitted/sec, ARIMA(2,1,2) CSS-CGD, 1M x 1024 pts",
    "c1": "series fitted/sec, ARIMA(1,0,1) CSS-CGD, 10k x 500 pts (BASELINE.json configs[0])",
    "c4": "series fitted/sec, ARIMA(5,1,5)+c CSS-CGD, 1M x 4096 pts (BASELINE.json configs[3])",
}
FP64_PEAK_TFLOPS = 78.6    # MI355X fp64 vector peak (spec)
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E (MI355X_MICROARCH.md)
# HBM bytes per k_cg_fit launch from the last rocprofv3 PMC passes of this same workload (FETCH_SIZE and
# WRITE_SIZE in their own runs, gfx950 corrections per MI355X_MICROARCH.md; tools/profile.sh ->
# tools/summarize_prof.py --traffic). Counters cannot be read inside a timed bench run, so the measured value
# is carried in this tracked file and reported only when its workload (and build tag) matches the one run.
PMC_TRAFFIC_FILE = os.path.join(ROOT, "tools", "pmc_traffic_c2.json")
LIB_PATH = os.path.join(ROOT, "spark-timeseries_amd", "libsparkts_arima.so")
SEED = 20261015
ISO_STEPS = 3              # isolated launches behind roofline.launch_ms (their median)


def build_sha():
    """sha256 of the HIP library this run loads: the key that ties carried PMC numbers to the measured build."""
    from sparkts_amd.buildinfo import library_sha
    return library_sha()


def pmc_traffic(workload, sha):
    """Carried PMC record of this workload AND this build: the library's sha256, else the sha256 of the build's
    inputs (hipcc output is not byte-reproducible, sparkts_amd/buildinfo.py). (None, None) for any mismatch."""
    from sparkts_amd.buildinfo import match_record, source_sha
    try:
        with open(PMC_TRAFFIC_FILE) as f:
            recs = json.load(f)
    except (OSError, ValueError):
        return None, None
    # the source fallback only for the default library: a dev library (SPARKTS_ARIMA_LIB) is built from the same
    # sources with extra -D flags that the source sha cannot see
    src = None if os.environ.get("SPARKTS_ARIMA_LIB") else source_sha()
    return match_record(recs if isinstance(recs, list) else [recs], workload, sha, src)


def physical_cores():
    """Physical cores of the host (unique (package, core) pairs of /proc/cpuinfo), or None."""
    try:
        pairs, phys, core = set(), None, None
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    phys = line.split(":")[1].strip()
                elif line.startswith("core id"):
                    core = line.split(":")[1].strip()
                elif not line.strip():
                    if phys is not None and core is not None:
                        pairs.add((phys, core))
                    phys = core = None
        return len(pairs) or None
    except OSError:
        return None


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class heartbeat:
    """A line on stderr every `every` s while a long device call runs (a silent minute reads as a hang on the box);
    ctypes releases the GIL during the call, so the thread gets to run."""

    def __init__(self, what, every=30):
        self.what, self.every = what, every

    def __enter__(self):
        import threading
        self.done, t0 = threading.Event(), time.perf_counter()

        def beat():
            while not self.done.wait(self.every):
                log(f"{self.what} ... {time.perf_counter() - t0:.0f} s")
        self.th = threading.Thread(target=beat, daemon=True)
        self.th.start()
        return self

    def __exit__(self, *exc):
        self.done.set()
        self.th.join()
        return False


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """Re-run this script under torch.distributed.run with n ranks, as a CHILD process (no exec: nothing here
    has touched the GPU, and the parent never does). Returns the child's exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def cpu_baseline(series_host, p, d, q, I, smear, target_s):
    """The CPU restatement (oracle/, kind "port") on a bounded sample: OpenMP over this rank's CPU share (the lease's
    threads), then the same sample on ONE core, so the figure can be read per core.

    The sample (the first rows of rank 0's shard) is fitted repeatedly until ~target_s seconds have passed."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    affinity = len(os.sched_getaffinity(0))
    omp_env = os.environ.get("OMP_NUM_THREADS")
    cores = int(omp_env or "0") or affinity
    cores = max(1, min(cores, affinity, 64))

    first = {}

    def timed(threads, sample, budget):
        os.environ["OMP_NUM_THREADS"] = str(threads)
        O.set_threads(threads)
        done, rounds, conv = 0, 0, 0
        t0 = time.perf_counter()
        while True:
            st, coef, ll, cnt = O.fit_batch(sample, p, d, q, I, smear=smear)
            if not first:                  # the oracle's results, for the parity check of the timed step
                first.update(status=st, coef=coef, ll=ll, n_eval=cnt[:, 0], n_grad=cnt[:, 1])
            done += len(sample)
            rounds += 1
            conv = int((st == 0).sum())
            if time.perf_counter() - t0 >= budget:
                break
        return done / (time.perf_counter() - t0), rounds, conv

    O.lib()
    rate, rounds, conv = timed(cores, series_host, target_s)
    oracle_rows = dict(first)
    one = series_host[: max(1, len(series_host) // 16)]
    rate1, rounds1, _ = timed(1, one, max(2.0, target_s / 3))
    os.environ["OMP_NUM_THREADS"] = str(cores)
    O.set_threads(cores)
    phys = physical_cores()
    return oracle_rows, {"value": rate, "unit": "series fitted/sec", "cores": cores, "kind": "port",
            "value_1core": rate1, "host_physical_cores": phys, "host_cpus": os.cpu_count(), "affinity_cpus": affinity,
            "projected_all_physical_cores": rate1 * phys if phys else None,
            "sample": f"{len(series_host)} synthetic series of the benchmark workload (first rows of rank 0's shard) "
                      f"fitted {rounds}x by the C restatement oracle/arima_oracle.c with {cores} OpenMP threads "
                      f"(OMP_NUM_THREADS={omp_env}: the lease's CPU share; {affinity} CPUs in this process's affinity, "
                      f"{os.cpu_count()} CPUs / {phys} physical cores on the host); {conv}/{len(series_host)} converged; "
                      f"value_1core: the first {len(one)} of them {rounds1}x on one thread; "
                      f"projected_all_physical_cores = value_1core x physical cores (linear, not measured); "
                      f"not the spark-ts JVM"}


def oracle_rows(series_host, p, d, q, I, smear, budget_s):
    """The CPU restatement's fits of the first rows of this rank's shard (the parity check of ranks that do not time
    a CPU baseline): chunks of rows until every row is fitted or about budget_s seconds have passed."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    affinity = len(os.sched_getaffinity(0))
    O.set_threads(max(1, min(int(os.environ.get("OMP_NUM_THREADS", "0") or "0") or affinity, affinity, 64)))
    parts = []
    t0 = time.perf_counter()
    step = 256
    for b in range(0, len(series_host), step):
        st, coef, ll, cnt = O.fit_batch(series_host[b:b + step], p, d, q, I, smear=smear)
        parts.append((st, coef, ll, cnt))
        if time.perf_counter() - t0 >= budget_s:
            break
    st, coef, ll, cnt = (np.concatenate([x[i] for x in parts]) for i in range(4))
    return dict(status=st, coef=coef, ll=ll, n_eval=cnt[:, 0], n_grad=cnt[:, 1])


def run_default_leg(args):
    """the drop-in as a caller gets it -- arima_fit_batch_device with the ABI's default options
    (no arima_set_option call: fit_pipeline 3, the default scheduler knobs) under the box's own GPU_MAX_HW_QUEUES, in a
    child process that runs to completion before this process touches the GPU. Returns its JSON line (or an error)."""
    env = dict(os.environ, SPARKTS_BENCH_DEFAULT_LEG="1")
    if _BOX_QUEUES is None:
        env.pop("GPU_MAX_HW_QUEUES", None)
    else:
        env["GPU_MAX_HW_QUEUES"] = _BOX_QUEUES
    env.pop("SPARKTS_OPTIONS", None)
    cmd = [sys.executable, os.path.abspath(__file__), "--default-leg-child", "--config", args.config,
           "--series", str(args.series), "--steps", "5", "--warmup", "1"]
    try:
        out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    for line in out.stderr.splitlines():
        log(line)
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    if out.returncode != 0 or not lines:
        return {"error": f"exit {out.returncode}", "stderr_tail": out.stderr[-400:]}
    return json.loads(lines[-1])


def default_leg_child(args):
    import torch
    import sparkts_amd._lib as L
    p, d, q, I, T, base, jitter = CONFIGS[args.config]
    N, k = args.series, p + q + I
    dev_id = int(os.environ.get("SPARKTS_DEVICE", "") or 0)
    dev = torch.device("cuda", dev_id)
    eng = L.Engine.get(dev_id)                  # no set_option: the ABI's defaults
    series = torch.empty((N, T), dtype=torch.float64, device=dev)
    eng.sample_device(series.data_ptr(), N, T, T, p, d, q, I, base, jitter, SEED, 0)
    # every call writes its own result buffers, as consecutive partitions of a mapSeries would (calls that share
    # buffers would be ordered by the library: tests/test_gpu_parity.py::test_pipelined_fits_that_share_buffers_...)
    outs = [dict(coef=torch.empty((N, k), dtype=torch.float64, device=dev),
                 ll=torch.empty(N, dtype=torch.float64, device=dev), status=torch.empty(N, dtype=torch.int32, device=dev),
                 n_eval=torch.empty(N, dtype=torch.int32, device=dev),
                 n_grad=torch.empty(N, dtype=torch.int32, device=dev),
                 flags=torch.empty(N, dtype=torch.uint8, device=dev)) for _ in range(args.warmup + args.steps)]
    calls = [0]

    def step():
        o = outs[calls[0] % len(outs)]
        calls[0] += 1
        eng.fit_batch_device(series.data_ptr(), N, T, T, p, d, q, I, o["coef"].data_ptr(), o["ll"].data_ptr(),
                             o["status"].data_ptr(), o["n_eval"].data_ptr(), o["n_grad"].data_ptr(),
                             o["flags"].data_ptr(), blocking=False)
    for _ in range(args.warmup):
        step()
        eng.synchronize()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.synchronize()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    st = eng.stats()
    print(json.dumps({
        "value": N * args.steps / dt, "unit": "series fitted/sec", "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "series": N,
        "options": {n: eng.get_option(n) for n in ("fit_pipeline", "merge_live", "express_blocks", "hr_grid")},
        "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES") or "unset (HIP default: 4)",
        "series_done": st["series_done"],
        "kernel_ms": {"difference": st["ms_difference"], "hr_init": st["ms_hr_init"], "cg_fit": st["ms_cg_fit"]},
        "source": "bench.py default leg: arima_fit_batch_device with the ABI's default options in a child process "
                  "that keeps the box's hardware-queue setting (VERDICT r4 item 4a)"}), flush=True)


def same_bits(a, b):
    """Per-row bitwise equality of two device tensors of the same shape (rows = series)."""
    import torch
    if a.dtype == torch.float64:
        a, b = a.view(torch.int64), b.view(torch.int64)
    eq = a == b
    return eq.reshape(eq.shape[0], -1).all(dim=1) if eq.dim() > 1 else eq


def outputs_match(x, y):
    """Series whose every output (coef, LL, status, n_eval, n_grad, flags) is bit-identical in x and y."""
    ok = None
    for k in ("coef", "ll", "status", "n_eval", "n_grad", "flags"):
        e = same_bits(x[k], y[k])
        ok = e if ok is None else ok & e
    return ok


def oracle_row_parity(res, exp):
    """Rows of the timed step bit-identical to the oracle (status, n_eval, n_grad exact; coef, LL and flags bit for
    bit where the fit returned normally, NaN coefficients where it failed): the count of matching rows."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    st = exp["status"]
    ok = (res["status"] == st) & (res["n_eval"] == exp["n_eval"]) & (res["n_grad"] == exp["n_grad"])
    good = st == 0
    cb = res["coef"].view(np.int64) == exp["coef"].view(np.int64)
    lb = res["ll"].view(np.int64) == exp["ll"].view(np.int64)
    p, q, I = exp["pqi"]
    fl = np.array([O.model_flags(exp["coef"][i], p, q, I) if good[i] else 0 for i in range(len(st))], dtype=np.uint8)
    ok &= np.where(good, cb.all(axis=1) & lb & (res["flags"] == fl), np.isnan(res["coef"]).all(axis=1))
    return int(ok.sum())


def end_to_end(eng, series, p, d, q, I, last, barrier, world, dist, max_over_ranks):
    """the same fit from the caller's (pageable) host memory through the blocking host entry
    point arima_fit_batch -- the rows uploaded chunk by chunk straight from pageable memory (host_copy_threads 0, the
    default: staging through pinned blocks measured no faster) while the fits of earlier chunks run, results back
    through pinned staging into the caller's arrays. Every rank runs it at once on its own
    shard (barrier, max over ranks), so at N > 1 the line carries the host DRAM / PCIe contention of N GPUs. One
    warm-up call on the first chunk sizes the staging buffers. The results must equal the device path's (the last
    timed step) bit for bit on every row."""
    import numpy as np
    host = series.cpu().numpy()
    eng.fit_batch(host[: 1 << 18], p, d, q, bool(I))
    barrier()
    t0 = time.perf_counter()
    r = eng.fit_batch(host, p, d, q, bool(I))
    dt = time.perf_counter() - t0
    barrier()
    dt_max = max_over_ranks(dt, dist if world > 1 else None)
    same = np.ones(len(host), dtype=bool)
    for k, v in r.items():
        ref = last[k].cpu().numpy()
        a, b = (v.view(np.int64), ref.view(np.int64)) if v.dtype == np.float64 else (v, ref)
        same &= (a == b).reshape(len(host), -1).all(axis=1)
    from sparkts_amd.sharding import parity_over_ranks
    par = parity_over_ranks(int(same.sum()), len(host), dist if world > 1 else None)
    total = len(host) * world
    return {"value": total / dt_max, "unit": "series fitted/sec", "seconds": dt_max, "series": total,
            "n_ranks": world, "bytes_in": int(host.nbytes) * world, "GBps_in": host.nbytes * world / dt_max / 1e9,
            "converged_fraction": float((r["status"] == 0).mean()),
            "bit_identical_to_device_path": par["every_rank_bit_identical"], "rows_compared": par["oracle_rows"],
            "rows_identical": par["bit_identical"],
            "options": {n: eng.get_option(n) for n in ("host_chunk", "host_pipeline", "host_copy_threads")},
            "path": "arima_fit_batch on every rank at once: pageable host N x T -> chunked uploads to HBM (over the "
                    "host_pipeline fit contexts) -> fused differencing / HR / CG fit -> pinned staging -> caller's "
                    "arrays; value = all ranks' series / the slowest rank's time"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default: 20 for c2/c3, 5 for c4, 2 for c5)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed warmup steps (default: 3; 1 for c5)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--series", type=int, default=0, help="series per GPU (weak scaling; 0: 1M, 10 000 for c1)")
    ap.add_argument("--total-series", type=int, default=0, help="fixed total series over all GPUs (strong scaling)")
    ap.add_argument("--smear", type=int, default=1, choices=[0, 1])
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU-baseline sample budget (0 = skip)")
    ap.add_argument("--grid-blocks", type=int, default=0)
    ap.add_argument("--pipeline", type=int, default=0,
                    help="fit contexts (0: 6, or 4 for c4, whose 1M x 4096 fit then stays one slice of free HBM)")
    ap.add_argument("--express-blocks", type=int, default=-1, help="express workgroups of the fit kernel (-1: CUs/16)")
    ap.add_argument("--e2e", type=int, default=1, choices=[0, 1])
    ap.add_argument("--default-leg", type=int, default=1, choices=[0, 1])
    ap.add_argument("--default-leg-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--device", type=int, default=None, help="GPU of every rank (default: LOCAL_RANK's)")
    ap.add_argument("--search-lanes", type=int, default=0,
                    help="c5: concurrent search lanes (0: 12; 8 / 10 / 12 / 16 / 24 lanes: 18.1 / 20.3 / 21.3 / 19.5 / "
                         "18.2 k series/s at 262 144, profiles/r04/w_lanes, v_cfg)")
    ap.add_argument("--dry-run", action="store_true")
    args = ap.parse_args()
    if args.device is not None:
        os.environ["SPARKTS_DEVICE"] = str(args.device)
    if args.series <= 0:
        args.series = DEFAULT_SERIES.get(args.config, 1 << 20)
    if args.default_leg_child:
        return default_leg_child(args)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))

    import numpy as np
    import torch
    import torch.distributed as dist

    from sparkts_amd.sharding import max_over_ranks, shard_range, weak_scaling_range

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev_id = int(os.environ["SPARKTS_DEVICE"]) if os.environ.get("SPARKTS_DEVICE", "") != "" else local
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        if not args.dry_run:
            torch.cuda.set_device(dev_id)
        # the data path has no collective; gloo (CPU) carries only the timing barrier and max-reduction. gloo's C++
        # side prints its connection report to stdout; it goes to stderr here so rank 0's JSON line stays the only
        # stdout line a driver has to parse
        sys.stdout.flush()
        saved_fd = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved_fd, 1)
            os.close(saved_fd)

    p, d, q, I, T, base, jitter = CONFIGS[args.config]
    if args.steps is None:                  # enough steps that the pipeline's fill is amortised (C2: 3 steps read
        args.steps = {"c4": 5, "c5": 2, "af": 1}.get(args.config, 20)   # 9.35 M series/s, 20 steps 11.0, profiles/r04/zz_check)
    if args.warmup is None:
        args.warmup = 1 if args.config in ("c5", "af") else 3
    if args.pipeline <= 0:
        args.pipeline = 4 if args.config == "c4" else 6
    if args.config == "c5" and not args.total_series:
        args.total_series = 1 << 20                 # configs[4]: 1M series over the node's GPUs
    if args.total_series:
        first, last = shard_range(args.total_series, rank, world)     # strong scaling: fixed total
        scaling = "strong"
    else:
        first, last = weak_scaling_range(args.series, rank)          # weak scaling: fixed per GPU
        scaling = "weak"
    N = last - first
    total_series = args.total_series or args.series * world
    k = p + q + I

    def barrier():
        if world > 1:
            dist.barrier()

    if args.dry_run:
        barrier()
        from sparkts_amd.sharding import gather_results
        shards = gather_results([np.array([[first, last]], dtype=np.int64)], dist if world > 1 else None)[0].tolist()
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "scaling": scaling, "total_series": total_series,
                              "shards": shards}), flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    # the drop-in as a caller gets it: ABI defaults in a child process that keeps the box's
    # hardware-queue setting, run to completion BEFORE this process touches the GPU
    default_leg = None
    if args.config == "c2" and world == 1 and args.default_leg:
        default_leg = run_default_leg(args)
    import sparkts_amd._lib as L
    dev = torch.device("cuda", dev_id)
    eng = L.Engine.get(dev_id)
    eng.set_option("smear", args.smear)
    eng.set_option("fit_pipeline", args.pipeline)
    eng.set_option("express_blocks", args.express_blocks)
    if args.grid_blocks:
        eng.set_option("grid_blocks", args.grid_blocks)
    if args.config == "c5":
        eng.set_option("search_lanes", args.search_lanes or 12)

    series = torch.empty((N, T), dtype=torch.float64, device=dev)
    eng.sample_device(series.data_ptr(), N, T, T, p, d, q, I, base, jitter, SEED, first)
    if args.config == "c5":
        return run_c5(args, eng, series, N, T, total_series, world, rank, dev, barrier, dist, max_over_ranks, scaling)
    if args.config == "af":
        return run_af(args, eng, series, N, T, total_series, world, rank, dev, barrier, dist, max_over_ranks, scaling)
    # one output set per fit context: pipelined steps never write the same buffers concurrently
    outs = [dict(coef=torch.empty((N, k), dtype=torch.float64, device=dev),
                 ll=torch.empty(N, dtype=torch.float64, device=dev),
                 status=torch.empty(N, dtype=torch.int32, device=dev),
                 n_eval=torch.empty(N, dtype=torch.int32, device=dev),
                 n_grad=torch.empty(N, dtype=torch.int32, device=dev),
                 flags=torch.empty(N, dtype=torch.uint8, device=dev)) for _ in range(max(1, args.pipeline))]
    torch.cuda.synchronize(dev)
    calls = [0]

    def step():
        # asynchronous: enqueues difference -> HR init -> CG fit on the next fit context's stream and returns
        o = outs[calls[0] % len(outs)]
        calls[0] += 1
        eng.fit_batch_device(series.data_ptr(), N, T, T, p, d, q, I, o["coef"].data_ptr(), o["ll"].data_ptr(),
                             o["status"].data_ptr(), o["n_eval"].data_ptr(), o["n_grad"].data_ptr(),
                             o["flags"].data_ptr(), blocking=False)

    for i in range(args.warmup):
        t0 = time.perf_counter()
        step()
        eng.synchronize()
        s = eng.stats()
        log(f"[rank {rank}] warmup {i}: {time.perf_counter() - t0:.3f} s (cg {s['ms_cg_fit']:.1f} ms)")
    barrier()
    eng.synchronize()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    eng.synchronize()
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dist if world > 1 else None)
    s0 = eng.stats()                      # the last timed step
    if s0["series_done"] != N:            # every series of the step must have a written result
        raise SystemExit(f"bench.py: the last step wrote {s0['series_done']} of {N} results (fault {s0['fault']})")
    log(f"[rank {rank}] {args.steps} steps in {elapsed:.3f} s; last step: difference {s0['ms_difference']:.1f} ms, "
        f"hr {s0['ms_hr_init']:.1f} ms, cg {s0['ms_cg_fit']:.1f} ms")

    st_h = outs[(calls[0] - 1) % len(outs)]["status"].cpu().numpy()
    conv = float((st_h == 0).mean()) if N else 1.0
    n = T - d
    M = max(p, q)
    S = n - M
    ff = 2 * (p + q) + 4
    fg = ff + 2 * k * q + 1 + p + q + 2 * k

    def cg_flops(st):
        # U distinct objective points that needed a pass (bulk objective passes, objective requests
        # served by gradient passes, express objective passes, speculative points the optimizer used), G gradient
        # passes (without those riders)
        U = st["f_passes"] + st["ride_passes"] + st["express_f_passes"] + st["spec_hits"]
        G = st["g_passes"] - st["ride_passes"] + st["express_g_passes"]
        return U * S * ff + G * S * fg, U, G

    flops_step, U, G = cg_flops(s0)
    # the last timed step's outputs, kept for the parity checks below (the isolated step may reuse its buffers)
    last = {k: v.clone() for k, v in outs[(calls[0] - 1) % len(outs)].items()}
    # the dominant kernel's own launch duration: steps alone on the GPU (fit_pipeline 1), HIP events; the median of
    # ISO_STEPS launches (one launch alone once read 224 vs 134-142 ms in the warmups: profiles/r06/q_fuse)
    eng.set_option("fit_pipeline", 1)
    iso_ms, s1 = [], None
    for _ in range(ISO_STEPS):
        step()
        eng.synchronize()
        s1 = eng.stats()
        if s1["series_done"] != N:
            raise SystemExit(f"bench.py: the isolated step wrote {s1['series_done']} of {N} results")
        iso_ms.append(s1["ms_cg_fit"])
    eng.set_option("fit_pipeline", args.pipeline)
    # parity of the configuration that was timed: the last pipelined step against the isolated step,
    # every series, bit for bit (max over ranks of the mismatching series)
    iso = outs[(calls[0] - 1) % len(outs)]
    iso_mismatch = int(max_over_ranks(float(N - int(outputs_match(last, iso).sum().item())),
                                      dist if world > 1 else None))
    if iso_mismatch:
        log(f"[rank {rank}] PARITY: {iso_mismatch} series of the timed step differ from the isolated step")
    flops_iso, _, _ = cg_flops(s1)
    cg_ms = sorted(iso_ms)[len(iso_ms) // 2]
    achieved_tf = flops_iso / (cg_ms * 1e-3) / 1e12 if cg_ms > 0 else 0.0
    step_tf = flops_step / (elapsed / args.steps) / 1e12
    wave_passes = s0["wave_f_passes"] + s0["wave_g_passes"] + s0["wave_multi_passes"]
    served = s0["f_passes"] + s0["g_passes"]
    lane_util = served / (64.0 * wave_passes) if wave_passes else None
    # HBM bytes the fit kernel streams by construction: one series row per served lane-pass
    passes_bytes = (served + s0["express_series"]) * n * 8.0

    # oracle parity of the timed step on EVERY rank: each rank fits the first rows of its own shard
    # with the CPU restatement (bounded by --cpu-seconds) and the verdicts meet in gloo min / sum reductions
    cpu = None
    rows_checked, rows_ok = 0, 0
    if args.cpu_seconds > 0 and N > 0:
        cap = 1024 if args.config == "c4" else 4096
        host = series[: min(N, cap)].cpu().numpy()
        if world == 1:
            exp, cpu = cpu_baseline(host, p, d, q, I, args.smear, args.cpu_seconds)
        else:
            exp = oracle_rows(host, p, d, q, I, args.smear, args.cpu_seconds)
        rows_checked = len(exp["status"])
        res = {k_: v[:rows_checked].cpu().numpy() for k_, v in last.items()}
        exp["pqi"] = (p, q, int(I))
        rows_ok = oracle_row_parity(res, exp)
        if rows_ok != rows_checked:
            log(f"[rank {rank}] PARITY: {rows_checked - rows_ok} of {rows_checked} oracle rows differ from the timed step")
    from sparkts_amd.sharding import parity_over_ranks
    node_parity = parity_over_ranks(rows_ok, rows_checked, dist if world > 1 else None)
    # the drop-in's own path from host memory, every rank at once
    e2e = end_to_end(eng, series, p, d, q, I, last, barrier, world, dist, max_over_ranks) if args.e2e else None

    if rank == 0:
        sha = build_sha()
        # the record key names the fit kernel and any non-default engine options too: a record of another variant
        # never stands for this run's kernel
        pmc, pmc_key = pmc_traffic({"series": N, "T": T, "p": p, "d": d, "q": q, "I": int(I), "smear": args.smear,
                                    "fit_kernel": 0,
                                    "options": os.environ.get("SPARKTS_OPTIONS", "")}, sha)
        result = {
            "metric": METRICS.get(args.config, f"series fitted/sec, {args.config}"),
            "value": total_series * args.steps / elapsed,
            "unit": "series fitted/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic: ARIMAModel.sample semantics on device, seed {SEED}, coef jitter +-{jitter}",
            "config": {"workload": f"ARIMA({p},{d},{q}){'+c' if I else ''} css-cgd, "
                                   + (f"{total_series} series total over {world} GPU(s)" if scaling == "strong"
                                      else f"{N} series x {T} pts per GPU")
                                   + {"c1": " (BASELINE.json configs[0])", "c4": " (BASELINE.json configs[3])"}.get(
                                       args.config, " (BASELINE.json configs[1]/[2])"),
                       "series_per_gpu": N, "series_total": total_series, "series_len": T,
                       "parallelism": f"series-sharded x{world}, no collective",
                       "breeze_overlap": "smear" if args.smear else "shift",
                       "fit_kernel": "k_cg_fit (LDS slots, 1 wave/SIMD)", "fit_pipeline": args.pipeline,
                       "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                       "converged_fraction": conv, "series_done": s0["series_done"],
                       "mean_n_eval": s0["n_eval"] / max(N, 1), "mean_n_grad": s0["n_grad"] / max(N, 1),
                       "lane_f_passes_per_series": s0["f_passes"] / max(N, 1),
                       "lane_g_passes_per_series": s0["g_passes"] / max(N, 1),
                       "kernel_ms": {"difference": s0["ms_difference"], "hr_init": s0["ms_hr_init"],
                                     "cg_fit": s0["ms_cg_fit"]}},
            "roofline": {"bound": "fp64-valu", "kernel": "k_cg_fit", "achieved": achieved_tf,
                         "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": achieved_tf / FP64_PEAK_TFLOPS,
                         "launch_ms": cg_ms, "launch_ms_each": iso_ms,
                         "achieved_source": "algorithmic flops of one k_cg_fit launch (SURVEY.md 8(d): U*S*(2(p+q)+4) "
                                            "+ G*S*(2(p+q)+4+2kq+1+p+q+2k), U and G counted by the kernel) / that "
                                            "launch's HIP-event duration, the launch alone on the GPU (the median "
                                            "of three extra steps at fit_pipeline 1 after the timed region)",
                         "U_per_series": U / max(N, 1), "G_per_series": G / max(N, 1),
                         "achieved_pipelined": step_tf,
                         "achieved_pipelined_source": "the timed steps' k_cg_fit algorithmic flops / ms_per_step "
                                                      "(steady state, launches overlapping)",
                         "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                         "traffic_unit": "bytes/launch (HBM read+write, rocprofv3 PMC)",
                         "traffic_source": pmc["source"] if pmc else
                         "no rocprofv3 PMC record of this workload for this build (library sha256 " + str(sha)[:16] + ")",
                         "build_sha": sha,
                         "traffic_matched_on": pmc_key,
                         "hbm_GBps_pmc": (pmc["hbm_bytes_per_launch"] / (cg_ms * 1e-3) / 1e9) if pmc and cg_ms else None,
                         "hbm_frac_pmc": (pmc["hbm_bytes_per_launch"] / (cg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS)
                         if pmc and cg_ms else None,
                         "valu_busy_pmc": pmc.get("valu_busy") if pmc else None,
                         "wait_frac_pmc": pmc.get("wait_frac") if pmc else None,
                         "traffic_model_GBps": passes_bytes / (cg_ms * 1e-3) / 1e9 if cg_ms else None,
                         "hbm_peak_GBps": HBM_PEAK_GBS,
                         "lane_utilisation": lane_util,
                         "objective_chain_use": (s0["spec_chains"] / s0["wave_chains"]) if s0.get("wave_chains") else None,
                         "low_util_wave_passes": s0.get("low_util_passes"),
                         "express_pit_passes": {"f": s0.get("express_pit_passes"), "g": s0.get("express_pit_g_passes"),
                                                "sweeps": s0.get("express_pit_sweeps")},
                         "spec_hits_per_series": s0["spec_hits"] / max(N, 1),
                         "ride_passes_per_series": s0["ride_passes"] / max(N, 1),
                         "express_series": s0["express_series"],
                         "merge": {"series": s0.get("merge_series"), "waves": s0.get("merge_waves")},
                         "wave_passes": {"f": s0["wave_f_passes"], "g": s0["wave_g_passes"],
                                         "multi": s0["wave_multi_passes"]}},
            "cpu_baseline": cpu,
        }
        if default_leg is not None:
            result["default_config"] = default_leg
        if e2e is not None:
            result["end_to_end_host"] = e2e
        parity = {"configuration": f"the last timed step: fit_pipeline {args.pipeline} on GPU_MAX_HW_QUEUES="
                                   f"{os.environ.get('GPU_MAX_HW_QUEUES')}",
                  "vs_isolated": iso_mismatch == 0, "isolated_mismatch_series": iso_mismatch,
                  "isolated_compared_series": total_series,
                  "oracle_rows": node_parity["oracle_rows"], "bit_identical": node_parity["bit_identical"],
                  "ranks_checked": node_parity["ranks"],
                  "every_rank_bit_identical": node_parity["every_rank_bit_identical"],
                  "min_rank_fraction": node_parity["min_rank_fraction"],
                  "oracle_source": "oracle/arima_oracle.c on the first rows of every rank's shard (rank 0: the "
                                   "cpu_baseline sample), gloo sum / min over ranks"}
        result["parity"] = parity
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def run_c5(args, eng, series, N, T, total_series, world, rank, dev, barrier, dist, max_over_ranks, scaling):
    """configs[4]: a step = the full (d <= 2, p <= 5, q <= 5, +-c) order search (216 fits per series, min approxAIC
    among stationary and invertible fits, ARIMA.scala:826-830 / :342) over this rank's shard, device-resident."""
    import torch
    order = torch.empty((max(N, 1), 4), dtype=torch.int32, device=dev)
    coef = torch.empty((max(N, 1), 11), dtype=torch.float64, device=dev)
    aic = torch.empty(max(N, 1), dtype=torch.float64, device=dev)

    def step():                            # a full-size search runs for minutes
        eng.order_search_device(series.data_ptr(), N, T, T, 5, 2, 5, 2, order.data_ptr(), coef.data_ptr(),
                                aic.data_ptr(), blocking=False)
        with heartbeat(f"[rank {rank}] searching"):
            eng.synchronize()

    for i in range(args.warmup):
        step()
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
        log(f"[rank {rank}] search step {i} done at {time.perf_counter() - t0:.1f} s")
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dist if world > 1 else None)
    st = eng.stats()                      # the last search: counter sums and algorithmic flops over its 216 fits
    o = order[:N].cpu().numpy()
    found = float((o[:, 0] >= 0).mean()) if N else 1.0
    if rank == 0:
        search_ms = st["ms_total"]
        achieved = st["flops"] / (search_ms * 1e-3) / 1e12 if search_ms > 0 else 0.0
        roofline = {"bound": "fp64-valu", "kernel": "k_cg_fit (+ k_hr_init, k_ar_fit) over the 216 grid fits",
                    "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": achieved / FP64_PEAK_TFLOPS, "launch_ms": search_ms,
                    "achieved_source": "algorithmic flops of every grid fit of the last search step (SURVEY.md 8(d): "
                                       "U*S*ff + G*S*fg + W_HR per fit, U and G from each fit kernel's own counters, "
                                       "summed on the device per search lane) / the search's HIP-event duration",
                    "flops_per_step": st["flops"], "fits": st["n_series"],
                    "U_per_fit": (st["f_passes"] + st["ride_passes"] + st["express_f_passes"] + st["spec_hits"])
                    / max(st["n_series"], 1),
                    "G_per_fit": (st["g_passes"] - st["ride_passes"] + st["express_g_passes"]) / max(st["n_series"], 1),
                    "mean_n_eval_per_fit": st["n_eval"] / max(st["n_series"], 1),
                    "series_done": st["series_done"], "express_series": st["express_series"],
                    "express_pit_passes": st["express_pit_passes"],
                    "express_wave_passes": st["express_f_passes"] + st["express_g_passes"],
                    "bulk_wave_passes": st["wave_f_passes"] + st["wave_g_passes"] + st["wave_multi_passes"],
                    "merge": {"series": st.get("merge_series"), "waves": st.get("merge_waves")}}
        sha = build_sha()
        pmc, pmc_key = pmc_traffic({"config": "c5", "series": N, "T": T, "smear": args.smear,
                                    "options": os.environ.get("SPARKTS_OPTIONS", "")}, sha)
        roofline.update({
            "traffic": pmc["hbm_bytes_per_step"] if pmc else None,
            "traffic_unit": "bytes per search step (HBM read+write of every kernel of the 216 grid fits, rocprofv3 PMC)",
            "traffic_source": pmc["source"] if pmc else
            "no rocprofv3 PMC record of this workload for this build (library sha256 " + str(sha)[:16] + ")",
            "build_sha": sha, "traffic_matched_on": pmc_key,
            "hbm_GBps_pmc": (pmc["hbm_bytes_per_step"] / (search_ms * 1e-3) / 1e9) if pmc and search_ms else None,
            "hbm_frac_pmc": (pmc["hbm_bytes_per_step"] / (search_ms * 1e-3) / 1e9 / HBM_PEAK_GBS)
            if pmc and search_ms else None})
        cpu, parity = None, None
        if world == 1 and args.cpu_seconds > 0:
            cpu, parity = c5_cpu_baseline(series, o, coef, aic, T, args.smear)
        sel = {}
        for r in o[: min(N, 65536)]:
            key = f"({r[0]},{r[1]},{r[2]}){'+c' if r[3] == 1 else ''}" if r[0] >= 0 else "none"
            sel[key] = sel.get(key, 0) + 1
        print(json.dumps({
            "metric": "series searched/sec, ARIMA order search p,q<=5 d<=2 +-c (216 CSS-CGD fits/series, min approxAIC), "
                      "x 1024 pts",
            "value": total_series * args.steps / elapsed, "unit": "series searched/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "f64",
            "data": f"synthetic C2-shaped series (ARIMAModel.sample semantics on device, seed {SEED})",
            "config": {"workload": f"order search over {total_series} series x {T} pts "
                                   f"({'total over ' + str(world) + ' GPU(s)' if scaling == 'strong' else 'per GPU'};"
                                   f" BASELINE.json configs[4])",
                       "series_per_gpu": N, "series_total": total_series, "fits_per_series": 216,
                       "fits_per_sec": total_series * 216 * args.steps / elapsed,
                       "search_lanes": eng.get_option("search_lanes"),
                       "search_express_cus": eng.get_option("search_express_blocks"),
                       "merge_live": eng.get_option("merge_live"),
                       "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                       "found_fraction": found, "selected_orders_top":
                           dict(sorted(sel.items(), key=lambda kv: -kv[1])[:6]),
                       "parallelism": f"series-sharded x{world}, no collective"},
            "roofline": roofline,
            "roofline_note": "per grid point (flops, evaluations, MaxEval fraction): tools/grid_profile.py",
            "parity": parity,
            "cpu_baseline": cpu}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def run_af(args, eng, series, N, T, total_series, world, rank, dev, barrier, dist, max_over_ranks, scaling):
    """ARIMA.autoFit per series (ARIMA.scala:280-375): a step = arima_autofit_batch_device over
    this rank's shard, device-resident; parity = every rank's first rows against oracle.autofit, bit for bit."""
    import numpy as np
    import torch
    from sparkts_amd.sharding import parity_over_ranks
    out = dict(order=torch.empty((max(N, 1), 4), dtype=torch.int32, device=dev),
               coef=torch.empty((max(N, 1), 11), dtype=torch.float64, device=dev),
               aic=torch.empty(max(N, 1), dtype=torch.float64, device=dev),
               status=torch.empty(max(N, 1), dtype=torch.int32, device=dev),
               n_fits=torch.empty(max(N, 1), dtype=torch.int32, device=dev))

    def step():
        with heartbeat(f"[rank {rank}] auto-fitting"):
            eng.autofit_device(series.data_ptr(), N, T, T, 5, 2, 5, out["order"].data_ptr(), out["coef"].data_ptr(),
                               out["aic"].data_ptr(), out["status"].data_ptr(), out["n_fits"].data_ptr(),
                               blocking=True)
    for _ in range(args.warmup):
        step()
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
        log(f"[rank {rank}] autofit step {i} done at {time.perf_counter() - t0:.2f} s")
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dist if world > 1 else None)
    res = {k: v[:N].cpu().numpy() for k, v in out.items()}
    fits = int(res["n_fits"].sum())
    cpu, rows_checked, rows_ok = None, 0, 0
    if args.cpu_seconds > 0 and N > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        affinity = len(os.sched_getaffinity(0))
        host = series[: min(N, 256)].cpu().numpy()
        t1 = time.perf_counter()
        exp = []
        for row in host:                                 # the restatement, one series at a time (bounded)
            exp.append(O.autofit(row, 5, 2, 5))
            if time.perf_counter() - t1 > args.cpu_seconds:
                break
        dt = time.perf_counter() - t1
        rows_checked = len(exp)
        for i, e in enumerate(exp):
            coef_same = np.array_equal(res["coef"][i].view(np.int64), e["coef"].view(np.int64)) or \
                (np.isnan(res["coef"][i]).all() and np.isnan(e["coef"]).all())
            same = (res["status"][i] == e["status"] and tuple(res["order"][i]) == tuple(e["order"]) and
                    res["n_fits"][i] == e["n_fits"] and coef_same and
                    res["aic"][i].view(np.int64) == np.float64(e["aic"]).view(np.int64))
            rows_ok += int(bool(same))
        if world == 1:
            phys = physical_cores()
            cpu = {"value": rows_checked / dt, "unit": "series auto-fitted/sec", "cores": 1, "kind": "port",
                   "host_physical_cores": phys, "projected_all_physical_cores": rows_checked / dt * phys if phys else None,
                   "sample": f"the first {rows_checked} series of the shard through oracle.autofit (C restatement fits "
                             f"and KPSS, the walk in Python) on one thread; not the spark-ts JVM"}
    par = parity_over_ranks(rows_ok, rows_checked, dist if world > 1 else None)
    if rank == 0:
        st = res["status"]
        sel = {}
        for r in res["order"][: min(N, 65536)]:
            key = f"({r[0]},{r[1]},{r[2]}){'+c' if r[3] == 1 else ''}" if r[0] >= 0 else "none"
            sel[key] = sel.get(key, 0) + 1
        print(json.dumps({
            "metric": "series auto-fitted/sec, ARIMA.autoFit (KPSS d <= 2, stepwise p, q <= 5, css-cgd), x 1024 pts",
            "value": total_series * args.steps / elapsed, "unit": "series auto-fitted/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "f64",
            "data": f"synthetic C2-shaped series (ARIMAModel.sample semantics on device, seed {SEED})",
            "config": {"workload": f"autoFit over {N} series x {T} pts per GPU (SURVEY.md 8(f) row 2)",
                       "series_per_gpu": N, "series_total": total_series, "fits_per_series": fits / max(N, 1),
                       "fits_per_sec": fits * world * args.steps / elapsed,
                       "status_counts": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
                       "selected_orders_top": dict(sorted(sel.items(), key=lambda kv: -kv[1])[:6]),
                       "parallelism": f"series-sharded x{world}, no collective"},
            "roofline": None,
            "roofline_note": "autoFit's fits are k_cg_fit launches (roofline: the C2 line); the KPSS passes and the "
                             "walk's gathers are HBM streams",
            "parity": {"oracle_rows": par["oracle_rows"], "bit_identical": par["bit_identical"],
                       "every_rank_bit_identical": par["every_rank_bit_identical"], "ranks_checked": par["ranks"],
                       "checked": "status, (p, d, q, intercept), n_fits, coefficients and approxAIC, bit for bit"},
            "cpu_baseline": cpu}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def c5_cpu_baseline(series, order, coef, aic, T, smear):
    """C5 on the CPU restatement (oracle/, kind "port"): oracle.order_search over the first rows of the shard with
    OpenMP on the lease's CPU share, then fewer rows on one core; and the parity of those rows' selections (order,
    approxAIC and coefficients bit for bit) with the GPU search's."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    affinity = len(os.sched_getaffinity(0))
    cores = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "0") or "0") or affinity, affinity, 64))
    O.lib()
    rows = min(series.shape[0], 128)
    host = series[:rows].cpu().numpy()
    O.set_threads(cores)
    t0 = time.perf_counter()
    o_o, c_o, a_o = O.order_search(host, 5, 2, 5, 2, smear=smear)
    rate = rows / (time.perf_counter() - t0)
    one = host[:4]
    O.set_threads(1)
    t0 = time.perf_counter()
    O.order_search(one, 5, 2, 5, 2, smear=smear)
    rate1 = len(one) / (time.perf_counter() - t0)
    O.set_threads(cores)
    g_o = order[:rows]
    g_c = coef[:rows].cpu().numpy()
    g_a = aic[:rows].cpu().numpy()
    same = (g_o == o_o).all(axis=1) & (g_a.view(np.int64) == a_o.view(np.int64)) & \
        ((g_c.view(np.int64) == c_o.view(np.int64)) | (np.isnan(g_c) & np.isnan(c_o))).all(axis=1)
    phys = physical_cores()
    cpu = {"value": rate, "unit": "series searched/sec", "cores": cores, "kind": "port", "value_1core": rate1,
           "host_physical_cores": phys, "projected_all_physical_cores": rate1 * phys if phys else None,
           "sample": f"the first {rows} series of the shard searched over the full (5, 2, 5, +-c) grid by "
                     f"oracle.order_search (C restatement fits, {cores} OpenMP threads); value_1core: the first "
                     f"{len(one)} on one thread; not the spark-ts JVM"}
    parity = {"oracle_rows": rows, "bit_identical": int(same.sum()),
              "checked": "selected (p, d, q, intercept), approxAIC and coefficients, bit for bit"}
    return cpu, parity


if __name__ == "__main__":
    main()
