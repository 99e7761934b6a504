#!/bin/bash
# Kernel trace of the pipelined C2 bench (the timed configuration: 6 fit contexts on 8 hardware queues) for
# tools/pipe_overlap.py (run ON the GPU box from the repo root): how much of the span has a k_cg_fit running.
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/${TAG:-n_pipe}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --e2e 0 --default-leg 0 > $O/bench.json 2> $O/bench.err
