#!/bin/bash
# One GPU-box session (run from the repo root via gpurun): gpu parity tests, smoke, headline bench, rocprof passes.
# Every GPU step has its own time limit and the chain stops at the first failure.
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
bash tools/profile.sh > gpurun_out/profile.log 2>&1
