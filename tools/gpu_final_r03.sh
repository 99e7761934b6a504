#!/bin/bash
# Final round-3 GPU session of the committed build: GPU parity tests, smoke, the driver's headline command, and the
# C2 rocprofv3 passes (kernel trace + PMC) that bench.py's roofline.traffic is matched to (tools/pmc_traffic_c2.json).
# Every GPU step has its own time limit; the chain stops at the first failure. Run ON the GPU box from the repo root.
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${FINAL_OUT:-r03/final2}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err &&
OUT=$OUT/prof bash tools/profile.sh > $OUT/profile.log 2>&1
