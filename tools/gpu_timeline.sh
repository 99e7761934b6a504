#!/bin/bash
# kernel timeline of the pipelined bench (rocprofv3 kernel trace only; run from the repo root via gpurun)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-timeline}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --steps 6 --warmup 1 --pipeline ${P:-3} --e2e 0 --cpu-seconds 0 > $OUT/bench.json 2> $OUT/bench.err
