#!/bin/bash
# The drop-in with the ABI's defaults (bench.py's default leg, box hardware queues) by "call_slices" (0 = off, -1 = auto):
# run ON the GPU box from the repo root after tools/gpu_session.sh (same OUT).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05/${TAG:-s}
mkdir -p "$OUT"
for cs in ${SLICES:-1 2 3 4}; do
    SPARKTS_BENCH_DEFAULT_LEG=1 SPARKTS_OPTIONS=call_slices=$cs timeout -k 10 200 python -u bench.py --default-leg-child \
        --config c2 --steps 5 --warmup 1 > "$OUT/default_cs$cs.json" 2> "$OUT/default_cs$cs.err" || exit 1
done
