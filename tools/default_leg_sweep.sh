#!/bin/bash
# The drop-in with the ABI's defaults (bench.py's default leg, box hardware queues) under option overrides:
# OPTS="fit_pipeline=1 fit_pipeline=3" (one SPARKTS_OPTIONS value per run; STEPS
# consecutive asynchronous calls, default 5). Run ON the GPU box from the repo root after tools/gpu_session.sh (same OUT).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05/${TAG:-s}
mkdir -p "$OUT"
for o in ${OPTS:-fit_pipeline=1}; do
    SPARKTS_BENCH_DEFAULT_LEG=1 SPARKTS_OPTIONS=$o timeout -k 10 200 python -u bench.py --default-leg-child \
        --config c2 --steps ${STEPS:-5} --warmup 1 > "$OUT/default_${o/=/}_s${STEPS:-5}.json" \
        2> "$OUT/default_${o/=/}_s${STEPS:-5}.err" || exit 1
done
