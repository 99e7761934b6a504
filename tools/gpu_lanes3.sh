#!/bin/bash
# C5 order search with more than 16 search lanes (kSearchMaxLanes 32): every grid point's time is its slowest
# series' serial chain (profiles/r03/b_c3_c5/grid_65536.jsonl), so more grid points in flight hide more of it.
# Run ON the GPU box from the repo root.
set -o pipefail
OUT=gpurun_out/${TAG:-r03/lanes3}
mkdir -p $OUT
for L in ${LANES:-16 24 32}; do
  GPU_MAX_HW_QUEUES=32 timeout -k 10 300 python bench.py --config c5 --total-series 131072 --steps 1 --warmup 0 \
      --search-lanes $L --cpu-seconds 0 --e2e 0 > $OUT/c5_131072_l${L}_q32.json 2>> $OUT/err.log || exit 1
  echo "131072 lanes $L ok"
done
for L in ${LANES262:-24 32}; do
  GPU_MAX_HW_QUEUES=32 timeout -k 10 400 python bench.py --config c5 --total-series 262144 --steps 1 --warmup 0 \
      --search-lanes $L --cpu-seconds 0 --e2e 0 > $OUT/c5_262144_l${L}_q32.json 2>> $OUT/err.log || exit 1
  echo "262144 lanes $L ok"
done
