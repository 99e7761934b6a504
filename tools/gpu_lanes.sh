#!/bin/bash
# C5 order search at 131 072 series (one GPU's share of configs[4]): search lanes x hardware queues
set -o pipefail
OUT=gpurun_out/${TAG:-r03/lanes}
mkdir -p $OUT
for lq in "8 8" "12 16" "16 16" "16 24"; do
  set -- $lq
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 400 python bench.py --config c5 --total-series 131072 --steps 1 --warmup 0 --search-lanes $1 > $OUT/c5_l$1_q$2.json 2>> $OUT/err.log || exit 1
  echo "l$1 q$2 ok"
done
