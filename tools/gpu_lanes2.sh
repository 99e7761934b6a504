#!/bin/bash
set -o pipefail
OUT=gpurun_out/${TAG:-r03/lanes2}
mkdir -p $OUT
GPU_MAX_HW_QUEUES=32 timeout -k 10 400 python bench.py --config c5 --total-series 131072 --steps 1 --warmup 0 --search-lanes 16 > $OUT/c5_131072_l16_q32.json 2>> $OUT/err.log || exit 1
echo ok1
GPU_MAX_HW_QUEUES=24 timeout -k 10 500 python bench.py --config c5 --total-series 262144 --steps 1 --warmup 0 --search-lanes 16 > $OUT/c5_262144_l16_q24.json 2>> $OUT/err.log || exit 1
echo ok2
for q in 8 24; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 20 --warmup 2 --e2e 0 --cpu-seconds 0 > $OUT/c2_q$q.json 2>> $OUT/err.log || exit 1
  echo "c2 q$q ok"
done
