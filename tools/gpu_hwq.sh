#!/bin/bash
# hardware queues per process (GPU_MAX_HW_QUEUES, HIP default 4) vs concurrent streams: C5 search lanes, C2 contexts
set -o pipefail
OUT=gpurun_out/${TAG:-r03/hwq}
mkdir -p $OUT
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python bench.py --config c5 --total-series 65536 --steps 1 --warmup 0 > $OUT/c5_q$q.json 2>> $OUT/err.log || exit 1
  echo "c5 q$q ok"
done
for qp in "4 3" "8 3" "8 4" "8 6"; do
  set -- $qp
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 300 python bench.py --steps 12 --warmup 2 --pipeline $2 --e2e 0 --cpu-seconds 0 > $OUT/c2_q$1_p$2.json 2>> $OUT/err.log || exit 1
  echo "c2 q$1 p$2 ok"
done
