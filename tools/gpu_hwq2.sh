#!/bin/bash
set -o pipefail
OUT=gpurun_out/${TAG:-r03/hwq2}
mkdir -p $OUT
for qp in "8 5" "8 6" "8 8" "16 6" "16 8"; do
  set -- $qp
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 300 python bench.py --steps 20 --warmup 2 --pipeline $2 --e2e 0 --cpu-seconds 0 > $OUT/c2_q$1_p$2.json 2>> $OUT/err.log || exit 1
  echo "c2 q$1 p$2 ok"
done
for qp in "8 3" "8 4"; do
  set -- $qp
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 400 python bench.py --config c4 --series 1048576 --steps 4 --warmup 1 --pipeline $2 --e2e 0 --cpu-seconds 0 > $OUT/c4_q$1_p$2.json 2>> $OUT/err.log || exit 1
  echo "c4 q$1 p$2 ok"
done
