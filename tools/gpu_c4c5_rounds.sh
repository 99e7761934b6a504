#!/bin/bash
# fit_kernel 0 vs 2 on C4 (ARIMA(5,1,5)+c, T = 4096) and C5 (order search), full library
set -o pipefail
OUT=gpurun_out/${TAG:-r03/c4c5}
mkdir -p $OUT
for v in 2 0; do
  timeout -k 10 300 python bench.py --config c4 --series ${C4SER:-131072} --steps 2 --warmup 1 --pipeline 1 --e2e 0 --cpu-seconds 0 --fit-kernel $v > $OUT/c4_k${v}_p1.json 2>> $OUT/err.log || exit 1
  echo "c4 p1 $v ok"
  timeout -k 10 300 python bench.py --config c4 --series ${C4SER:-131072} --steps 4 --warmup 1 --pipeline 3 --e2e 0 --cpu-seconds 0 --fit-kernel $v > $OUT/c4_k${v}_p3.json 2>> $OUT/err.log || exit 1
  echo "c4 p3 $v ok"
done
for v in 2 0; do
  timeout -k 10 400 python bench.py --config c5 --total-series ${C5SER:-65536} --steps 1 --warmup 0 --fit-kernel $v > $OUT/c5_k$v.json 2>> $OUT/err.log || exit 1
  echo "c5 $v ok"
done
