#!/bin/bash
# Rounds fit (fit_kernel 2) on the GPU: parity subsets with forced rounds (no early hand-off), then C2 throughput.
# DEV=<tag>: use spark-timeseries_amd/libsparkts_arima_dev_<tag>.so (ARIMA(2,.,2) smear only: TESTK restricts tests)
set -o pipefail
OUT=gpurun_out/${TAG:-r03/rounds}
mkdir -p $OUT
if [ -n "$DEV" ]; then export SPARKTS_ARIMA_LIB=$PWD/spark-timeseries_amd/libsparkts_arima_dev_${DEV}.so; fi
K=${TESTK:-c2_batch or full_size}
for opt in "fit_kernel=2,rounds_tail=0,rounds_max=400" "fit_kernel=2,rounds_tail=0,rounds_max=12"; do
  SPARKTS_OPTIONS=$opt timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" >> $OUT/pytest.log 2>&1 || { echo "tests failed: $opt"; exit 1; }
  echo "tests ok: $opt"
done
for v in ${BENCHV:-2 0}; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --e2e 0 --cpu-seconds 0 --fit-kernel $v > $OUT/bench_k$v.json 2>> $OUT/bench.err || exit 1
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --pipeline 1 --e2e 0 --cpu-seconds 0 --fit-kernel $v > $OUT/bench_k${v}_p1.json 2>> $OUT/bench.err || exit 1
done
echo bench ok
