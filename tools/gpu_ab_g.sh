#!/bin/bash
# A/B of the fit kernels: full GPU parity suite with k_cg_fit_g (SPARKTS_FIT_KERNEL=1), then C2 throughput of both
set -o pipefail
OUT=gpurun_out/${TAG:-r03/g}
mkdir -p $OUT
if [ -n "$DEV" ]; then export SPARKTS_ARIMA_LIB=$PWD/spark-timeseries_amd/libsparkts_arima_dev_${DEV}.so; fi
SPARKTS_FIT_KERNEL=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > $OUT/pytest_g.log 2>&1 || exit 1
echo tests ok
for v in 1 0 1 0; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --e2e 0 --cpu-seconds 0 --fit-kernel $v > $OUT/bench_k${v}_$RANDOM.json 2>> $OUT/bench.err || exit 1
done
echo bench ok
