#!/bin/bash
# cost-aware pass choice (STS_GW_PCT dev builds): parity subset, then C4 131k and C2 1M
set -o pipefail
OUT=gpurun_out/${TAG:-r03/gw}
mkdir -p $OUT
for v in ${C4V:-c4gw0 c4gw200 c4gw400}; do
  export SPARKTS_ARIMA_LIB=$PWD/spark-timeseries_amd/libsparkts_arima_dev_$v.so
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "c4_T4096 or c4_515" >> $OUT/pytest.log 2>&1 || { echo "tests $v failed"; exit 1; }
  timeout -k 10 300 python bench.py --config c4 --series 131072 --steps 2 --warmup 1 --pipeline 1 --e2e 0 --cpu-seconds 0 > $OUT/${v}_p1.json 2>> $OUT/err.log || exit 1
  timeout -k 10 300 python bench.py --config c4 --series 131072 --steps 4 --warmup 1 --e2e 0 --cpu-seconds 0 > $OUT/${v}.json 2>> $OUT/err.log || exit 1
  echo "$v ok"
done
for v in ${C2V:-c2gw0 c2gw200 c2gw300}; do
  export SPARKTS_ARIMA_LIB=$PWD/spark-timeseries_amd/libsparkts_arima_dev_$v.so
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "c2_batch" >> $OUT/pytest.log 2>&1 || { echo "tests $v failed"; exit 1; }
  timeout -k 10 300 python bench.py --steps 12 --warmup 2 --e2e 0 --cpu-seconds 0 > $OUT/${v}.json 2>> $OUT/err.log || exit 1
  echo "$v ok"
done
