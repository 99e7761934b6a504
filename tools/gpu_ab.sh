#!/bin/bash
# A/B of dev-library variants on the pipelined C2 bench: LIBS="a b" ROUNDS=2 bash tools/gpu_ab.sh (run via gpurun)
set -o pipefail
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
for i in $(seq 1 ${ROUNDS:-2}); do for lib in ${LIBS}; do
  SPARKTS_ARIMA_LIB=spark-timeseries_amd/libsparkts_arima_dev_$lib.so timeout -k 10 200 python bench.py --steps ${STEPS:-12} --warmup 2 --pipeline ${P:-3} --e2e 0 --cpu-seconds 0 ${ARGS} > $OUT/${lib}_$i.json 2> $OUT/${lib}_$i.err || exit $?
  echo "$lib $i done"
done; done
