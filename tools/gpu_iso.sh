#!/bin/bash
# isolated-launch comparison of dev-library variants: fit_diag (one fit at a time), REPS each, LIBS alternating
set -o pipefail
OUT=gpurun_out/${TAG:-iso}; mkdir -p $OUT
for i in 1 2; do for lib in ${LIBS}; do
  SPARKTS_ARIMA_LIB=spark-timeseries_amd/libsparkts_arima_dev_$lib.so timeout -k 10 150 python tools/fit_diag.py --reps ${REPS:-3} > $OUT/${lib}_$i.json 2> $OUT/${lib}_$i.err || exit $?
  echo "$lib $i done"
done; done
