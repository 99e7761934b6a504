#!/bin/bash
# fit-kernel variant comparison (dev libraries, tools/fit_diag.py): LIBS="tag1 tag2 ..." ARGS="..." bash tools/gpu_diag.sh
set -o pipefail
OUT=gpurun_out/${TAG:-diag}
mkdir -p $OUT
for lib in ${LIBS:-timing}; do
  SPARKTS_ARIMA_LIB=spark-timeseries_amd/libsparkts_arima_dev_$lib.so timeout -k 10 120 python tools/fit_diag.py --reps ${REPS:-2} ${ARGS} > $OUT/$lib.json 2> $OUT/$lib.err
  rc=$?
  echo "variant $lib rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
