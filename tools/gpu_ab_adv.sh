#!/bin/bash
# Register-copy advance A/B (dev libraries advreg / advlds): outputs bit-identical, then alternating timings.
set -o pipefail
OUT=gpurun_out/${TAG:-r03/ab_adv}
mkdir -p $OUT
for lib in advreg advlds; do
  SPARKTS_ARIMA_LIB=$PWD/spark-timeseries_amd/libsparkts_arima_dev_$lib.so timeout -k 10 120 python tools/fit_dump.py $OUT/$lib.npz > /dev/null 2>> $OUT/err.log || exit 1
done
python -c "
import numpy as np,sys
a=np.load('$OUT/advreg.npz');b=np.load('$OUT/advlds.npz')
bad=[k for k in a.files if a[k].tobytes()!=b[k].tobytes()]
print('bit-identical' if not bad else 'DIFFER '+str(bad)); sys.exit(1 if bad else 0)" > $OUT/compare.txt || exit 1
LIBS="advlds advreg" ROUNDS=${ROUNDS:-2} TAG=${TAG:-r03/ab_adv} bash tools/gpu_ab_lib.sh
