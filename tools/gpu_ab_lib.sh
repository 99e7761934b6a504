#!/bin/bash
# A/B of dev libraries on one box (C2, p = q = 2 instantiations only): LIBS="a b" ROUNDS=2 bash tools/gpu_ab_lib.sh
# Alternates the variants; isolated launches (--pipeline 1) and the pipelined headline step. Run ON the GPU box.
set -o pipefail
OUT=gpurun_out/${TAG:-r03/ab_lib}
mkdir -p $OUT
ISO="python bench.py --steps 2 --warmup 1 --pipeline 1 --e2e 0 --cpu-seconds 0"
PIPE="python bench.py --steps 20 --warmup 5 --e2e 0 --cpu-seconds 0"
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in ${LIBS:-oldsel newsel}; do
    L=$PWD/spark-timeseries_amd/libsparkts_arima_dev_$lib.so
    SPARKTS_ARIMA_LIB=$L timeout -k 10 120 $ISO > $OUT/${lib}_iso_$r.json 2>> $OUT/err.log || exit 1
    SPARKTS_ARIMA_LIB=$L timeout -k 10 180 $PIPE > $OUT/${lib}_pipe_$r.json 2>> $OUT/err.log || exit 1
    echo "round $r $lib ok"
  done
done
