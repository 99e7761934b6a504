#!/bin/bash
# k_hr_init A/B: grid of single-wave workgroups (hr_grid option; 0 = a lane per series, 256-lane blocks) and the
# Householder prefetch depth (dev library built with DEVFLAGS=-DSTS_HR_PF=4). Isolated launches (--pipeline 1):
# the bench line's kernel_ms.hr_init is the HIP-event time of the HR launch alone.
set -o pipefail
OUT=gpurun_out/${TAG:-r03/hr}
mkdir -p $OUT
B="python bench.py --steps 2 --warmup 1 --pipeline 1 --e2e 0 --cpu-seconds 0"
for g in ${GRIDS:-0 256 512 1024 2048 4096}; do
  SPARKTS_OPTIONS=hr_grid=$g timeout -k 10 120 $B > $OUT/c2_g$g.json 2>> $OUT/err.log || exit 1
  if [ -f spark-timeseries_amd/libsparkts_arima_dev_hrpf4.so ]; then
    SPARKTS_ARIMA_LIB=$PWD/spark-timeseries_amd/libsparkts_arima_dev_hrpf4.so SPARKTS_OPTIONS=hr_grid=$g \
      timeout -k 10 120 $B > $OUT/c2pf4_g$g.json 2>> $OUT/err.log || exit 1
  fi
  echo "grid $g done"
done
for g in ${C4GRIDS:-0 512 2048}; do
  SPARKTS_OPTIONS=hr_grid=$g timeout -k 10 300 $B --config c4 --series 131072 --steps 1 > $OUT/c4_g$g.json 2>> $OUT/err.log || exit 1
  echo "c4 grid $g done"
done
