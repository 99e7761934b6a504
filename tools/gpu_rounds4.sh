#!/bin/bash
# rounds fit: pipelined C2 throughput over (hand-off round, tail grid, contexts)
set -o pipefail
OUT=gpurun_out/${TAG:-r03/rounds7}
mkdir -p $OUT
export SPARKTS_ARIMA_LIB=$PWD/spark-timeseries_amd/libsparkts_arima_dev_${DEV:-rounds}.so
run() {  # name pipeline options
  SPARKTS_OPTIONS=$3 timeout -k 10 300 python bench.py --steps ${STEPS:-12} --warmup 2 --pipeline $2 --e2e 0 --cpu-seconds 0 --fit-kernel 2 > $OUT/$1.json 2>> $OUT/bench.err || exit 1
  echo "$1 ok"
}
run A_r96_full_p3 3 "rounds_max=96,rounds_tail=0"
run B_r150_t64x32_p3 3 "rounds_max=150,rounds_tail=0,rounds_tail_cus=64,rounds_tail_xcus=32"
run B_r150_t64x32_p5 5 "rounds_max=150,rounds_tail=0,rounds_tail_cus=64,rounds_tail_xcus=32"
run C_r300_t32x32_p5 5 "rounds_max=300,rounds_tail=0,rounds_tail_cus=32,rounds_tail_xcus=32"
run E_r150_t0x64_p5 5 "rounds_max=150,rounds_tail=0,rounds_tail_cus=0,rounds_tail_xcus=64"
run D_r2000_p6 6 "rounds_max=2000,rounds_tail=0"
