#!/bin/bash
# ad-hoc GPU experiment steps (round 2); each step under its own limit, stop at the first failure
set -o pipefail
OUT=gpurun_out/${TAG:-x}
mkdir -p $OUT
D=spark-timeseries_amd
for step in "$@"; do
  case $step in
    diag_base)   timeout -k 10 120 python tools/fit_diag.py --reps 2 > $OUT/diag_base.json 2> $OUT/diag_base.err ;;
    diag_d128)   SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_don128.so timeout -k 10 120 python tools/fit_diag.py --reps 2 > $OUT/diag_d128.json 2> $OUT/diag_d128.err ;;
    diag_d64)    SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_don64.so timeout -k 10 120 python tools/fit_diag.py --reps 2 > $OUT/diag_d64.json 2> $OUT/diag_d64.err ;;
    rep_x0)      SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_p3q2.so timeout -k 10 60 python tools/grid_profile.py --orders "3,1,2,0;3,1,2,1" --express-blocks 0 > $OUT/rep_x0.jsonl 2> $OUT/rep_x0.err ;;
    rep_xd)      SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_p3q2.so timeout -k 10 60 python tools/grid_profile.py --orders "3,1,2,0;3,1,2,1" > $OUT/rep_xd.jsonl 2> $OUT/rep_xd.err ;;
    xtests)      timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "express or order_search" > $OUT/xtests.log 2>&1 ;;
    rep_p1)      SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_p1q1.so timeout -k 10 90 python tools/grid_profile.py --orders "1,2,1,0;1,2,1,1;1,1,1,1;1,0,1,1" > $OUT/rep_p1.jsonl 2> $OUT/rep_p1.err ;;
    search1)     timeout -k 10 400 python tools/bench_search.py --series 131072 --lanes 1 > $OUT/search1.json 2> $OUT/search1.err ;;
    search4)     timeout -k 10 400 python tools/bench_search.py --series 131072 --lanes 4 > $OUT/search4.json 2> $OUT/search4.err ;;
    search4big)  timeout -k 10 600 python tools/bench_search.py --series 262144 --lanes 4 > $OUT/search4big.json 2> $OUT/search4big.err ;;
    search4s)    timeout -k 10 300 python tools/bench_search.py --series 32768 --lanes 4 > $OUT/search4s.json 2> $OUT/search4s.err ;;
    search1s)    timeout -k 10 300 python tools/bench_search.py --series 32768 --lanes 1 > $OUT/search1s.json 2> $OUT/search1s.err ;;
    bench)       timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err ;;
    predictor)   timeout -k 10 300 python tools/predictor_study.py > $OUT/predictor.json 2> $OUT/predictor.err ;;
    diag_x32)    timeout -k 10 120 python tools/fit_diag.py --reps 2 --express-blocks 32 > $OUT/diag_x32.json 2> $OUT/diag_x32.err ;;
    diag_x48)    timeout -k 10 120 python tools/fit_diag.py --reps 2 --express-blocks 48 > $OUT/diag_x48.json 2> $OUT/diag_x48.err ;;
    grid)        timeout -k 10 600 python tools/grid_profile.py > $OUT/grid.jsonl 2> $OUT/grid.err ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $step rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
