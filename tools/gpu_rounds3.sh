#!/bin/bash
# rounds: full per-round distribution (1000 rounds, no early hand-off) per pass-kernel build, isolated C2 fits
set -o pipefail
OUT=gpurun_out/${TAG:-r03/rounds6}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in ${VARS:-rounds pf4}; do
  SPARKTS_ARIMA_LIB=$PWD/spark-timeseries_amd/libsparkts_arima_dev_$v.so timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/p_$v -o run --output-format csv -- python3 tools/rounds_trace.py 1048576 ${RMAX:-1000} 0 > $OUT/trace_$v.jsonl 2> $OUT/err_$v.txt || exit 1
  echo "trace $v ok"
done
for v in ${BVARS:-rounds pf4 pf8}; do
  SPARKTS_ARIMA_LIB=$PWD/spark-timeseries_amd/libsparkts_arima_dev_$v.so SPARKTS_OPTIONS=rounds_tail_express=0 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --pipeline 1 --e2e 0 --cpu-seconds 0 --fit-kernel 2 > $OUT/bench_$v.json 2>> $OUT/bench.err || exit 1
  echo "bench $v ok"
done
