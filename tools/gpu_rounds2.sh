#!/bin/bash
# rounds fit: parity subset, per-round trace, C2 throughput over hand-off points (dev library DEV=<tag>)
set -o pipefail
OUT=gpurun_out/${TAG:-r03/rounds2}
mkdir -p $OUT
export SPARKTS_ARIMA_LIB=$PWD/spark-timeseries_amd/libsparkts_arima_dev_${DEV:-rounds}.so
for opt in "fit_kernel=2,rounds_tail=0,rounds_max=400" "fit_kernel=2,rounds_tail=0,rounds_max=12" "fit_kernel=2,rounds_tail=1000,rounds_max=400"; do
  SPARKTS_OPTIONS=$opt timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTK:-c2_batch or full_size}" >> $OUT/pytest.log 2>&1 || { echo "tests failed: $opt"; exit 1; }
  echo "tests ok: $opt"
done
(cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/p -o run --output-format csv -- python3 tools/rounds_trace.py 1048576 ${RMAX:-96} ${RTAIL:--1} > $OUT/trace.jsonl 2> $OUT/trace.err) || exit 1
echo trace ok
for ta in ${TAILS:--1 200000 400000}; do
  SPARKTS_OPTIONS=rounds_tail=$ta timeout -k 10 300 python bench.py --steps 6 --warmup 2 --e2e 0 --cpu-seconds 0 --fit-kernel 2 > $OUT/bench_t$ta.json 2>> $OUT/bench.err || exit 1
  SPARKTS_OPTIONS=rounds_tail=$ta timeout -k 10 300 python bench.py --steps 2 --warmup 1 --pipeline 1 --e2e 0 --cpu-seconds 0 --fit-kernel 2 > $OUT/bench_t${ta}_p1.json 2>> $OUT/bench.err || exit 1
  echo "bench $ta ok"
done
