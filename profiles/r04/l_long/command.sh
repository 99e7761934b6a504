# session l_long: dev libraries p = q = 5 with STS_PIT_LONG=1 (long55; tlong55 + STS_TIMING): express objective
# passes over 64 x 64-step rows parallel in time with one chain (reverted: slower)
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-l_long}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_long55.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "c4_T4096 or c4_515 or long_fits" > $OUT/pytest_long.log 2>&1 || exit 1
B="timeout -k 10 200 python -u bench.py --config c4 --cpu-seconds 0 --e2e 0"
for lib in long55 main; do
  L=$D/libsparkts_arima.so; [ $lib = long55 ] && L=$D/libsparkts_arima_dev_long55.so
  SPARKTS_ARIMA_LIB=$L $B --pipeline 1 --steps 1 --warmup 1 > $OUT/c4_iso_$lib.json 2> $OUT/c4_iso_$lib.err || exit 1
  SPARKTS_ARIMA_LIB=$L $B --steps 3 --warmup 1 > $OUT/c4_pipe_$lib.json 2> $OUT/c4_pipe_$lib.err || exit 1
done
SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_tlong55.so timeout -k 10 200 python -u tools/fit_diag.py --order 5,1,5,1 --T 4096 --reps 1 > $OUT/diag_c4.json 2> $OUT/diag_c4.err || exit 1
