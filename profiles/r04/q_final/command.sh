cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-q_final}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/libsparkts_arima.so > $OUT/library.sha256
sha256sum $D/libsparkts_arima_prev.so > $OUT/library_prev.sha256
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
B="timeout -k 10 200 python -u bench.py --cpu-seconds 0 --e2e 0"
for r in 1 2; do for lib in prev new; do
  L=$D/libsparkts_arima.so; [ $lib = prev ] && L=$D/libsparkts_arima_prev.so
  SPARKTS_ARIMA_LIB=$L $B --steps 10 --warmup 3 > $OUT/ab_c2_${lib}_$r.json 2> $OUT/ab_c2_${lib}_$r.err || exit 1
done; done
for lib in prev new; do
  L=$D/libsparkts_arima.so; [ $lib = prev ] && L=$D/libsparkts_arima_prev.so
  SPARKTS_ARIMA_LIB=$L $B --config c4 --steps 3 --warmup 1 > $OUT/ab_c4_$lib.json 2> $OUT/ab_c4_$lib.err || exit 1
done
SPARKTS_ARIMA_LIB=$D/libsparkts_arima_prev.so $B --config c5 --total-series 262144 --steps 1 --warmup 0 > $OUT/ab_c5_prev.json 2> $OUT/ab_c5_prev.err || exit 1
timeout -k 10 300 python -u bench.py --config c5 --total-series 262144 --steps 1 --warmup 0 --cpu-seconds 10 > $OUT/c5_262144.json 2> $OUT/c5.err || exit 1
timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --cpu-seconds 5 > $OUT/c4_1048576.json 2> $OUT/c4.err || exit 1
OUT=$OUT/prof_c2 timeout -k 10 600 bash tools/profile.sh > $OUT/profile_c2.log 2>&1 || exit 1
CONFIG=c4 SER=1048576 OUT=$OUT/prof_c4 timeout -k 10 600 bash tools/profile.sh > $OUT/profile_c4.log 2>&1 || exit 1
