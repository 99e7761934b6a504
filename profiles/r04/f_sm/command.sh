# session f_sm (gpurun --timeout 1200 -- 'TAG=f_sm bash <this file>'); dev libraries built from 7ad7603 + the
# objective pass width choice: ncc = STS_NCH_CHOICE=1, nonc = STS_NCH_CHOICE=0, timing4 = ncc + STS_TIMING;
# libsparkts_arima_r3.so = the round-3 library (c3c893a), libsparkts_arima.so = 7ad7603
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-f_sm}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
for r in 1 2; do for lib in ncc nonc; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so timeout -k 10 150 python -u bench.py --pipeline 1 --steps 3 --warmup 1 --cpu-seconds 0 --e2e 0 > $OUT/iso_${lib}_$r.json 2> $OUT/iso_${lib}_$r.err || exit 1
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so timeout -k 10 150 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --e2e 0 > $OUT/pipe_${lib}_$r.json 2> $OUT/pipe_${lib}_$r.err || exit 1
done; done
SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_timing4.so timeout -k 10 150 python -u tools/fit_timing.py --fit-kernel 0 > $OUT/timing.jsonl 2> $OUT/timing.err || exit 1
for lib in r3 main; do
  L=$D/libsparkts_arima.so; [ $lib = r3 ] && L=$D/libsparkts_arima_r3.so
  SPARKTS_ARIMA_LIB=$L timeout -k 10 200 python -u bench.py --config c5 --total-series 262144 --steps 1 --warmup 0 --cpu-seconds 0 > $OUT/c5_$lib.json 2> $OUT/c5_$lib.err || exit 1
  SPARKTS_ARIMA_LIB=$L timeout -k 10 200 python -u bench.py --config c4 --steps 3 --warmup 1 --cpu-seconds 0 --e2e 0 > $OUT/c4_$lib.json 2> $OUT/c4_$lib.err || exit 1
done
