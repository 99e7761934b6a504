cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/c_ab; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_timing.so timeout -k 10 200 python -u tools/fit_timing.py --fit-kernel 0 3 > $OUT/timing.jsonl 2> $OUT/timing.err &&
for lib in spl32 pf4; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so timeout -k 10 150 python -u bench.py --fit-kernel 3 --steps 10 --warmup 3 --cpu-seconds 0 --e2e 0 > $OUT/bench_$lib.json 2> $OUT/bench_$lib.err || exit 1
done
