cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/d_pit; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
for r in 1 2; do for lib in pit nopit advinl; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so timeout -k 10 150 python -u bench.py --pipeline 1 --steps 3 --warmup 1 --cpu-seconds 0 --e2e 0 > $OUT/iso_${lib}_$r.json 2> $OUT/iso_${lib}_$r.err || exit 1
done; done
SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_timing2.so timeout -k 10 150 python -u tools/fit_timing.py --fit-kernel 0 > $OUT/timing.jsonl 2> $OUT/timing.err || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 5 > $OUT/bench.json 2> $OUT/bench.err
