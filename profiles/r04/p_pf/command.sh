cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-p_pf}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_pff3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "(c2_212 and not shift) or c2_batch or express_path or drain_merge or full_size" > $OUT/pytest_pff3.log 2>&1 || exit 1
B="timeout -k 10 150 python -u bench.py --cpu-seconds 0 --e2e 0"
for r in 1 2; do for lib in base22 pff3 pff2 pff3g1 pff2g1; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so $B --steps 10 --warmup 3 > $OUT/pipe_${lib}_$r.json 2> $OUT/pipe_${lib}_$r.err || exit 1
done; done
for lib in base22 pff3 pff2 pff3g1 pff2g1; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so $B --pipeline 1 --steps 3 --warmup 1 > $OUT/iso_${lib}.json 2> $OUT/iso_${lib}.err || exit 1
done
