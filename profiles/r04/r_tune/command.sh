cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-r_tune}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
B="timeout -k 10 150 python -u bench.py --cpu-seconds 0 --e2e 0"
# dev libraries p = q = 2 on the final defaults: objective pass cost model (kChainOverhead16 6 -> 4 / 9) and the
# long-running priority threshold (kOldEvals 128 -> 64 / 256)
for r in 1 2; do for lib in nb22 ovh4 ovh9 old64 old256; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so $B --steps 10 --warmup 3 > $OUT/pipe_${lib}_$r.json 2> $OUT/pipe_${lib}_$r.err || exit 1
done; done
for lib in nb22 ovh4 ovh9 old64 old256; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so $B --pipeline 1 --steps 3 --warmup 1 > $OUT/iso_${lib}.json 2> $OUT/iso_${lib}.err || exit 1
done
