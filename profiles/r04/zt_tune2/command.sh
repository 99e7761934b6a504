cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-zt_tune2}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
B="timeout -k 10 150 python -u bench.py --cpu-seconds 0 --e2e 0"
# dev libraries p = q = 2 on the final defaults: priority threshold 64, fixed objective pass width, no objective
# rides on gradient passes, pass cost model overhead 3
for r in 1 2 3; do for lib in nb old64 nonc noride ovh3; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so $B --steps 20 --warmup 3 > $OUT/pipe_${lib}_$r.json 2> $OUT/pipe_${lib}_$r.err || exit 1
done; done
for lib in nb old64 nonc noride ovh3; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so $B --pipeline 1 --steps 3 --warmup 1 > $OUT/iso_${lib}.json 2> $OUT/iso_${lib}.err || exit 1
done
