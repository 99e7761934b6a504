cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-s_c4pf}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
B="timeout -k 10 200 python -u bench.py --config c4 --cpu-seconds 0 --e2e 0"
# C4 (dev libraries p = q = 5): objective / gradient chunks in flight per lane 3 / 1 (default), 2 / 1, 3 / 2, 2 / 2
for r in 1 2; do for lib in c4pf31 c4pf21 c4pf32 c4pf22; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so $B --steps 3 --warmup 1 > $OUT/pipe_${lib}_$r.json 2> $OUT/pipe_${lib}_$r.err || exit 1
done; done
