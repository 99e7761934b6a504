cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-w_lanes}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/libsparkts_arima.so > $OUT/library.sha256
C5="timeout -k 10 200 python -u bench.py --config c5 --total-series 262144 --steps 1 --warmup 0 --cpu-seconds 0"
for r in 1 2; do
  for sl in 8 10 12; do $C5 --search-lanes $sl > $OUT/c5_l${sl}_$r.json 2> $OUT/c5_l${sl}_$r.err || exit 1; done
  for ml in 24 32; do SPARKTS_OPTIONS=merge_live=$ml $C5 --search-lanes 12 > $OUT/c5_l12_m${ml}_$r.json 2> $OUT/c5_l12_m${ml}_$r.err || exit 1; done
done
