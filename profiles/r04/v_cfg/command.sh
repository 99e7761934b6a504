cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-v_cfg}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/libsparkts_arima.so > $OUT/library.sha256
C5="timeout -k 10 200 python -u bench.py --config c5 --total-series 262144 --steps 1 --warmup 0 --cpu-seconds 0"
for sl in 12 24; do $C5 --search-lanes $sl > $OUT/c5_l$sl.json 2> $OUT/c5_l$sl.err || exit 1; done
for ml in 8 32; do SPARKTS_OPTIONS=merge_live=$ml $C5 > $OUT/c5_m$ml.json 2> $OUT/c5_m$ml.err || exit 1; done
$C5 > $OUT/c5_base.json 2> $OUT/c5_base.err || exit 1
timeout -k 10 300 python -u bench.py --total-series 8388608 --steps 2 --warmup 1 --cpu-seconds 0 --e2e 0 > $OUT/c3.json 2> $OUT/c3.err || exit 1
timeout -k 10 200 python -u bench.py --smear 0 --steps 10 --warmup 3 --cpu-seconds 0 --e2e 0 > $OUT/c2_shift.json 2> $OUT/c2_shift.err || exit 1
