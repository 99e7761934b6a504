cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-y_c4rt}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/libsparkts_arima.so > $OUT/library.sha256
B="timeout -k 10 250 python -u bench.py --config c4 --cpu-seconds 0 --e2e 0 --steps 3 --warmup 1"
# C4 runtime knobs on the final library: fit contexts, express CUs, merge threshold
$B > $OUT/c4_base_1.json 2> $OUT/c4_base_1.err || exit 1
for P in 3 5 6; do $B --pipeline $P > $OUT/c4_P$P.json 2> $OUT/c4_P$P.err || exit 1; done
for xb in 8 32; do $B --express-blocks $xb > $OUT/c4_x$xb.json 2> $OUT/c4_x$xb.err || exit 1; done
for ml in 8 32; do SPARKTS_OPTIONS=merge_live=$ml $B > $OUT/c4_m$ml.json 2> $OUT/c4_m$ml.err || exit 1; done
$B > $OUT/c4_base_2.json 2> $OUT/c4_base_2.err || exit 1
