cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-x_c5}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/libsparkts_arima.so > $OUT/library.sha256
# C5 with bench.py's new default of 12 search lanes: the line with roofline, CPU baseline and selection parity
timeout -k 10 300 python -u bench.py --config c5 --total-series 262144 --steps 1 --warmup 0 --cpu-seconds 10 > $OUT/c5_262144.json 2> $OUT/c5.err || exit 1
timeout -k 10 300 python -u bench.py --config c5 --total-series 262144 --steps 2 --warmup 0 --cpu-seconds 0 > $OUT/c5_262144_2steps.json 2> $OUT/c5_2.err || exit 1
