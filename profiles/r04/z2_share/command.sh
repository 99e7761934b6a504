cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-z2_share}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/libsparkts_arima.so > $OUT/library.sha256
# the HR init's share of the pipelined C2 step on the final library, and the pipelined kernel trace
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/hr_share.py --config c2 > $OUT/hr_share_c2.json 2> $OUT/hr_share_c2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/pipe_trace -o run -- python3 bench.py --steps 8 --warmup 2 --cpu-seconds 0 --e2e 0 > $OUT/pipe_trace.json 2> $OUT/pipe_trace.err || exit 1
