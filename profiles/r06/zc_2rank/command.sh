cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/zc_2rank; mkdir -p $O
sha256sum spark-timeseries_amd/libsparkts_arima.so > $O/library.sha256
timeout -k 10 500 python -u bench.py --gpus 2 --device 0 --series 524288 --steps 10 --warmup 2 > $O/c2_2ranks.json 2> $O/c2_2ranks.err
echo "rc=$?" > $O/rc.txt
