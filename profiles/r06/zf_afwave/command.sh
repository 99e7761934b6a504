cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/zf_afwave; mkdir -p $O
sha256sum spark-timeseries_amd/libsparkts_arima.so > $O/library.sha256
SPARKTS_OPTIONS=bobyqa_wave=0 timeout -k 10 400 python -u bench.py --config af > $O/af_lane.json 2> $O/af_lane.err &&
timeout -k 10 400 python -u bench.py --config af > $O/af_default.json 2> $O/af_default.err
echo "rc=$?" > $O/rc.txt
