cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/y_lines; mkdir -p $O
sha256sum spark-timeseries_amd/libsparkts_arima.so > $O/library.sha256
timeout -k 10 300 python -u bench.py --config c1 > $O/c1.json 2> $O/c1.err &&
timeout -k 10 400 python -u bench.py --config c4 > $O/c4.json 2> $O/c4.err &&
timeout -k 10 400 python -u bench.py --config af > $O/af.json 2> $O/af.err &&
timeout -k 10 500 python -u bench.py --config c5 > $O/c5.json 2> $O/c5.err
echo "rc=$?" > $O/rc.txt
