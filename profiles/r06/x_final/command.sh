cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/x_final; mkdir -p $O
sha256sum spark-timeseries_amd/libsparkts_arima.so > $O/library.sha256
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
echo "rc=$?" > $O/rc.txt
