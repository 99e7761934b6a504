cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-zv_tests}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/libsparkts_arima.so > $OUT/library.sha256
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "express_and_hr_grid or hr_grid_is_transparent" > $OUT/pytest_new.log 2>&1 || exit 1
