cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/z_sweep; mkdir -p $O
sha256sum spark-timeseries_amd/libsparkts_arima.so > $O/library.sha256
timeout -k 10 1000 python -u tools/parity_sweep.py --series 4096 --T 1024 --out $O/parity_sweep_4096x1024.jsonl > $O/sweep_big.log 2>&1
echo "rc=$?" > $O/rc.txt
