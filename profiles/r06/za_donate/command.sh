cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/za_donate; mkdir -p $O
sha256sum spark-timeseries_amd/libsparkts_arima.so > $O/library.sha256
for o in "" "donate_evals=128" "donate_evals=64" "donate_evals_drained=16" "donate_evals_drained=64" "donate_evals=128,donate_evals_drained=16"; do
  tag=$(echo "x$o" | tr ',=' '__')
  SPARKTS_OPTIONS="$o" timeout -k 10 200 python -u bench.py --cpu-seconds 0 --e2e 0 --default-leg 0 > $O/$tag.json 2> $O/$tag.err || break
done
echo "rc=$?" > $O/rc.txt
