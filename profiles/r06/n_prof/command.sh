cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/n_prof; mkdir -p $O
sha256sum spark-timeseries_amd/libsparkts_arima.so > $O/library.sha256
OUT=$O/prof_c2 bash tools/profile.sh > $O/profile_c2.log 2>&1 &&
TAG=n_pipe timeout -k 10 450 bash tools/trace_c2_pipe.sh > $O/pipe.log 2>&1
echo "rc=$?" > $O/rc.txt
