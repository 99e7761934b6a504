cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/w_prof5; mkdir -p $O
sha256sum spark-timeseries_amd/libsparkts_arima.so > $O/library.sha256
PASSES="trace fetch write" CONFIG=c5 SER=1048576 OUT=$O/prof_c5 bash tools/profile.sh > $O/profile_c5.log 2>&1
echo "rc=$?" > $O/rc.txt
