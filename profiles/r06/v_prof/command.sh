cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/v_prof; mkdir -p $O
sha256sum spark-timeseries_amd/libsparkts_arima.so > $O/library.sha256
OUT=$O/prof_c2 bash tools/profile.sh > $O/profile_c2.log 2>&1 &&
PASSES="trace fetch write" CONFIG=c4 SER=1048576 OUT=$O/prof_c4 bash tools/profile.sh > $O/profile_c4.log 2>&1
echo "rc=$?" > $O/rc.txt
