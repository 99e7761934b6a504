cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/zd_knobs; mkdir -p $O
sha256sum spark-timeseries_amd/libsparkts_arima.so > $O/library.sha256
B="--cpu-seconds 0 --e2e 0 --default-leg 0"
run() { tag=$1; shift; timeout -k 10 200 "$@" > $O/$tag.json 2> $O/$tag.err; }
run base python -u bench.py $B &&
run xb0 python -u bench.py $B --express-blocks 0 &&
run xb8 python -u bench.py $B --express-blocks 8 &&
run xb24 python -u bench.py $B --express-blocks 24 &&
run p5 python -u bench.py $B --pipeline 5 &&
run p7 python -u bench.py $B --pipeline 7 &&
SPARKTS_OPTIONS=merge_live=32 run ml32 python -u bench.py $B &&
SPARKTS_OPTIONS=merge_live=8 run ml8 python -u bench.py $B &&
run base2 python -u bench.py $B
echo "rc=$?" > $O/rc.txt
