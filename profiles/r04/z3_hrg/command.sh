cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-z3_hrg}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/libsparkts_arima.so > $OUT/library.sha256
B="timeout -k 10 150 python -u bench.py --cpu-seconds 0 --e2e 0 --steps 20 --warmup 3"
for r in 1 2; do for hg in 1024 256 512 4096; do
  SPARKTS_OPTIONS=hr_grid=$hg $B > $OUT/pipe_h${hg}_$r.json 2> $OUT/pipe_h${hg}_$r.err || exit 1
done; done
