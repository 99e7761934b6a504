cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-u_rt}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
B="timeout -k 10 150 python -u bench.py --cpu-seconds 0 --e2e 0 --steps 10 --warmup 3"
# runtime knobs on the final library: express CUs, fit contexts, merge threshold
for r in 1 2; do
  $B > $OUT/pipe_base_$r.json 2> $OUT/pipe_base_$r.err || exit 1
  for xb in 8 24; do $B --express-blocks $xb > $OUT/pipe_x${xb}_$r.json 2> $OUT/pipe_x${xb}_$r.err || exit 1; done
  for P in 5 8; do $B --pipeline $P > $OUT/pipe_P${P}_$r.json 2> $OUT/pipe_P${P}_$r.err || exit 1; done
  for ml in 8 24; do SPARKTS_OPTIONS=merge_live=$ml $B > $OUT/pipe_m${ml}_$r.json 2> $OUT/pipe_m${ml}_$r.err || exit 1; done
done
