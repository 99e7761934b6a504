cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-m_hrgrid}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
B="timeout -k 10 150 python -u bench.py --cpu-seconds 0 --e2e 0"
for r in 1 2; do for hg in 512 1024 2048 0; do
  SPARKTS_OPTIONS=hr_grid=$hg $B --steps 10 --warmup 3 > $OUT/pipe_h${hg}_$r.json 2> $OUT/pipe_h${hg}_$r.err || exit 1
done; done
for hg in 1024 0; do
  SPARKTS_OPTIONS=hr_grid=$hg $B --pipeline 1 --steps 3 --warmup 1 > $OUT/iso_h${hg}.json 2> $OUT/iso_h${hg}.err || exit 1
  SPARKTS_OPTIONS=hr_grid=$hg timeout -k 10 200 python -u bench.py --config c4 --steps 3 --warmup 1 --cpu-seconds 0 --e2e 0 > $OUT/c4_h${hg}.json 2> $OUT/c4_h${hg}.err || exit 1
  SPARKTS_OPTIONS=hr_grid=$hg timeout -k 10 200 python -u bench.py --config c5 --total-series 262144 --steps 1 --warmup 0 --cpu-seconds 0 > $OUT/c5_h${hg}.json 2> $OUT/c5_h${hg}.err || exit 1
done
