# session i_don (library of 96b9e99)
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-i_don}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
B="timeout -k 10 150 python -u bench.py --cpu-seconds 0 --e2e 0"
for r in 1 2; do for de in 32 48 64 0; do
  SPARKTS_OPTIONS=donate_evals=$de $B --pipeline 1 --steps 3 --warmup 1 > $OUT/iso_d${de}_$r.json 2> $OUT/iso_d${de}_$r.err || exit 1
done; done
for r in 1 2; do for de in 64 32 0; do
  SPARKTS_OPTIONS=donate_evals=$de $B --steps 10 --warmup 3 > $OUT/pipe_d${de}_$r.json 2> $OUT/pipe_d${de}_$r.err || exit 1
done; done
timeout -k 10 300 python -u tools/hr_share.py --config c2 > $OUT/hr_share_c2.json 2> $OUT/hr_share_c2.err || exit 1
timeout -k 10 300 python -u tools/hr_share.py --config c4 --series 262144 --steps 4 > $OUT/hr_share_c4.json 2> $OUT/hr_share_c4.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/pipe_trace -o run -- python3 bench.py --steps 8 --warmup 2 --cpu-seconds 0 --e2e 0 > $OUT/pipe_trace.json 2> $OUT/pipe_trace.err || exit 1
