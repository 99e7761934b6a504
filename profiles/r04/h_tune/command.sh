# session h_tune (gpurun --timeout 1200 -- 'TAG=h_tune bash <this file>'), library = 705dffc + merge pool 3/4 of
# the ring, search_express_blocks (default 0), donate_evals / donate_evals_drained options
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-h_tune}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
B="timeout -k 10 150 python -u bench.py --cpu-seconds 0 --e2e 0"
for xb in -1 32; do for de in 0 128 64; do
  SPARKTS_OPTIONS=donate_evals=$de $B --pipeline 1 --steps 3 --warmup 1 --express-blocks $xb > $OUT/iso_x${xb}_d${de}.json 2> $OUT/iso_x${xb}_d${de}.err || exit 1
done; done
for r in 1 2; do
  for ml in 16 24 32; do
    SPARKTS_OPTIONS=merge_live=$ml $B --steps 10 --warmup 3 > $OUT/pipe_m${ml}_$r.json 2> $OUT/pipe_m${ml}_$r.err || exit 1
  done
  for xb in 0 4; do
    $B --steps 10 --warmup 3 --express-blocks $xb > $OUT/pipe_x${xb}_$r.json 2> $OUT/pipe_x${xb}_$r.err || exit 1
  done
done
timeout -k 10 200 python -u bench.py --config c5 --total-series 262144 --steps 1 --warmup 0 --cpu-seconds 0 > $OUT/c5.json 2> $OUT/c5.err || exit 1
for ml in 16 32; do
  SPARKTS_OPTIONS=merge_live=$ml timeout -k 10 200 python -u bench.py --config c4 --steps 3 --warmup 1 --cpu-seconds 0 --e2e 0 > $OUT/c4_m$ml.json 2> $OUT/c4_m$ml.err || exit 1
done
