# session g_merge (gpurun --timeout 1200 -- 'TAG=g_merge bash <this file>'), library at 705dffc
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-g_merge}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
for r in 1 2; do for ml in 0 16 32; do
  SPARKTS_OPTIONS=merge_live=$ml timeout -k 10 150 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --e2e 0 > $OUT/pipe_m${ml}_$r.json 2> $OUT/pipe_m${ml}_$r.err || exit 1
done; done
for ml in 0 16; do
  SPARKTS_OPTIONS=merge_live=$ml timeout -k 10 150 python -u bench.py --pipeline 1 --steps 3 --warmup 1 --cpu-seconds 0 --e2e 0 > $OUT/iso_m${ml}.json 2> $OUT/iso_m${ml}.err || exit 1
done
for xb in -1 4 0; do
  timeout -k 10 200 python -u bench.py --config c5 --total-series 262144 --steps 1 --warmup 0 --cpu-seconds 0 --express-blocks $xb > $OUT/c5_x$xb.json 2> $OUT/c5_x$xb.err || exit 1
done
timeout -k 10 200 python -u bench.py --config c4 --steps 3 --warmup 1 --cpu-seconds 0 --e2e 0 > $OUT/c4.json 2> $OUT/c4.err || exit 1
timeout -k 10 200 python -u bench.py --config c4 --pipeline 1 --steps 1 --warmup 1 --cpu-seconds 0 --e2e 0 > $OUT/c4_iso.json 2> $OUT/c4_iso.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c5prof -o c5 -- python -u bench.py --config c5 --total-series 65536 --steps 1 --warmup 0 --cpu-seconds 0 > $OUT/c5prof.log 2>&1 || exit 1
