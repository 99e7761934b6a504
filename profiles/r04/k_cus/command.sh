# session k_cus (library of 96b9e99)
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-k_cus}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
B="timeout -k 10 150 python -u bench.py --cpu-seconds 0 --e2e 0 --steps 10 --warmup 3"
for r in 1 2; do
  for cfg in "0 0" "224 0" "208 0" "224 256" "224 1024" "0 1024" "192 0"; do
    set -- $cfg
    SPARKTS_OPTIONS=hr_grid=$2 $B --grid-blocks $1 > $OUT/pipe_g$1_h$2_$r.json 2> $OUT/pipe_g$1_h$2_$r.err || exit 1
  done
done
for p in 8 4; do
  $B --pipeline $p > $OUT/pipe_P${p}.json 2> $OUT/pipe_P${p}.err || exit 1
done
