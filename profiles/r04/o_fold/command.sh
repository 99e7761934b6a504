# session o_fold: dev libraries p = q = 2: base22 (-DSTS_PIT_FOLD_RL=0), rl22 (express P-I-T folds as one uniform
# chain over v_readlane_b32 reads: reverted, slower), pfg3 / pfg1 (-DSTS_PREFETCH_G=3 / 1), pff3 (-DSTS_PREFETCH_F=3),
# trl22 / tb22 (+ STS_TIMING)
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-o_fold}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_rl22.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "(c2_212 and not shift) or c2_batch or express_path or drain_merge or full_size" > $OUT/pytest_rl.log 2>&1 || exit 1
B="timeout -k 10 150 python -u bench.py --cpu-seconds 0 --e2e 0"
for r in 1 2; do for lib in base22 rl22; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so $B --pipeline 1 --steps 3 --warmup 1 > $OUT/iso_${lib}_$r.json 2> $OUT/iso_${lib}_$r.err || exit 1
done; done
for r in 1 2; do for lib in base22 rl22 pfg3 pfg1 pff3; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so $B --steps 10 --warmup 3 > $OUT/pipe_${lib}_$r.json 2> $OUT/pipe_${lib}_$r.err || exit 1
done; done
for lib in trl22 tb22; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so timeout -k 10 150 python -u tools/fit_diag.py --reps 1 > $OUT/diag_$lib.json 2> $OUT/diag_$lib.err || exit 1
done
