# session j_cores: dev libraries (make dev, p = q = 2) base / hr1 (-DSTS_HR_PF=1: k_hr_init 186 VGPRs) / nopit
# (-DSTS_PIT=0 -DSTS_PIT_G=0: k_cg_fit 256 VGPR + 32 AGPR) / nopithr1 (both); timing22 / timing55 = -DSTS_TIMING
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-j_cores}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
B="timeout -k 10 150 python -u bench.py --cpu-seconds 0 --e2e 0"
for r in 1 2; do for lib in base hr1 nopit nopithr1; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so $B --steps 10 --warmup 3 > $OUT/pipe_${lib}_$r.json 2> $OUT/pipe_${lib}_$r.err || exit 1
done; done
for lib in base nopithr1; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so $B --pipeline 1 --steps 3 --warmup 1 > $OUT/iso_${lib}.json 2> $OUT/iso_${lib}.err || exit 1
  GPU_MAX_HW_QUEUES=8 SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so timeout -k 10 300 python -u tools/hr_share.py --config c2 > $OUT/hr_share_$lib.json 2> $OUT/hr_share_$lib.err || exit 1
done
SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_timing55.so timeout -k 10 200 python -u tools/fit_diag.py --order 5,1,5,1 --T 4096 --reps 1 > $OUT/diag_c4.json 2> $OUT/diag_c4.err || exit 1
SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_timing55.so timeout -k 10 200 python -u tools/fit_timing.py --order 5,1,5,1 --T 4096 --fit-kernel 0 --reps 1 > $OUT/timing_c4.jsonl 2> $OUT/timing_c4.err || exit 1
SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_timing22.so timeout -k 10 150 python -u tools/fit_diag.py --reps 1 > $OUT/diag_c2.json 2> $OUT/diag_c2.err || exit 1
