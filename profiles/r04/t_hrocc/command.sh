cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-t_hrocc}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
B="timeout -k 10 150 python -u bench.py --cpu-seconds 0 --e2e 0"
# k_hr_init occupancy (dev libraries p = q = 2): default (2 chunks, 249 VGPRs), 1 chunk (186), 1 chunk at 3 and 4 waves
# per SIMD (compiler-capped registers)
for r in 1 2; do for lib in hrb hrp1 hrp1w3 hrp1w4; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so $B --steps 10 --warmup 3 > $OUT/pipe_${lib}_$r.json 2> $OUT/pipe_${lib}_$r.err || exit 1
done; done
for lib in hrb hrp1 hrp1w3 hrp1w4; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so $B --pipeline 1 --steps 2 --warmup 1 > $OUT/iso_${lib}.json 2> $OUT/iso_${lib}.err || exit 1
done
