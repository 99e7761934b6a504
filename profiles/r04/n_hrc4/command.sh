# session n_hrc4: dev libraries p = q = 5 (make dev DEVP=5 DEVQ=5) with -DSTS_HR_PF=1 / (default 2) / 3
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/${TAG:-n_hrc4}; mkdir -p $OUT
D=$PWD/spark-timeseries_amd
sha256sum $D/*.so > $OUT/library.sha256
B="timeout -k 10 200 python -u bench.py --config c4 --cpu-seconds 0 --e2e 0"
for lib in hrpf1_55 hrpf2_55 hrpf3_55; do
  SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_$lib.so $B --pipeline 1 --steps 1 --warmup 1 > $OUT/iso_$lib.json 2> $OUT/iso_$lib.err || exit 1
done
for hg in 1024 4096 16384; do
  SPARKTS_OPTIONS=hr_grid=$hg SPARKTS_ARIMA_LIB=$D/libsparkts_arima_dev_hrpf2_55.so $B --pipeline 1 --steps 1 --warmup 1 > $OUT/iso_pf2_h$hg.json 2> $OUT/iso_pf2_h$hg.err || exit 1
done
