set -o pipefail
mkdir -p gpurun_out/r02i
export SPARKTS_ARIMA_LIB=$PWD/spark-timeseries_amd/libsparkts_arima_dev_x2.so
TAG=r02i ./tools/gpu_step.sh devtests || exit 1
for v in x1 x2 x1 x2; do
  SPARKTS_ARIMA_LIB=$PWD/spark-timeseries_amd/libsparkts_arima_dev_$v.so timeout -k 10 200 python tools/fit_diag.py --reps 3 >> gpurun_out/r02i/diag_$v.jsonl 2>> gpurun_out/r02i/diag.err || exit 1
done
