set -o pipefail
mkdir -p gpurun_out/diag
export SPARKTS_ARIMA_LIB=spark-timeseries_amd/libsparkts_arima_dev_timing.so
timeout -k 10 120 python tools/fit_diag.py --reps 2 > gpurun_out/diag/timing.json 2> gpurun_out/diag/timing.err &&
timeout -k 10 120 python tools/fit_diag.py --reps 2 --express-blocks 0 > gpurun_out/diag/timing_x0.json 2> gpurun_out/diag/timing_x0.err
