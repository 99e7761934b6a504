#!/bin/bash
# Every BASELINE config on the final round-3 build, one MI355X: C3 (8M series, sliced), C4 (1M x 4096), C5 (262k,
# 16 lanes), the "shift" reading of ARIMA.scala:526, and the C4 rocprofv3 passes at 131 072 series.
# Each step has its own time limit; the chain stops at the first failure. Run ON the GPU box from the repo root.
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03/configs
mkdir -p $OUT
timeout -k 10 240 python -u bench.py --total-series 8388608 --steps 2 --warmup 1 --e2e 0 --cpu-seconds 0 > $OUT/bench_c3.json 2> $OUT/c3.err && echo c3 ok &&
timeout -k 10 240 python -u bench.py --config c4 --steps 4 --warmup 1 --e2e 0 --cpu-seconds 0 > $OUT/bench_c4_1048576.json 2> $OUT/c4.err && echo c4 ok &&
timeout -k 10 240 python -u bench.py --config c5 --total-series 262144 --steps 1 --warmup 0 --e2e 0 --cpu-seconds 0 > $OUT/bench_c5_262144.json 2> $OUT/c5.err && echo c5 ok &&
timeout -k 10 200 python -u bench.py --smear 0 --steps 10 --warmup 2 --e2e 0 --cpu-seconds 0 > $OUT/bench_shift.json 2> $OUT/shift.err && echo shift ok &&
CONFIG=c4 SER=131072 OUT=$OUT/prof_c4 bash tools/profile.sh > $OUT/prof_c4.log 2>&1 && echo c4 prof ok
