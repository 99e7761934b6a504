#!/bin/bash
# Profile the headline bench with rocprofv3 (run ON the GPU box, from the repo root):
#   1) kernel trace + stats  -> gpurun_out/prof_trace/...  (per-kernel average durations)
#   2) PMC pass: FETCH_SIZE, WRITE_SIZE (HBM traffic) -> gpurun_out/prof_pmc/...
#   3) PMC pass: SQ counters (VALU / waves / wait) -> gpurun_out/prof_sq/...
# PASSES (default "trace fetch write sq sqwait tcc") picks the runs; each is its own rocprofv3 run under a time limit.
# Counters are collected in their own runs with --kernel-trace only (no sys/runtime trace), per the guide.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SER=${SER:-1048576}
OUT=${OUT:-gpurun_out}
CFG=${CONFIG:-c2}
PASSES=" ${PASSES:-trace fetch write sq sqwait tcc} "
mkdir -p $OUT
has() { [[ "$PASSES" == *" $1 "* ]]; }
has trace && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- \
    python3 bench.py --config $CFG --series $SER --steps 2 --warmup 1 --cpu-seconds 0 --pipeline 1 --e2e 0 --default-leg 0 > $OUT/prof_bench.json 2> $OUT/prof_bench.err
has fetch && timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/prof_fetch -o run --output-format csv -- \
    python3 bench.py --config $CFG --series $SER --steps 1 --warmup 0 --cpu-seconds 0 --pipeline 1 --e2e 0 --default-leg 0 > /dev/null 2>&1
has write && timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/prof_write -o run --output-format csv -- \
    python3 bench.py --config $CFG --series $SER --steps 1 --warmup 0 --cpu-seconds 0 --pipeline 1 --e2e 0 --default-leg 0 > /dev/null 2>&1
has sq && timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/prof_sq -o run --output-format csv -- \
    python3 bench.py --config $CFG --series $SER --steps 1 --warmup 0 --cpu-seconds 0 --pipeline 1 --e2e 0 --default-leg 0 > /dev/null 2>&1
has sqwait && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d $OUT/prof_sqwait -o run --output-format csv -- \
    python3 bench.py --config $CFG --series $SER --steps 1 --warmup 0 --cpu-seconds 0 --pipeline 1 --e2e 0 --default-leg 0 > /dev/null 2>&1
has tcc && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/prof_tcc -o run --output-format csv -- \
    python3 bench.py --config $CFG --series $SER --steps 1 --warmup 0 --cpu-seconds 0 --pipeline 1 --e2e 0 --default-leg 0 > /dev/null 2>&1
exit 0
