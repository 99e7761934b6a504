#!/bin/bash
# rocprofv3 passes over tools/fit_diag.py (one C2 fit; ON the GPU box, repo root). Each PMC pass is its own run
# with --kernel-trace only (MI355X_MICROARCH.md: one pass holds <= 8 SQ / 4 TCC / 2 GRBM counters).
#   TAG=name LIB=path/to/lib.so tools/profile_fit.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-prof}
mkdir -p $OUT
[ -n "${LIB:-}" ] && export SPARKTS_ARIMA_LIB=$LIB
ARGS=${ARGS:-"--reps 1"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- \
    python3 tools/fit_diag.py $ARGS > $OUT/diag.json 2> $OUT/diag.err
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    -d $OUT/prof_sq -o run --output-format csv -- python3 tools/fit_diag.py $ARGS > /dev/null 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $OUT/prof_fetch -o run --output-format csv -- \
    python3 tools/fit_diag.py $ARGS > /dev/null 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/prof_write -o run --output-format csv -- \
    python3 tools/fit_diag.py $ARGS > /dev/null 2>&1
python3 tools/summarize_prof.py $OUT $OUT/summary.txt
