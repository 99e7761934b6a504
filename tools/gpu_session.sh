#!/bin/bash
# One GPU session on the box (run ON the GPU box from the repo root, via gpurun). Steps, each under its own time
# limit and chained with && so the first failure ends the session:
#   TESTS=1        python -m pytest tests -m gpu          -> $OUT/pytest_gpu.log   (SEL=... adds a -k filter)
#   SMOKE=1        __graft_entry__.smoke()                -> $OUT/smoke.log
#   BENCH="args"   python bench.py <args>                 -> $OUT/bench.json (+ .err)   (BENCH2/BENCH3 likewise)
#   PROF=1         tools/profile.sh (kernel trace + PMC passes of the C2 bench; CONFIG/SER as there) -> $OUT/prof
# OUT defaults to gpurun_out/r06/<TAG>. Every record kept under profiles/ names the TAG of the session it came from.
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r06/${TAG:-s}
mkdir -p "$OUT"
sha256sum spark-timeseries_amd/libsparkts_arima.so > "$OUT/library.sha256"
ok=0
run_tests() {
    [ "${TESTS:-0}" = 1 ] || return 0
    timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread ${SEL:+-k "$SEL"} \
        > "$OUT/pytest_gpu.log" 2>&1
}
run_smoke() {
    [ "${SMOKE:-0}" = 1 ] || return 0
    timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
}
run_bench() {   # $1 = args, $2 = name
    [ -n "$1" ] || return 0
    timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py $1 > "$OUT/$2.json" 2> "$OUT/$2.err"
}
run_prof() {
    [ "${PROF:-0}" = 1 ] || return 0
    OUT=$OUT/prof bash tools/profile.sh > "$OUT/profile.log" 2>&1
}
run_tests && run_smoke && run_bench "$BENCH" bench && run_bench "$BENCH2" bench2 && run_bench "$BENCH3" bench3 && run_prof
rc=$?
echo "session rc=$rc" > "$OUT/rc.txt"
exit $rc
