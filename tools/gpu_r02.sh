#!/bin/bash
# round-2 GPU steps (run from the repo root via gpurun); each step under its own limit, stop at the first failure
set -o pipefail
OUT=gpurun_out/${TAG:-r02}
mkdir -p $OUT
for step in "$@"; do
  case $step in
    newtests) timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "host_path or pipelined or c4_T4096" > $OUT/newtests.log 2>&1 ;;
    tests)    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 ;;
    smoke)    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 ;;
    bench)    timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup 2 > $OUT/bench.json 2> $OUT/bench.err ;;
    bench_p1) timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --pipeline 1 --e2e 0 --cpu-seconds 0 > $OUT/bench_p1.json 2> $OUT/bench_p1.err ;;
    bench_p3) timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --pipeline 3 --e2e 0 --cpu-seconds 0 > $OUT/bench_p3.json 2> $OUT/bench_p3.err ;;
    bench_c4) timeout -k 10 600 python bench.py --config c4 --series ${C4SER:-131072} --steps 2 --warmup 1 --e2e 0 --cpu-seconds 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err ;;
    sweep)    for P in 2 3; do for XB in 16 32 64; do
                timeout -k 10 200 python bench.py --steps 10 --warmup 2 --pipeline $P --express-blocks $XB --e2e 0 --cpu-seconds 0 > $OUT/sweep_p${P}_x${XB}.json 2> $OUT/sweep_p${P}_x${XB}.err || exit $?
              done; done ;;
    search)   timeout -k 10 700 python tools/bench_search.py --series ${SSER:-262144} --lanes ${SLANES:-4} > $OUT/search.json 2> $OUT/search.err ;;
    prof_c4)  (cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT:-/root/repo}" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4 -o run --output-format csv -- python3 bench.py --config c4 --series ${C4SER:-131072} --steps 1 --warmup 1 --pipeline 1 --e2e 0 --cpu-seconds 0 > $OUT/prof_c4.json 2> $OUT/prof_c4.err) ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $step rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
