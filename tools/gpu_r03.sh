#!/bin/bash
# round-3 GPU steps (run from the repo root via gpurun); each step under its own limit, stop at the first failure
set -o pipefail
OUT=gpurun_out/${TAG:-r03}
mkdir -p $OUT
for step in "$@"; do
  case $step in
    tests)    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 ;;
    smoke)    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 ;;
    bench)    timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup 2 > $OUT/bench.json 2> $OUT/bench.err ;;
    bench_q)  timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --e2e 0 --cpu-seconds 0 > $OUT/bench_q.json 2> $OUT/bench_q.err ;;
    bench_shift) timeout -k 10 300 python bench.py --smear 0 --steps ${STEPS:-10} --warmup 2 --e2e 0 --cpu-seconds 0 > $OUT/bench_shift.json 2> $OUT/bench_shift.err ;;
    bench_c4) timeout -k 10 600 python bench.py --config c4 --series ${C4SER:-131072} --steps ${C4STEPS:-2} --warmup 1 --e2e 0 --cpu-seconds 0 > $OUT/bench_c4_${C4SER:-131072}.json 2> $OUT/bench_c4_${C4SER:-131072}.err ;;
    bench_c3) timeout -k 10 900 python bench.py --total-series 8388608 --steps ${C3STEPS:-2} --warmup 1 --e2e 0 --cpu-seconds 0 > $OUT/bench_c3.json 2> $OUT/bench_c3.err ;;
    c5)       timeout -k 10 900 python bench.py --config c5 --total-series ${C5SER:-65536} --steps 1 --warmup 0 > $OUT/bench_c5_${C5SER:-65536}.json 2> $OUT/bench_c5_${C5SER:-65536}.err ;;
    grid)     timeout -k 10 900 python tools/grid_profile.py --series ${GSER:-65536} > $OUT/grid_${GSER:-65536}.jsonl 2> $OUT/grid.err ;;
    pmc)      OUT=$OUT/pmc_${CONFIG:-c2} SER=${PSER:-1048576} timeout -k 10 1000 tools/profile.sh > $OUT/pmc_${CONFIG:-c2}.log 2>&1 ;;
    search)   timeout -k 10 700 python tools/bench_search.py --series ${SSER:-262144} > $OUT/search.json 2> $OUT/search.err ;;
    prof_c4)  (cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT:-/root/repo}" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4 -o run --output-format csv -- python3 bench.py --config c4 --series ${C4SER:-131072} --steps 1 --warmup 1 --pipeline 1 --e2e 0 --cpu-seconds 0 > $OUT/prof_c4.json 2> $OUT/prof_c4.err) ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $step rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
