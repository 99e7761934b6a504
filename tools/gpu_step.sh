#!/bin/bash
# One GPU session step list (round 2): each step under its own time limit, stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
for step in "$@"; do
  case $step in
    passbench) timeout -k 10 240 ./tools/pass_bench ${PASSES:-20} > $OUT/pass_bench.txt 2>&1 ;;
    tests)     timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 ;;
    smoke)     timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 ;;
    bench)     timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 > $OUT/bench.json 2> $OUT/bench.err ;;
    bench_shift) timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --smear 0 --cpu-seconds 0 > $OUT/bench_shift.json 2> $OUT/bench_shift.err ;;
    devtests)  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c2_batch or full_size or golden_fixture and (p2d1q2i1 or c2_212 or kat_mt10_212 or p2d0q2i1 or p2d2q2i1) and not shift" > $OUT/pytest_dev.log 2>&1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $step rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
