#!/bin/bash
# express workgroups (CUs' worth) vs C2 isolated launch and pipelined throughput
set -o pipefail
OUT=gpurun_out/${TAG:-r03/xb}
mkdir -p $OUT
for xb in ${XBS:-16 32 64 96}; do
  timeout -k 10 300 python bench.py --steps 12 --warmup 2 --e2e 0 --cpu-seconds 0 --express-blocks $xb > $OUT/c2_xb$xb.json 2>> $OUT/err.log || exit 1
  echo "xb $xb ok"
done
