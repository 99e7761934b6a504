#!/bin/bash
# Row-stride A/B (option row_pad, doubles added to the differenced rows' 8-KB / 32-KB power-of-two stride):
#   isolated launches (--pipeline 1, kernel_ms = HIP-event time of each kernel alone) and the pipelined headline
#   step (default contexts), C2 and a C4 slice. Run ON the GPU box from the repo root.
set -o pipefail
OUT=gpurun_out/${TAG:-r03/rowpad}
mkdir -p $OUT
ISO="python bench.py --steps 2 --warmup 1 --pipeline 1 --e2e 0 --cpu-seconds 0"
PIPE="python bench.py --steps 10 --warmup 3 --e2e 0 --cpu-seconds 0"
for r in ${PADS:-0 16 32 64}; do
  SPARKTS_OPTIONS=row_pad=$r timeout -k 10 120 $ISO > $OUT/c2_iso_pad$r.json 2>> $OUT/err.log || exit 1
  SPARKTS_OPTIONS=row_pad=$r timeout -k 10 120 $PIPE > $OUT/c2_pipe_pad$r.json 2>> $OUT/err.log || exit 1
  echo "pad $r done"
done
for r in ${C4PADS:-0 16}; do
  SPARKTS_OPTIONS=row_pad=$r timeout -k 10 300 $ISO --config c4 --series 262144 --steps 1 > $OUT/c4_iso_pad$r.json 2>> $OUT/err.log || exit 1
  echo "c4 pad $r done"
done
