#!/bin/bash
# Run tools/variant_run.py for every dev library named in $VARIANTS (space separated tags) on the GPU box,
# then optional extra commands from $EXTRA. Each run has its own time limit; the chain stops at the first failure.
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/variants.jsonl
# an entry is TAG or TAG@opt=value (a runtime option for that run)
for e in $VARIANTS; do
    t=${e%%@*}
    o=""; [ "$e" != "$t" ] && o="--opt ${e#*@}"
    SPARKTS_ARIMA_LIB=spark-timeseries_amd/libsparkts_arima_dev_$t.so timeout -k 10 120 \
        python -u tools/variant_run.py ${VARGS:-} $o >> gpurun_out/variants.jsonl 2> gpurun_out/variant_$t.err || exit 1
done
if [ -n "${EXTRA:-}" ]; then bash -c "$EXTRA" || exit 1; fi
cat gpurun_out/variants.jsonl
