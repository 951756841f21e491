#!/bin/bash
# Host issue timestamps (FLOAM_BENCH_HOST_TRACE, CLOCK_MONOTONIC) beside a kernel trace of the same run.
set -o pipefail
TAG=${1:-r4q}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
FLOAM_BENCH_HOST=1 FLOAM_BENCH_HOST_TRACE=$OUT/host_trace.json timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
    -d $OUT/tr -o run -- python3 bench.py --cpu-baseline-seconds 0 --no-secondary --no-roofline > $OUT/tr.log 2>&1 \
    || { tail -20 $OUT/tr.log; exit 1; }
grep -E "\[host\]" $OUT/tr.log
echo all-done
