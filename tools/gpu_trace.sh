#!/bin/bash
# Kernel-trace-only profile of the C3 bench (no counters): gpurun_out/<tag>/prof_trace
set -o pipefail
TAG=${1:-trace}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_trace -o run -- \
    python3 bench.py --cpu-baseline-seconds 0 --no-roofline > $OUT/prof_trace.log 2>&1 || { tail -30 $OUT/prof_trace.log; exit 1; }
tail -1 $OUT/prof_trace.log
