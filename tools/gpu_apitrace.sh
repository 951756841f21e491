#!/bin/bash
# HIP API trace (no counters) of the C3 bench: gpurun_out/<tag>/api
set -o pipefail
TAG=${1:-api}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $OUT/api -o run -- \
    python3 bench.py --cpu-baseline-seconds 0 --no-roofline --no-secondary > $OUT/api.log 2>&1 || { tail -30 $OUT/api.log; exit 1; }
tail -1 $OUT/api.log | cut -c1-120
