#!/bin/bash
# Kernel trace of a short C3 bench at a given pipeline depth (queue timeline analysis).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tdepth
FLOAM_BENCH_DEPTH=${1:-3} timeout -k 10 300 rocprofv3 --kernel-trace ${HIPTRACE:+--hip-trace} --output-format csv -d gpurun_out/tdepth/raw -o run -- \
  python3 bench.py --steps 30 --warmup 8 --cpu-baseline-seconds 0 --no-roofline > gpurun_out/tdepth/b.json 2> gpurun_out/tdepth/b.err
rc=$?
f=$(find gpurun_out/tdepth/raw -name '*kernel_trace.csv' | head -n 1)
[ -n "$f" ] && cp "$f" gpurun_out/tdepth/kernel_trace.csv
h=$(find gpurun_out/tdepth/raw -name "*hip_api_trace.csv" | head -n 1)
[ -n "$h" ] && cp "$h" gpurun_out/tdepth/hip_api_trace.csv
cat gpurun_out/tdepth/b.json
exit $rc
