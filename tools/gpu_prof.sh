#!/bin/bash
# Bench + rocprofv3 kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE passes of the same bench command (no
# tests; the device-code hash of the tree into code_hash.txt).  Usage (GPU box, repo root): bash tools/gpu_prof.sh TAG
# [bench args...]; then on the host python tools/prof_summary.py gpurun_out/TAG TAG --config <config> --steps <steps>
set -o pipefail
TAG=${1:-prof}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
python -c "import bench; print(bench.code_hash())" > $OUT/code_hash.txt
timeout -k 10 400 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_trace -o run -- \
    python3 bench.py --cpu-baseline-seconds 0 --no-secondary "$@" > $OUT/prof_trace.log 2>&1 || { tail -30 $OUT/prof_trace.log; exit 1; }
[ -n "$PROF_TRACE_ONLY" ] && { echo done; exit 0; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/prof_fetch -o run -- \
    python3 bench.py --cpu-baseline-seconds 0 --no-roofline --no-secondary "$@" > $OUT/prof_fetch.log 2>&1 || { tail -30 $OUT/prof_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/prof_write -o run -- \
    python3 bench.py --cpu-baseline-seconds 0 --no-roofline --no-secondary "$@" > $OUT/prof_write.log 2>&1 || { tail -30 $OUT/prof_write.log; exit 1; }
echo done
