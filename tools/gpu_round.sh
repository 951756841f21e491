#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel-trace stats, PMC HBM-byte passes.
# Usage (from the repo root, on the GPU box): bash tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-r01}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== pytest -m gpu"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
echo "== bench"
timeout -k 10 400 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "== rocprofv3 kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_trace -o run -- \
    python3 bench.py --cpu-baseline-seconds 0 "$@" > $OUT/prof_trace.log 2>&1 || { tail -30 $OUT/prof_trace.log; exit 1; }
echo "== rocprofv3 FETCH_SIZE"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/prof_fetch -o run -- \
    python3 bench.py --cpu-baseline-seconds 0 --no-roofline "$@" > $OUT/prof_fetch.log 2>&1 || { tail -30 $OUT/prof_fetch.log; exit 1; }
echo "== rocprofv3 WRITE_SIZE"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/prof_write -o run -- \
    python3 bench.py --cpu-baseline-seconds 0 --no-roofline "$@" > $OUT/prof_write.log 2>&1 || { tail -30 $OUT/prof_write.log; exit 1; }
find $OUT -name '*.csv' | head -20
echo done
