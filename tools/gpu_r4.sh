#!/bin/bash
# Round-4 GPU session: focused tests first (fail fast), the whole GPU suite, the bench, and a rocprofv3 kernel trace
# of the bench (per-kernel stats + the main-stream timeline).  Usage: bash tools/gpu_r4.sh TAG [bench args...]
set -o pipefail
TAG=${1:-r4}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
if [ -n "$FOCUS" ]; then
  echo "== focused: $FOCUS"
  timeout -k 10 600 $PYT $FOCUS > $OUT/pytest_focus.log 2>&1; rc=$?; tail -5 $OUT/pytest_focus.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NOFULL" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 $PYT tests -m gpu > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
echo "== bench"
timeout -k 10 400 python bench.py --cpu-baseline-seconds ${CPUS:-3} "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d.get('roofline') or {}
print('scans/s', d['value'], 'ms/step', d['ms_per_step'], 'knn us', r.get('avg_us'), 'geom', r.get('knn_geometry_avg_us'),
      'lm', r.get('lm_solve_avg_us'), 'pose', d.get('pose_vs_oracle'))
print('secondary', json.dumps(d.get('secondary')))
PY
if [ -z "$NOPROF" ]; then
  echo "== rocprofv3 kernel trace"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_trace -o run -- \
      python3 bench.py --cpu-baseline-seconds 0 --no-secondary --no-roofline "$@" > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  f=$(find $OUT/prof_trace -name '*kernel_trace.csv' | head -1)
  python tools/timeline.py $f 10 > $OUT/timeline.txt 2>&1 || true
  tail -25 $OUT/timeline.txt
fi
echo done
