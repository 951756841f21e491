#!/bin/bash
# Quick A/B: the C3 bench line, then per-kernel average times from a short rocprofv3 --kernel-trace --stats run.
# Usage (GPU box, repo root): bash tools/gpu_quickprof.sh TAG [bench args...]
set -o pipefail
TAG=${1:-qp}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --no-secondary "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); r=d.get('roofline') or {}
print('value', d['value'], 'knn', r.get('avg_us'), 'geom', r.get('knn_geometry_avg_us'), 'lm', r.get('lm_solve_avg_us'), 'pose', d.get('pose_vs_oracle'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p -o run -- \
    python3 bench.py --steps 30 --cpu-baseline-seconds 0 --no-roofline --no-secondary "$@" > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 - "$OUT/p/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name'].replace('floam::(anonymous namespace)::', '').replace('void ', '').split('(')[0][:40]
    print(f"{n:42s} calls {int(r['Calls']):6d} avg {float(r['AverageNs'])/1e3:8.2f} us  total {float(r['TotalDurationNs'])/1e6:8.2f} ms")
PY
