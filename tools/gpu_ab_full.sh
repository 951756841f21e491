#!/bin/bash
# The whole GPU suite under the tree's defaults, then alternating bench runs: base (env $1) vs the default tree
# (scans/s, kNN and geometry launch times).  Usage: bash tools/gpu_ab_full.sh VAR=VAL   (VAR=VAL restores the old path)
set -o pipefail
mkdir -p gpurun_out/abf
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abf/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/abf/pytest.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for v in base:$1 new:X=0; do
    name=${v%%:*}
    env ${v#*:} timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 > gpurun_out/abf/$name$k.json 2> gpurun_out/abf/$name$k.err || { tail -5 gpurun_out/abf/$name$k.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/abf/$name$k.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', d['value'], 'knn us', r['avg_us'], 'geom us', r['knn_geometry_avg_us'], 'pose', d['pose_vs_oracle']['max_dt_m'])"
  done
done
