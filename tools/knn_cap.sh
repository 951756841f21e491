#!/bin/bash
# kNN grid-cap sweep (tuning): bench with FLOAM_KNN_MAXBLOCKS = each argument, roofline replay on.
set -o pipefail
mkdir -p gpurun_out/cap
for c in "$@"; do
  FLOAM_KNN_MAXBLOCKS=$c timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 > gpurun_out/cap/b$c.json 2> gpurun_out/cap/b$c.err || { tail -5 gpurun_out/cap/b$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/cap/b$c.json')); r=d['roofline']; print('cap $c', d['value'], d['ms_per_step'], r['avg_us'], r['correspondence_pass_avg_us'], r['knn_geometry_avg_us'])"
done
