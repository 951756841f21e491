#!/bin/bash
# Tuning sweep of the kNN kernel variants (FLOAM_KNN_VARIANT) on the C3 bench; prints per-variant timings.
set -o pipefail
mkdir -p gpurun_out/var
for v in ${VARIANTS:-0 1 2 3 4 6 7 8}; do
  FLOAM_KNN_VARIANT=$v timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 > gpurun_out/var/v$v.json 2> gpurun_out/var/v$v.err || { tail -5 gpurun_out/var/v$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/var/v$v.json')); r=d['roofline']
print('variant $v', d['ms_per_step'], 'ms/step', r['avg_us'], r['correspondence_pass_avg_us'], r.get('knn_geometry_avg_us'), d['pose_vs_oracle'] if d['pose_vs_oracle'] else '')"
done
