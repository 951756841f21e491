#!/bin/bash
# A/B of prebuilt library variants on one box: floam_amd/libfloam_amd_<name>.so copied over libfloam_amd.so before
# each C3 bench run (no secondary lines, no CPU leg).  Usage (GPU box): bash tools/gpu_ab.sh base variant1 ... base
set -o pipefail
mkdir -p gpurun_out/ab
for v in "$@"; do
  cp floam_amd/libfloam_amd_$v.so floam_amd/libfloam_amd.so
  timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-secondary > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || { tail -5 gpurun_out/ab/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$v.json')); r=d['roofline']; print('$v', d['value'], r['avg_us'], r['knn_geometry_avg_us'], r['lm_solve_avg_us'], d['pose_vs_oracle'])"
done
wc -l gpurun_out/ab/base.json
