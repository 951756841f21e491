#!/bin/bash
# Per-scan pose agreement with the oracle at C5 for prebuilt library variants (FLOAM_BENCH_POSE_LOG).
# Usage (GPU box): bash tools/gpu_c5_pose.sh variant...
set -o pipefail
mkdir -p gpurun_out/c5pose
for v in "$@"; do
  cp floam_amd/libfloam_amd_$v.so floam_amd/libfloam_amd.so
  FLOAM_BENCH_POSE_LOG=1 timeout -k 10 400 python bench.py --config c5 --cpu-baseline-seconds 25 --no-roofline --no-secondary \
      > gpurun_out/c5pose/$v.json 2> gpurun_out/c5pose/$v.err || { tail -5 gpurun_out/c5pose/$v.err; exit 1; }
  echo "$v $(cut -c1-60 gpurun_out/c5pose/$v.json | grep -o '"value": [0-9.]*')"
  grep "\[pose\]" gpurun_out/c5pose/$v.err | awk '$4 > 1e-9' | head -5
done
