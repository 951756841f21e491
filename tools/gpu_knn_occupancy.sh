#!/bin/bash
# The kNN search at lower occupancy (VERDICT r05 item 2's role-split launch: one kernel that also runs the geometry
# fits is allocated the geometry's 118 VGPRs, i.e. 4 waves per SIMD instead of the search's 6): dynamic LDS pads
# (FLOAM_KNN_LDS_PAD, diagnostic build) cap the search's blocks per CU at 6 (no pad), 5 and 4; C3 bench with the
# roofline replay (kNN µs by kernel events), two rounds.  Usage: bash tools/gpu_knn_occupancy.sh TAG [bench args]
set -o pipefail
OUT=gpurun_out/${1:-knnocc}; shift || true
mkdir -p $OUT
export TMPDIR=/tmp FLOAM_AMD_LIB=diag
for round in 1 2; do
  for pad in 0 24640 32768; do
    FLOAM_KNN_LDS_PAD=$pad timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --no-secondary "$@" \
        > $OUT/pad${pad}_$round.json 2> $OUT/pad${pad}_$round.err || { tail -20 $OUT/pad${pad}_$round.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/pad${pad}_$round.json')); r=d['roofline']; print('pad $pad', '$round', d['value'], 'knn', r['avg_us'], 'geom', r.get('knn_geometry_avg_us'), 'lm', r.get('lm_solve_avg_us'))"
  done
done
echo done
