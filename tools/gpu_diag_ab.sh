#!/bin/bash
# A diagnostic-build variant (an environment switch read by libfloam_amd_diag.so) against the same library without
# it: the stage / odometry parity tests with the switch on, then bench lines alternating without / with it at each
# config (kNN and pass times from the roofline replay).  Usage: bash tools/gpu_diag_ab.sh TAG VAR [CONFIG...]
#   e.g. bash tools/gpu_diag_ab.sh r06d FLOAM_KNN_SPLIT c3 c5
set -o pipefail
TAG=$1; VAR=$2; shift 2
CFGS=${@:-c3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp FLOAM_AMD_LIB=diag
env $VAR=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_parity.py -x -v \
    --timeout 300 --timeout-method thread -k "knn or odometry or golden or record" > $OUT/pytest_$VAR.log 2>&1 \
    || { tail -30 $OUT/pytest_$VAR.log; exit 1; }
echo "tests with $VAR=1: $(grep -c PASSED $OUT/pytest_$VAR.log) passed"; tail -1 $OUT/pytest_$VAR.log
for cfg in $CFGS; do
  for round in 1 2; do
    for v in base var; do
      E=""; [ $v = var ] && E="$VAR=1"
      env $E timeout -k 10 400 python bench.py --config $cfg --steps 20 --warmup 5 --cpu-baseline-seconds 0 \
          --no-secondary > $OUT/${cfg}_${v}_$round.json 2> $OUT/${cfg}_${v}_$round.err \
          || { tail -20 $OUT/${cfg}_${v}_$round.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/${cfg}_${v}_$round.json')); r=d['roofline']; print('$cfg', '$v', '$round', d['value'], 'knn', r['avg_us'], 'geom', r.get('knn_geometry_avg_us'), 'pass', r.get('correspondence_pass_avg_us'), 'lm', r.get('lm_solve_avg_us'), 'frac', r['frac'], 'same', r['replay_bitwise_identical'], d.get('pose_vs_oracle'))"
    done
  done
done
echo done
