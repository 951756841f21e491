#!/bin/bash
# The LDS-staged stage 1 (odom_kernels.hip knn_kernel_lds, diagnostic build FLOAM_KNN_LDS=1):
# the stage / odometry parity tests with it, then C3 and C5 bench lines (kNN µs by kernel events, algorithmic bytes)
# with and without it, alternating, and a rocprofv3 kernel-trace of each at C5.  Usage: bash tools/gpu_knn_lds.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-knnlds}
mkdir -p $OUT
export TMPDIR=/tmp FLOAM_AMD_LIB=diag
FLOAM_KNN_LDS=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_parity.py -x -v \
    --timeout 300 --timeout-method thread -k "knn or odometry or golden or record" > $OUT/pytest_lds.log 2>&1 \
    || { tail -30 $OUT/pytest_lds.log; exit 1; }
grep -c PASSED $OUT/pytest_lds.log; tail -1 $OUT/pytest_lds.log
for cfg in c3 c5; do
  for round in 1 2; do
    for v in global lds; do
      if [ $v = lds ]; then export FLOAM_KNN_LDS=1; else unset FLOAM_KNN_LDS; fi
      timeout -k 10 400 python bench.py --config $cfg --steps 20 --warmup 5 --cpu-baseline-seconds 0 --no-secondary \
          > $OUT/${cfg}_${v}_$round.json 2> $OUT/${cfg}_${v}_$round.err || { tail -20 $OUT/${cfg}_${v}_$round.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/${cfg}_${v}_$round.json')); r=d['roofline']; print('$cfg', '$v', '$round', d['value'], 'knn', r['avg_us'], 'frac', r['frac'], 'bytes', r['algorithmic_bytes_per_launch'], 'same', r['replay_bitwise_identical'], d.get('pose_vs_oracle'))"
    done
  done
done
unset FLOAM_KNN_LDS
echo done
