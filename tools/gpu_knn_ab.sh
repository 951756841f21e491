#!/bin/bash
# kNN variant A/B on one box: the stage / odometry parity tests under the variant, then alternating bench runs
# (scans/s and the kNN's HIP-event launch time).  Usage: bash tools/gpu_knn_ab.sh VAR=VAL
set -o pipefail
mkdir -p gpurun_out/kab
env $1 timeout -k 10 500 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_parity.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/kab/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/kab/pytest.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for v in base:X=0 var:$1; do
    name=${v%%:*}
    env ${v#*:} timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 > gpurun_out/kab/$name$k.json 2> gpurun_out/kab/$name$k.err || { tail -5 gpurun_out/kab/$name$k.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/kab/$name$k.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', d['value'], 'knn us', r['avg_us'], 'frac', r['frac'])"
  done
done
