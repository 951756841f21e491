#!/bin/bash
# Quick GPU check after a kernel change: GPU parity tests, then the C3 bench (roofline replay on, short CPU leg).
set -o pipefail
mkdir -p gpurun_out/q
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/q/pytest.log; [ $rc -eq 0 ] || exit $rc
FLOAM_BENCH_HOST=1 timeout -k 10 300 python bench.py --cpu-baseline-seconds 2 "$@" > gpurun_out/q/bench.json 2> gpurun_out/q/bench.err || { tail -20 gpurun_out/q/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/q/bench.json')); r=d['roofline']
print('scans/s', d['value'], 'ms/step', d['ms_per_step'], 'knn avg us', r['avg_us'], 'frac', r['frac'], 'corr pass', r['correspondence_pass_avg_us'], 'geom', r['knn_geometry_avg_us'], 'pose', d['pose_vs_oracle'])"
grep host gpurun_out/q/bench.err
if [ -n "$STAMPS" ]; then FLOAM_DEBUG_STAMPS=1 timeout -k 10 200 python bench.py --steps 20 --cpu-baseline-seconds 0 --no-roofline > gpurun_out/q/st.json 2> gpurun_out/q/st.err; grep stamps gpurun_out/q/st.err | head -3; fi
