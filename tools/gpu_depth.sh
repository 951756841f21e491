#!/bin/bash
# Pipeline-depth sweep of the C3 bench (updates in flight = the host's lead over the device).
set -o pipefail
mkdir -p gpurun_out/depth
for d in 2 3; do
  FLOAM_BENCH_DEPTH=$d FLOAM_BENCH_HOST=1 timeout -k 10 240 python bench.py --cpu-baseline-seconds 0 --no-roofline \
    > gpurun_out/depth/d$d.json 2> gpurun_out/depth/d$d.err || { tail -20 gpurun_out/depth/d$d.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/depth/d$d.json')); print('depth $d', d['value'], d['ms_per_step'])"
  grep host gpurun_out/depth/d$d.err
done
