#!/bin/bash
# A/B of runtime knobs on one box: bash tools/gpu_ab.sh "bench args" name[:VAR=VAL[,VAR=VAL...]] ...
# (each variant: one un-profiled bench.py run; prints name + value)
set -o pipefail
ARGS=$1; shift
mkdir -p gpurun_out/ab
for spec in "$@"; do
  name=${spec%%:*}
  envs=""
  [ "$spec" != "$name" ] && envs=$(echo "${spec#*:}" | tr ',' ' ')
  env $envs timeout -k 10 400 python3 bench.py $ARGS > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err || { tail -5 gpurun_out/ab/$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab/$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['config']['workload'][:40])"
done
