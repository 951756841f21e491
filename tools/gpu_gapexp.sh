#!/bin/bash
# Stream-gap experiment: kernel traces of the C3 bench under runtime knobs.  Usage: bash tools/gpu_gapexp.sh
# name[:VAR=VAL[,VAR=VAL...]] ...   (then /tmp/gaps.py-style analysis of gpurun_out/gap_<name>/prof_trace)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for spec in "$@"; do
  name=${spec%%:*}
  envs=""
  [ "$spec" != "$name" ] && envs=$(echo "${spec#*:}" | tr ',' ' ')
  mkdir -p gpurun_out/gap_$name
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap_$name/prof_trace -o run -- \
    python3 bench.py --cpu-baseline-seconds 0 --no-secondary --no-roofline > gpurun_out/gap_$name/bench.json 2> gpurun_out/gap_$name/err.log || { tail -5 gpurun_out/gap_$name/err.log; exit 1; }
  echo "$name $(cut -c1-120 gpurun_out/gap_$name/bench.json)"
done
