#!/bin/bash
# Runtime A/B of the C3 bench over environment settings, alternating, two rounds; then a kernel-trace timeline of
# each setting.  Usage: bash tools/gpu_envab.sh TAG "NAME:ENV=V,ENV2=V" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# every A/B and hook variable is read only by the diagnostic build (FLOAM_DIAG_ENV, floam_common.hpp); only FLOAM_GRAPH
# and FLOAM_MAP_MERGE reach the product library.  A spec is measured on the diagnostic library unless it names only those.
for spec in "$@"; do
  for kv in $(echo ${spec#*:} | tr ',' ' '); do
    case ${kv%%=*} in FLOAM_GRAPH|FLOAM_MAP_MERGE|FLOAM_AMD_LIB) ;; *) export FLOAM_AMD_LIB=diag ;; esac
  done
done
echo "library: ${FLOAM_AMD_LIB:-product}"
for round in 1 2; do
  for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    env $(echo $envs | tr ',' ' ') timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-secondary --no-roofline \
        > $OUT/b_${name}_$round.json 2> $OUT/b_${name}_$round.err || { tail -20 $OUT/b_${name}_$round.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_${name}_$round.json')); print('$name', '$round', d['value'])"
  done
done
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  for kv in $(echo $envs | tr ',' ' '); do export $kv; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_$name -o run -- \
      python3 bench.py --cpu-baseline-seconds 0 --no-secondary --no-roofline > $OUT/tr_$name.log 2>&1 || { tail -20 $OUT/tr_$name.log; exit 1; }
  for kv in $(echo $envs | tr ',' ' '); do unset ${kv%%=*}; done
  f=$(find $OUT/tr_$name -name '*kernel_trace.csv' | head -1)
  python tools/timeline.py $f 10 > $OUT/timeline_$name.txt 2>&1 || true
  echo "== $name"; tail -3 $OUT/timeline_$name.txt
done
echo done
