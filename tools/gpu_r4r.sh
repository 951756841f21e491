#!/bin/bash
# Untraced host split (issue / wait per scan) at depth 2 and 3, and with graph capture if the knob exists.
set -o pipefail
TAG=${1:-r4r}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
for v in d2 d3 d2b; do
  E="FLOAM_BENCH_HOST=1"; [ $v = d3 ] && E="$E FLOAM_BENCH_DEPTH=3"
  env $E FLOAM_BENCH_HOST_TRACE=$OUT/host_$v.json timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-secondary \
      --no-roofline > $OUT/b_$v.json 2> $OUT/b_$v.err || { tail -20 $OUT/b_$v.err; exit 1; }
  echo "$v $(python -c "import json; print(json.load(open('$OUT/b_$v.json'))['value'])") $(grep '\[host\]' $OUT/b_$v.err)"
done
echo all-done
