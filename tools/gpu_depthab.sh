#!/bin/bash
# Pipeline depth A/B of the C3 bench (FLOAM_BENCH_DEPTH 2 vs 3), host issue / wait split, then a kernel-trace timeline
# of each.  Usage: bash tools/gpu_depthab.sh TAG
set -o pipefail
O=gpurun_out/${1:-depth}; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2 3; do
  for d in 2 3; do
    FLOAM_BENCH_DEPTH=$d FLOAM_BENCH_HOST=1 timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-secondary \
        > $O/b_d${d}_$r.json 2> $O/b_d${d}_$r.err || { tail -20 $O/b_d${d}_$r.err; exit 1; }
    echo "depth $d round $r $(python -c "import json; print(json.load(open('$O/b_d${d}_$r.json'))['value'])") $(grep '\[host\]' $O/b_d${d}_$r.err)"
  done
done
for d in 2 3; do
  FLOAM_BENCH_DEPTH=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_d$d -o run -- \
      python3 bench.py --cpu-baseline-seconds 0 --no-secondary --no-roofline > $O/tr_d$d.log 2>&1 || { tail -20 $O/tr_d$d.log; exit 1; }
  f=$(find $O/tr_d$d -name '*kernel_trace.csv' | head -1)
  python tools/timeline.py $f 40 > $O/timeline_d$d.txt 2>&1 || true
  echo "== depth $d"; tail -1 $O/timeline_d$d.txt
done
