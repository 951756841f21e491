#!/bin/bash
# A/B of the tree's library against prebuilt ones (floam_amd/ab/libfloam_amd_<NAME>.so, built on the host from other
# commits): the C3 bench alternating over the variants, two rounds, then a kernel-trace timeline of each.
# Usage: bash tools/gpu_libab.sh TAG NAME...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cp floam_amd/libfloam_amd.so /tmp/lib_tree.so
trap 'cp /tmp/lib_tree.so floam_amd/libfloam_amd.so' EXIT
use() { if [ "$1" = tree ]; then cp /tmp/lib_tree.so floam_amd/libfloam_amd.so; else cp floam_amd/ab/libfloam_amd_$1.so floam_amd/libfloam_amd.so; fi; }
for round in 1 2; do
  for v in tree "$@"; do
    use $v
    timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-secondary > $OUT/b_${v}_$round.json \
        2> $OUT/b_${v}_$round.err || { tail -20 $OUT/b_${v}_$round.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_${v}_$round.json')); r=d['roofline']; print('$v', '$round', d['value'], 'knn', r['avg_us'], 'knn+geom', r['knn_geometry_avg_us'], 'lm', r['lm_solve_avg_us'])"
  done
done
[ -n "$NO_TRACE" ] && { echo done; exit 0; }
for v in tree "$@"; do
  use $v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_$v -o run -- \
      python3 bench.py --cpu-baseline-seconds 0 --no-secondary --no-roofline > $OUT/tr_$v.log 2>&1 || { tail -20 $OUT/tr_$v.log; exit 1; }
  f=$(find $OUT/tr_$v -name '*kernel_trace.csv' | head -1)
  python tools/timeline.py $f 10 > $OUT/timeline_$v.txt 2>&1 || true
  echo "== $v"; tail -2 $OUT/timeline_$v.txt
done
echo done
