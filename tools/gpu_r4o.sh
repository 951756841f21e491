#!/bin/bash
# GPU tests; A/B alternating: the tree, the previous library (3d1955e), the tree with FLOAM_LM_RPT=2; sort / merge /
# LM stamps; timeline.  Usage: bash tools/gpu_r4o.sh TAG
set -o pipefail
TAG=${1:-r4o}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log
case $rc in 0) ;; *) echo "stopping: rc $rc"; exit $rc;; esac
cp floam_amd/libfloam_amd.so /tmp/lib_tree.so
trap 'cp /tmp/lib_tree.so floam_amd/libfloam_amd.so' EXIT
for round in 1 2; do
  for v in tree prev rpt2; do
    if [ $v = prev ]; then cp floam_amd/ab/libfloam_amd_3d1955e.so floam_amd/libfloam_amd.so; else cp /tmp/lib_tree.so floam_amd/libfloam_amd.so; fi
    E=""; [ $v = rpt2 ] && E="FLOAM_LM_RPT=2"
    env $E timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-secondary > $OUT/b_${v}_$round.json \
        2> $OUT/b_${v}_$round.err || { tail -20 $OUT/b_${v}_$round.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_${v}_$round.json')); r=d['roofline']; print('$v', '$round', d['value'], 'knn', r['avg_us'], 'knn+geom', r['knn_geometry_avg_us'], 'lm', r['lm_solve_avg_us'])"
  done
done
cp /tmp/lib_tree.so floam_amd/libfloam_amd.so
FLOAM_BC_STAMPS=1 FLOAM_MM_STAMPS=1 FLOAM_DEBUG_STAMPS=1 timeout -k 10 300 python bench.py --steps 30 --cpu-baseline-seconds 0 \
    --no-roofline --no-secondary > $OUT/st.json 2> $OUT/st.err || { tail -20 $OUT/st.err; exit 1; }
grep -E "stamps\]" $OUT/st.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o run -- \
    python3 bench.py --cpu-baseline-seconds 0 --no-secondary --no-roofline > $OUT/tr.log 2>&1 || { tail -20 $OUT/tr.log; exit 1; }
python tools/timeline.py $OUT/tr/run_kernel_trace.csv 10 > $OUT/timeline.txt 2>&1; cat $OUT/timeline.txt
echo all-done
