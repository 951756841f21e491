#!/bin/bash
# The golden odometry test (tests/test_golden.py) with the tree's library and each prebuilt variant named
# (floam_amd/ab/libfloam_amd_<NAME>.so), one process each; a fault or a time limit stops the loop.
# Usage: bash tools/gpu_golden_ab.sh NAME...
set -o pipefail
mkdir -p gpurun_out/r05k
cp floam_amd/libfloam_amd.so /tmp/lib_tree.so
for v in tree "$@"; do
  if [ $v = tree ]; then cp /tmp/lib_tree.so floam_amd/libfloam_amd.so; else cp floam_amd/ab/libfloam_amd_$v.so floam_amd/libfloam_amd.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05k/golden_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/r05k/golden_$v.log)"
  case $rc in 0|1) ;; *) cp /tmp/lib_tree.so floam_amd/libfloam_amd.so; exit $rc ;; esac   # (a fault or a time limit: stop)
done
cp /tmp/lib_tree.so floam_amd/libfloam_amd.so
