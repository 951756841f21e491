#!/bin/bash
# tools/golden_trace.py with the tree's library and with the prebuilt variants named (floam_amd/ab/), one process each
set -o pipefail
mkdir -p gpurun_out/golden_trace
cp floam_amd/libfloam_amd.so /tmp/lib_tree.so
for v in tree "$@"; do
  if [ $v = tree ]; then cp /tmp/lib_tree.so floam_amd/libfloam_amd.so; else cp floam_amd/ab/libfloam_amd_$v.so floam_amd/libfloam_amd.so; fi
  timeout -k 10 200 python -u tools/golden_trace.py gpurun_out/golden_trace/$v.json > gpurun_out/golden_trace/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/golden_trace/$v.log; cp /tmp/lib_tree.so floam_amd/libfloam_amd.so; exit $rc; }
done
cp /tmp/lib_tree.so floam_amd/libfloam_amd.so
