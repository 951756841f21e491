#!/bin/bash
# Round-4 session: full GPU suite, bench + kernel trace, the N = 2 rehearsal on one GPU, the write-back attribution
# and the fused kNN + fit prototype A/B.  A test failure (exit 1) does not stop the later steps; a fault, an abort or
# a time limit (124, 134, 137, 139) does.
set -o pipefail
TAG=${1:-r4f}
step() { "$@"; rc=$?; case $rc in 0|1) return 0;; *) echo "stopping: rc $rc"; exit $rc;; esac; }
step bash tools/gpu_r4.sh $TAG
step bash tools/gpu_n2.sh ${TAG}_n2 --steps 30
[ -n "$WITH_WB" ] && step bash tools/gpu_wb.sh ${TAG}_wb
[ -n "$WITH_FUSED" ] && step bash tools/gpu_envab.sh ${TAG}_fused D:FLOAM_X=0 F1:FLOAM_KNN_FUSED_PROTO=1 F2:FLOAM_KNN_FUSED_PROTO=2
echo all-done
