#!/bin/bash
# Round-4 diagnostics: write-back attribution, the fused kNN + fit prototype A/B (item 4) and
# the control-step segment stamps (item 8; a scratch rebuild with -DFLOAM_CTRL_STAMPS, last: it replaces the .so).
set -o pipefail
TAG=${1:-diag}
step() { "$@"; rc=$?; case $rc in 0|1) return 0;; *) echo "stopping: rc $rc"; exit $rc;; esac; }
export TMPDIR=/tmp
[ -n "$WITH_WB" ] && step bash tools/gpu_wb.sh ${TAG}_wb
[ -z "$NO_AB" ] && step bash tools/gpu_envab.sh ${TAG}_ab D:FLOAM_X=0 I:FLOAM_TILE_BY_INDEX=1 F1:FLOAM_KNN_FUSED_PROTO=1 F2:FLOAM_KNN_FUSED_PROTO=2
OUT=gpurun_out/${TAG}_ctrl
mkdir -p $OUT
timeout -k 10 600 make -C floam_amd/csrc -j16 OBJDIR=/tmp/floam_ctrl_obj EXTRA=-DFLOAM_CTRL_STAMPS > $OUT/make.log 2>&1 \
    || { tail -20 $OUT/make.log; exit 1; }
FLOAM_DEBUG_STAMPS=1 timeout -k 10 300 python bench.py --steps 40 --cpu-baseline-seconds 0 --no-secondary --no-roofline \
    > $OUT/ctrl.json 2> $OUT/ctrl.err || { tail -20 $OUT/ctrl.err; exit 1; }
grep -E "floam ctrl|floam stamps" $OUT/ctrl.err
echo all-done
