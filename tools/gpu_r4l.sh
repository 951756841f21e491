#!/bin/bash
# Round-4 re-entry check of HEAD: the whole -m gpu suite, smoke, the write-back attribution, then the profiled bench.
# Usage: bash tools/gpu_r4l.sh TAG
set -o pipefail
TAG=${1:-r4l}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$TAG/pytest_gpu.log
case $rc in 0) ;; *) echo "stopping: rc $rc"; exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -2 gpurun_out/$TAG/smoke.log
bash tools/gpu_wb.sh ${TAG}_wb || exit $?
bash tools/gpu_prof.sh ${TAG}_prof --cpu-baseline-seconds 3 || exit $?
bash tools/gpu_knn_stages.sh ${TAG}_ks || exit $?
timeout -k 10 200 hipcc -O3 -std=c++17 -ffp-contract=fast --offload-arch=gfx950 tools/micro/lm_ctrl.hip -o /tmp/lm_ctrl \
    > gpurun_out/$TAG/lm_ctrl_build.log 2>&1 && timeout -k 10 60 /tmp/lm_ctrl > gpurun_out/$TAG/lm_ctrl.txt 2>&1; cat gpurun_out/$TAG/lm_ctrl.txt
bash tools/gpu_stamps.sh ${TAG}_st || exit $?
echo all-done
