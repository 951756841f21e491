#!/bin/bash
# Round-end check with an A/B in the same box: GPU suite, smoke, the tree against 4e6356b (grid kernels and key
# producers: speculative first-stride loads, splitter prefetch), then the profile and N = 2 steps of gpu_final.sh.
set -o pipefail
TAG=${1:-r4ab}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log
case $rc in 0) ;; *) echo "stopping: rc $rc"; exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash tools/gpu_libab.sh ${TAG}_ab 4e6356b || exit $?
bash tools/gpu_prof.sh ${TAG}_prof || exit $?
bash tools/gpu_n2.sh ${TAG}_n2 || exit $?
echo all-done
