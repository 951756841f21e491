#!/bin/bash
# GPU tests, A/B tree vs 27c702f and ceb8cfd (prologue loads hoisted above the ticket barrier), kernel stats of the tree.
set -o pipefail
TAG=${1:-r4z}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log
case $rc in 0) ;; *) echo "stopping: rc $rc"; exit $rc;; esac
bash tools/gpu_libab.sh ${TAG}_ab 27c702f ceb8cfd || exit $?
echo all-done
