#!/bin/bash
# focused tests of the LM / lookback changes, the ticket A/B and the control-step stamps
set -o pipefail
TAG=${1:-r4j}
step() { "$@"; rc=$?; case $rc in 0|1) return 0;; *) echo "stopping: rc $rc"; exit $rc;; esac; }
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stages.py \
    tests/test_gpu_parity.py tests/test_gpu_controls.py tests/test_gpu_mapmerge.py tests/test_gpu_voxel.py \
    > gpurun_out/$TAG/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$TAG/pytest.log
case $rc in 0|1) ;; *) echo "stopping: rc $rc"; exit $rc;; esac
step bash tools/gpu_envab.sh ${TAG}_ab D:FLOAM_X=0 I:FLOAM_TILE_BY_INDEX=1
NO_AB=1 bash tools/gpu_r4diag.sh ${TAG}
