#!/bin/bash
# focused tests after the scratch removals, then the write-back attribution and the full counter profile
set -o pipefail
TAG=${1:-r4k}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_voxel.py \
    tests/test_gpu_mapmerge.py tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_controls.py \
    > gpurun_out/$TAG/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$TAG/pytest.log
case $rc in 0) ;; *) echo "stopping: rc $rc"; exit $rc;; esac
bash tools/gpu_wb.sh ${TAG}_wb || exit $?
bash tools/gpu_prof.sh ${TAG}_prof --cpu-baseline-seconds 3 || exit $?
echo all-done
