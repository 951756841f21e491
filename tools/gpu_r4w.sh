#!/bin/bash
# GPU tests (speculative geometry loads), A/B tree vs 648109f, compaction stamps.
set -o pipefail
TAG=${1:-r4t}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log
case $rc in 0) ;; *) echo "stopping: rc $rc"; exit $rc;; esac
NO_TRACE=1 bash tools/gpu_libab.sh ${TAG}_ab 648109f || exit $?
FLOAM_BC_STAMPS=1 timeout -k 10 300 python bench.py --steps 30 --cpu-baseline-seconds 0 --no-roofline --no-secondary \
    > $OUT/st.json 2> $OUT/st.err || { tail -20 $OUT/st.err; exit 1; }
grep -E "stamps\]" $OUT/st.err
echo all-done
