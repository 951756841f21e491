#!/bin/bash
# GPU tests, LM micro-benchmark, A/B tree vs 3d1955e (alternating, 2 rounds), LM stamps.
set -o pipefail
TAG=${1:-r4s}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log
case $rc in 0) ;; *) echo "stopping: rc $rc"; exit $rc;; esac
timeout -k 10 200 hipcc -O3 -std=c++17 -ffp-contract=fast --offload-arch=gfx950 tools/micro/lm_ctrl.hip -o /tmp/lm_ctrl \
    > $OUT/lm_ctrl_build.log 2>&1 && timeout -k 10 60 /tmp/lm_ctrl > $OUT/lm_ctrl.txt 2>&1; cat $OUT/lm_ctrl.txt
NO_TRACE=1 bash tools/gpu_libab.sh ${TAG}_ab 3d1955e || exit $?
FLOAM_DEBUG_STAMPS=1 timeout -k 10 300 python bench.py --steps 30 --cpu-baseline-seconds 0 --no-roofline --no-secondary \
    > $OUT/st.json 2> $OUT/st.err || { tail -20 $OUT/st.err; exit 1; }
grep stamps $OUT/st.err
echo all-done
