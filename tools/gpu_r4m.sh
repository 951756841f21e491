#!/bin/bash
# GPU tests of the LM control-step trims, the A/B against the session-start library (60351fc), an API + kernel
# trace of the bench (main-stream gaps), the LM stamps and micro-benchmark.  Usage: bash tools/gpu_r4m.sh TAG
set -o pipefail
TAG=${1:-r4m}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$TAG/pytest_gpu.log
case $rc in 0) ;; *) echo "stopping: rc $rc"; exit $rc;; esac
NO_TRACE=1 bash tools/gpu_libab.sh ${TAG}_ab 60351fc || exit $?
bash tools/gpu_apitrace.sh ${TAG}_api || exit $?
FLOAM_DEBUG_STAMPS=1 timeout -k 10 300 python bench.py --steps 30 --cpu-baseline-seconds 0 --no-roofline --no-secondary \
    > gpurun_out/$TAG/st.json 2> gpurun_out/$TAG/st.err || { tail -20 gpurun_out/$TAG/st.err; exit 1; }
grep stamps gpurun_out/$TAG/st.err
timeout -k 10 200 hipcc -O3 -std=c++17 -ffp-contract=fast --offload-arch=gfx950 tools/micro/lm_ctrl.hip -o /tmp/lm_ctrl \
    > gpurun_out/$TAG/lm_ctrl_build.log 2>&1 && timeout -k 10 60 /tmp/lm_ctrl > gpurun_out/$TAG/lm_ctrl.txt 2>&1; cat gpurun_out/$TAG/lm_ctrl.txt
echo all-done
