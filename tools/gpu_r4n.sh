#!/bin/bash
# GPU tests, A/B against the previous tree's library (super-cell slots + no scratch vs d2339fb), timeline, sort /
# merge stamps and the kNN per-round-trip reads.  Usage: bash tools/gpu_r4n.sh TAG
set -o pipefail
TAG=${1:-r4n}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$TAG/pytest_gpu.log
case $rc in 0) ;; *) echo "stopping: rc $rc"; exit $rc;; esac
NO_TRACE=1 bash tools/gpu_libab.sh ${TAG}_ab d2339fb || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/tr -o run -- \
    python3 bench.py --cpu-baseline-seconds 0 --no-secondary --no-roofline > gpurun_out/$TAG/tr.log 2>&1 || { tail -20 gpurun_out/$TAG/tr.log; exit 1; }
python tools/timeline.py gpurun_out/$TAG/tr/run_kernel_trace.csv 10 > gpurun_out/$TAG/timeline.txt 2>&1; tail -3 gpurun_out/$TAG/timeline.txt
FLOAM_BC_STAMPS=1 FLOAM_MM_STAMPS=1 FLOAM_DEBUG_STAMPS=1 timeout -k 10 300 python bench.py --steps 30 --cpu-baseline-seconds 0 \
    --no-roofline --no-secondary > gpurun_out/$TAG/st.json 2> gpurun_out/$TAG/st.err || { tail -20 gpurun_out/$TAG/st.err; exit 1; }
grep -E "stamps\]" gpurun_out/$TAG/st.err
FLOAM_KNN_STAGES=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/$TAG/ks -o run -- \
    python3 bench.py --cpu-baseline-seconds 0 --no-secondary --steps 20 > gpurun_out/$TAG/ks.log 2>&1 || { tail -20 gpurun_out/$TAG/ks.log; exit 1; }
python tools/knn_stages.py gpurun_out/$TAG/ks/run_counter_collection.csv FETCH_SIZE --json gpurun_out/$TAG/knn_stages_FETCH_SIZE.json
echo all-done
