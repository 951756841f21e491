set -o pipefail
bash tools/gpu_trace.sh t4 >/dev/null && FLOAM_LM_PERSISTENT=0 bash tools/gpu_trace.sh t5 > /dev/null && echo ok
