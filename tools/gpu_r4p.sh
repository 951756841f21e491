#!/bin/bash
# The update-boundary idle time (FLOAM_UPDATE_NOP timeline) and the compaction's last-phase split.
set -o pipefail
TAG=${1:-r4p}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
FLOAM_UPDATE_NOP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o run -- \
    python3 bench.py --cpu-baseline-seconds 0 --no-secondary --no-roofline > $OUT/tr.log 2>&1 || { tail -20 $OUT/tr.log; exit 1; }
python tools/timeline.py $OUT/tr/run_kernel_trace.csv 10 > $OUT/timeline.txt 2>&1; cat $OUT/timeline.txt
FLOAM_BC_STAMPS=1 timeout -k 10 300 python bench.py --steps 30 --cpu-baseline-seconds 0 \
    --no-roofline --no-secondary > $OUT/st.json 2> $OUT/st.err || { tail -20 $OUT/st.err; exit 1; }
grep -E "stamps\]" $OUT/st.err
echo all-done
