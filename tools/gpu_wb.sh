#!/bin/bash
# Write-byte attribution of mm_merge and the ring-bucketing radix pass: WRITE_SIZE and
# FETCH_SIZE passes of the C3 bench with and without FLOAM_PROF_WB=1 (an L2 write-back dispatch before and after each
# of the two kernels).  Usage: bash tools/gpu_wb.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-wb}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
B="python3 bench.py --cpu-baseline-seconds 0 --no-roofline --no-secondary --steps 20"
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/plain_$c -o run -- $B \
      > $OUT/plain_$c.log 2>&1 || { tail -20 $OUT/plain_$c.log; exit 1; }
  FLOAM_PROF_WB=1 timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/wb_$c -o run -- $B \
      > $OUT/wb_$c.log 2>&1 || { tail -20 $OUT/wb_$c.log; exit 1; }
  echo "== $c (bracketed by L2 write-backs)"
  python tools/wb_attrib.py $OUT/wb_$c/run_counter_collection.csv $c --json $OUT/wb_$c.json
done
echo done
