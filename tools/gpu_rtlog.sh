#!/bin/bash
# ROCclr packet log of a few C3 bench scans (AMD_LOG_LEVEL=4): which barrier / marker packets the runtime puts on
# the streams between our kernels.  Output: gpurun_out/rtlog/{log.txt,summary.txt}
set -o pipefail
mkdir -p gpurun_out/rtlog
AMD_LOG_LEVEL=4 AMD_LOG_MASK=0x7FFFFFFF timeout -k 10 200 python3 bench.py --steps 4 --warmup 3 --cpu-baseline-seconds 0 --no-secondary --no-roofline > gpurun_out/rtlog/bench.json 2> gpurun_out/rtlog/log_full.txt
rc=$?
tail -c 30000000 gpurun_out/rtlog/log_full.txt > gpurun_out/rtlog/log.txt
rm -f gpurun_out/rtlog/log_full.txt
grep -o -E "(BarrierAND|BarrierOR|barrier|Marker|marker|ShaderName : [A-Za-z_0-9:]+|StreamQuery|hipStreamQuery|hipEventRecord|hipStreamWaitEvent|SIGNAL|signal)" gpurun_out/rtlog/log.txt | sort | uniq -c | sort -rn | head -60 > gpurun_out/rtlog/summary.txt
cat gpurun_out/rtlog/summary.txt | head -40
exit $rc
