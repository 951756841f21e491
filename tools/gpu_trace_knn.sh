#!/bin/bash
# kNN per-wave trace of a short bench run (diagnostic): FLOAM_KNN_TRACE dump + tools/knn_trace.py summary
set -o pipefail
mkdir -p gpurun_out/tr
FLOAM_KNN_TRACE=gpurun_out/tr/knn.bin timeout -k 10 200 python bench.py --steps 10 --cpu-baseline-seconds 0 --no-roofline > gpurun_out/tr/b.json 2> gpurun_out/tr/b.err || { tail -5 gpurun_out/tr/b.err; exit 1; }
python tools/knn_trace.py gpurun_out/tr/knn.bin | head -4
