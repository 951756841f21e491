#!/bin/bash
# Kernel-time profile of the C3 bench at each residual precision (fp64 Gram solve vs the per-record fp32 solve).
# Usage (GPU box, repo root): bash tools/gpu_prec_prof.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-pp}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for P in fp64 fp32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$P -o run -- \
    python3 bench.py --steps 30 --cpu-baseline-seconds 0 --no-secondary --precision $P > $OUT/$P.json 2> $OUT/$P.err \
    || { tail -20 $OUT/$P.err; exit 1; }
  cut -c1-200 $OUT/$P.json
done
