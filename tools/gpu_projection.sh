#!/bin/bash
# Per-rank compute projection of the sharded mode: one GPU runs only rank 0's 1/N
# of the correspondence queries and solves on them alone (diagnostic build, FLOAM_SHARD_SOLO=N: no exchange, so the
# poses are not the sharded run's — only its per-rank kernel time), at C4 and C5 for N = 1, 2, 4, 8; then a kernel-
# trace timeline of C4 at N = 1 and N = 8 (what shrinks with N and what every rank replicates).
# Usage (GPU box, repo root): bash tools/gpu_projection.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-proj}
mkdir -p $OUT
export TMPDIR=/tmp FLOAM_AMD_LIB=diag
for cfg in c4 c5; do
  for n in 1 2 4 8; do
    FLOAM_SHARD_SOLO=$n timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --cpu-baseline-seconds 0 \
        --no-secondary --no-roofline > $OUT/${cfg}_n$n.json 2> $OUT/${cfg}_n$n.err || { tail -20 $OUT/${cfg}_n$n.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${cfg}_n$n.json')); print('$cfg', 'N=$n', d['value'], d['ms_per_step'])"
  done
done
for n in 1 8; do
  FLOAM_SHARD_SOLO=$n timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_c4_n$n -o run -- \
      python3 bench.py --config c4 --steps 20 --warmup 5 --cpu-baseline-seconds 0 --no-secondary --no-roofline \
      > $OUT/tr_c4_n$n.log 2>&1 || { tail -20 $OUT/tr_c4_n$n.log; exit 1; }
  f=$(find $OUT/tr_c4_n$n -name '*kernel_trace.csv' | head -1)
  python tools/timeline.py $f 10 > $OUT/timeline_c4_n$n.txt 2>&1 || true
  echo "== C4 N=$n"; tail -2 $OUT/timeline_c4_n$n.txt
done
echo done
