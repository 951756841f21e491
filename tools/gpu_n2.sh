#!/bin/bash
# The N = 2 bench line rehearsed on one GPU: two ranks (processes) on device 0 (FLOAM_BENCH_DEVICE=0), default shard
# mode (C4 + the C3 sharded line; peer exchange through IPC-mapped buffers).  Usage: bash tools/gpu_n2.sh TAG [args]
set -o pipefail
OUT=gpurun_out/${1:-n2}; shift || true
mkdir -p $OUT
export TMPDIR=/tmp
FLOAM_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 "$@" > $OUT/n2.json 2> $OUT/n2.err \
    || { tail -30 $OUT/n2.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/n2.json')); print(json.dumps({k: d.get(k) for k in ('value','config','pose_vs_oracle','same_config_1gpu','c3_sharded')}))"
