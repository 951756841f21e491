#!/bin/bash
# The GPU test suite on the tree's library, then an A/B of prebuilt variants (tools/gpu_ab.sh).
# Usage (GPU box): bash tools/gpu_test_ab.sh TAG variant...
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $OUT/pytest.log | head -30; exit $rc; }
bash tools/gpu_ab.sh "$@"
