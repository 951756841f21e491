#!/bin/bash
# GPU check after a change: the GPU test suite (one process, per-test timeouts), then a short C3 bench with the
# roofline replay, then the resident solve's stamps.  Usage: bash tools/gpu_check.sh TAG [pytest -k expr]
set -o pipefail
OUT=gpurun_out/${1:-chk}
mkdir -p $OUT
K=${2:+-k "$2"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K \
    > $OUT/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -80
[ $rc -eq 0 ] || { tail -60 $OUT/pytest.log; exit $rc; }
timeout -k 10 300 python bench.py --cpu-baseline-seconds 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
FLOAM_DEBUG_STAMPS=1 timeout -k 10 200 python bench.py --steps 30 --cpu-baseline-seconds 0 --no-roofline \
    > $OUT/st.json 2> $OUT/st.err || { tail -20 $OUT/st.err; exit 1; }
grep stamps $OUT/st.err
