#!/bin/bash
# kNN read attribution per dependent round trip (tools/knn_stages.py): FETCH_SIZE and WRITE_SIZE passes of the C3
# bench with the roofline replay and FLOAM_KNN_STAGES=1.  Usage: bash tools/gpu_knn_stages.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-ks}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for c in FETCH_SIZE WRITE_SIZE; do
  FLOAM_AMD_LIB=diag FLOAM_KNN_STAGES=1 timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/st_$c -o run -- \
      python3 bench.py --cpu-baseline-seconds 0 --no-secondary --steps 20 > $OUT/st_$c.log 2>&1 || { tail -20 $OUT/st_$c.log; exit 1; }
  echo "== $c"
  python tools/knn_stages.py $OUT/st_$c/run_counter_collection.csv $c --json $OUT/knn_stages_$c.json
done
echo done
