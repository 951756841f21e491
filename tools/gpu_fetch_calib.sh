#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration for the kNN's access patterns (tools/micro/fetch_calib.hip).
# Usage (GPU box, repo root): bash tools/gpu_fetch_calib.sh
set -o pipefail
OUT=gpurun_out/calib
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
hipcc -O3 --offload-arch=gfx950 tools/micro/fetch_calib.hip -o $OUT/fetch_calib 2>/dev/null || exit 1
timeout -k 10 120 $OUT/fetch_calib > $OUT/run.log 2>&1 || { cat $OUT/run.log; exit 1; }
cat $OUT/run.log
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- $OUT/fetch_calib > $OUT/fetch.log 2>&1 || { tail $OUT/fetch.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace --output-format csv -d $OUT/rdreq -o run -- $OUT/fetch_calib > $OUT/rdreq.log 2>&1 || { tail $OUT/rdreq.log; exit 1; }
python3 - <<'PY'
import csv, glob
for tag in ("fetch", "rdreq"):
    for f in glob.glob(f"gpurun_out/calib/{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            print(tag, r.get("Kernel_Name", "")[:20], r.get("Counter_Name"), r.get("Counter_Value"))
PY
