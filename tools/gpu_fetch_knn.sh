#!/bin/bash
# FETCH_SIZE of the kNN launches in a short bench run (own --pmc pass), doubled per the gfx950 correction
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/fk
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/fk/p -o run -- \
  python3 bench.py --steps 20 --cpu-baseline-seconds 0 --no-roofline > gpurun_out/fk/log 2>&1 || { tail -5 gpurun_out/fk/log; exit 1; }
python3 - <<'PY'
import csv
rows = [r for r in csv.DictReader(open('gpurun_out/fk/p/run_counter_collection.csv')) if r['Counter_Name'] == 'FETCH_SIZE']
for name in ('knn_kernel', 'geom_kernel', 'grid_count', 'radix_pass'):
    v = [float(r['Counter_Value']) for r in rows if name in r['Kernel_Name']][-80:]
    if v:
        print(name, 'FETCH bytes/launch (x2, KiB->B):', round(2 * 1024 * sum(v) / len(v)))
PY
