#!/bin/bash
# L2 (TCC) hits and misses of the kNN launches: one rocprofv3 --pmc pass over a short C3 bench, per-launch averages
# by launch position within the scan (the map is the same for a scan's four searches).  Usage: bash tools/gpu_knn_l2.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-l2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc -o run -- python3 bench.py \
    --steps 12 --warmup 4 --cpu-baseline-seconds 0 --no-secondary --no-roofline > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
f=$(find $OUT/pmc -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1]))]
by = collections.defaultdict(dict)
name = {}
for r in rows:
    d = int(r['Dispatch_Id']); by[d][r['Counter_Name']] = by[d].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    name[d] = r['Kernel_Name']
knn = sorted(d for d in by if 'knn_kernel' in name[d])
print('knn launches', len(knn))
for pos in range(4):   # position in the scan: call 1 pass 1, 2; call 2 pass 1, 2
    sel = knn[pos::4][2:]
    h = sum(by[d].get('TCC_HIT_sum', 0) for d in sel) / max(len(sel), 1)
    m = sum(by[d].get('TCC_MISS_sum', 0) for d in sel) / max(len(sel), 1)
    print(f'position {pos}: launches {len(sel)}, L2 hits {h:.0f}, misses {m:.0f}, hit rate {h / max(h + m, 1):.3f}')
other = collections.defaultdict(lambda: [0.0, 0.0, 0])
for d in by:
    k = name[d].split('(')[0][-40:]
    other[k][0] += by[d].get('TCC_HIT_sum', 0); other[k][1] += by[d].get('TCC_MISS_sum', 0); other[k][2] += 1
for k, (h, m, n) in sorted(other.items(), key=lambda x: -(x[1][0] + x[1][1]))[:12]:
    print(f'{k:42s} n {n:4d} hit rate {h / max(h + m, 1):.3f} misses/launch {m / n:.0f}')
PY
