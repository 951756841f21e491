#!/bin/bash
# SQ instruction / wave counters of the kNN launches for the tree's library and prebuilt ones (floam_amd/ab/): one
# rocprofv3 --pmc pass each over a short C3 bench.  Usage: bash tools/gpu_knn_pmc.sh TAG NAME...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cp floam_amd/libfloam_amd.so /tmp/lib_tree.so
trap 'cp /tmp/lib_tree.so floam_amd/libfloam_amd.so' EXIT
for v in tree "$@"; do
  if [ "$v" = tree ]; then cp /tmp/lib_tree.so floam_amd/libfloam_amd.so; else cp floam_amd/ab/libfloam_amd_$v.so floam_amd/libfloam_amd.so; fi
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH \
      --output-format csv -d $OUT/pmc_$v -o run -- python3 bench.py --steps 10 --warmup 4 --cpu-baseline-seconds 0 \
      --no-secondary --no-roofline > $OUT/pmc_$v.log 2>&1 || { tail -20 $OUT/pmc_$v.log; exit 1; }
  f=$(find $OUT/pmc_$v -name '*counter_collection.csv' | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'knn_kernel' in r['Kernel_Name']]
agg = collections.defaultdict(float); disp = set()
for r in rows:
    agg[r['Counter_Name']] += float(r['Counter_Value']); disp.add(r['Dispatch_Id'])
n = max(len(disp), 1)
print(sys.argv[2], 'dispatches', n, ' '.join(f"{k}={v / n:.4g}" for k, v in sorted(agg.items())))
PY
done
