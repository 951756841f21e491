#!/bin/bash
# Per-wave timeline of a C3 search launch: a scratch diagnostic build with -DFLOAM_KNN_WAVES, the bench (its handles
# dump the latest launch's waves at close), then tools/knn_waves.py.  Usage: bash tools/gpu_knn_waves.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-kw}
mkdir -p $OUT
cp floam_amd/libfloam_amd_diag.so /tmp/diag_keep.so
trap 'cp /tmp/diag_keep.so floam_amd/libfloam_amd_diag.so' EXIT
timeout -k 10 600 make -C floam_amd/csrc -j16 DIAGDIR=/tmp/floam_kw_obj EXTRA=-DFLOAM_KNN_WAVES ../libfloam_amd_diag.so \
    > $OUT/make.log 2>&1 || { tail -20 $OUT/make.log; exit 1; }
FLOAM_AMD_LIB=diag FLOAM_KNN_WAVES=$OUT/waves.bin timeout -k 10 300 python bench.py --steps 20 --cpu-baseline-seconds 0 \
    --no-roofline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python tools/knn_waves.py $OUT/waves.bin | tee $OUT/waves.txt
