#!/bin/bash
# LM solve time attribution on the GPU box: the C3 bench with the resident solve's stamps (FLOAM_DEBUG_STAMPS), then
# a rebuild of the diagnostic library with the control-step stamps (-DFLOAM_CTRL_STAMPS) into a scratch object dir.
set -o pipefail
OUT=gpurun_out/${1:-st}
mkdir -p $OUT
FLOAM_AMD_LIB=diag FLOAM_DEBUG_STAMPS=1 timeout -k 10 300 python bench.py --steps 30 --cpu-baseline-seconds 0 --no-roofline \
    > $OUT/st.json 2> $OUT/st.err || { tail -20 $OUT/st.err; exit 1; }
grep stamps $OUT/st.err
cat $OUT/st.json
timeout -k 10 600 make -C floam_amd/csrc -j16 DIAGDIR=/tmp/floam_stamps_obj EXTRA=-DFLOAM_CTRL_STAMPS ../libfloam_amd_diag.so > $OUT/make.log 2>&1 \
    || { tail -20 $OUT/make.log; exit 1; }
FLOAM_AMD_LIB=diag timeout -k 10 300 python bench.py --steps 30 --cpu-baseline-seconds 0 --no-roofline > $OUT/ctrl.json 2> $OUT/ctrl.err \
    || { tail -20 $OUT/ctrl.err; exit 1; }
grep "floam ctrl" $OUT/ctrl.err
