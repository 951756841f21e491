#!/bin/bash
# LM solve A/B on the GPU box: per-solve segment stamps (FLOAM_DEBUG_STAMPS) of the C3 bench with the tree's build,
# then with a scratch rebuild using EXTRA flags (default: the register-resident LM state), and the control-step
# microbenchmark.  Usage: bash tools/gpu_lmab.sh TAG [EXTRA]
set -o pipefail
OUT=gpurun_out/${1:-lmab}
B_EXTRA=${2:--DFLOAM_LM_STATE_REGS=1}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 hipcc -O3 -std=c++17 -ffp-contract=fast --offload-arch=gfx950 tools/micro/lm_ctrl.hip -o /tmp/lm_ctrl \
    > $OUT/lm_ctrl_build.log 2>&1 && timeout -k 10 60 /tmp/lm_ctrl > $OUT/lm_ctrl.txt 2>&1; cat $OUT/lm_ctrl.txt
for v in A B A B; do
  if [ $v = B ] && [ ! -f /tmp/floam_b.so ]; then
    cp floam_amd/libfloam_amd.so /tmp/floam_a.so
    timeout -k 10 600 make -C floam_amd/csrc -j16 OBJDIR=/tmp/floam_b_obj EXTRA="$B_EXTRA" > $OUT/make_b.log 2>&1 \
        || { tail -20 $OUT/make_b.log; exit 1; }
    cp floam_amd/libfloam_amd.so /tmp/floam_b.so
  fi
  [ -f /tmp/floam_$(echo $v | tr AB ab).so ] && cp /tmp/floam_$(echo $v | tr AB ab).so floam_amd/libfloam_amd.so
  FLOAM_DEBUG_STAMPS=1 timeout -k 10 300 python bench.py --steps 40 --cpu-baseline-seconds 0 --no-secondary \
      > $OUT/st_$v.json 2> $OUT/st_$v.err || { tail -20 $OUT/st_$v.err; exit 1; }
  echo "== $v"; grep stamps $OUT/st_$v.err | tail -2
  python -c "import json,sys; d=json.load(open('$OUT/st_$v.json')); r=d.get('roofline') or {}; print('scans/s', d['value'], 'lm', r.get('lm_solve_avg_us'))"
done
[ -f /tmp/floam_a.so ] && cp /tmp/floam_a.so floam_amd/libfloam_amd.so
echo done
