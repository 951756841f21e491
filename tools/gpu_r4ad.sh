#!/bin/bash
# GPU suite, smoke, A/B of the tree against 185b580 (branch-free Givens rotation and hypot in the edge fit),
# then the geometry stamps of the tree (diagnostic rebuild; last: it replaces the box copy's library).
set -o pipefail
TAG=${1:-r4ad}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log
case $rc in 0) ;; *) echo "stopping: rc $rc"; exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash tools/gpu_libab.sh ${TAG}_ab 185b580 || exit $?
timeout -k 10 600 make -C floam_amd/csrc -j16 OBJDIR=/tmp/floam_geom_obj EXTRA=-DFLOAM_GEOM_STAMPS > $OUT/make.log 2>&1 \
    || { tail -20 $OUT/make.log; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --cpu-baseline-seconds 0 --no-roofline --no-secondary > $OUT/geom.json \
    2> $OUT/geom.err || { tail -20 $OUT/geom.err; exit 1; }
grep "geom stamps" $OUT/geom.err
echo all-done
