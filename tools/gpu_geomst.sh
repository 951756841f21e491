#!/bin/bash
# Geometry-kernel phase attribution: the GPU suite on the product build, then a diagnostic rebuild with
# -DFLOAM_GEOM_STAMPS (scratch object dir; replaces the box copy's library) and the C3 bench with its stamps printed.
set -o pipefail
OUT=gpurun_out/${1:-geomst}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log
case $rc in 0) ;; *) echo "stopping: rc $rc"; exit $rc;; esac
timeout -k 10 600 make -C floam_amd/csrc -j16 OBJDIR=/tmp/floam_geom_obj EXTRA=-DFLOAM_GEOM_STAMPS > $OUT/make.log 2>&1 \
    || { tail -20 $OUT/make.log; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --cpu-baseline-seconds 0 --no-roofline --no-secondary > $OUT/geom.json \
    2> $OUT/geom.err || { tail -20 $OUT/geom.err; exit 1; }
grep "geom stamps" $OUT/geom.err
cut -c1-200 $OUT/geom.json
echo all-done
