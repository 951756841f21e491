#!/bin/bash
# One GPU session (run on the GPU box from the repo root), steps in the order given, stopping at the first failure:
#   tests[=EXPR]   the -m gpu suite in one process (per-test timeouts; EXPR: a pytest -k expression, commas for spaces)
#   smoke          __graft_entry__.smoke()
#   bench[=ARGS]   python bench.py ARGS (comma-separated), the JSON line to $OUT/bench.json
#   prof[=ARGS]    tools/gpu_prof.sh: bench + rocprofv3 kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes
#   proj           tools/gpu_projection.sh: per-rank compute of the sharded mode at C4 / C5, N = 1, 2, 4, 8
#   n2             tools/gpu_n2.sh: the N = 2 bench line rehearsed with two ranks on this one GPU
#   stamps         tools/gpu_stamps.sh: the LM solve's segment stamps (diagnostic build)
#   sweep=CONFIG   tools/precision_sweep.py: fp64 / fp32 / fp32-geometry poses against the oracle (8 scans)
#   envab=SPEC;..  tools/gpu_envab.sh over environment settings (SPEC NAME:VAR=V,VAR=V; ';'-separated)
#   libab=NAME,..  tools/gpu_libab.sh: the tree's library against prebuilt ones (floam_amd/ab/)
# Usage: bash tools/gpu_session.sh TAG STEP...
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for step in "$@"; do
  name=${step%%=*}; arg=""; [ "$step" != "$name" ] && arg=${step#*=}
  echo "== $step"
  case $name in
    tests)
      K=(); [ -n "$arg" ] && K=(-k "${arg//,/ }")   # (commas for spaces: "a,or,b")
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
          > $OUT/pytest_gpu.log 2>&1; rc=$?
      grep -cE "PASSED" $OUT/pytest_gpu.log; tail -3 $OUT/pytest_gpu.log
      [ $rc -eq 0 ] || { grep -E "FAILED|ERROR|Error|error" $OUT/pytest_gpu.log | tail -30; exit $rc; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
          || { tail -20 $OUT/smoke.log; exit 1; }
      tail -1 $OUT/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py ${arg//,/ } > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
      cut -c1-600 $OUT/bench.json ;;
    prof) bash tools/gpu_prof.sh ${TAG}/prof ${arg//,/ } || exit $? ;;
    n2) bash tools/gpu_n2.sh ${TAG}/n2 || exit $? ;;
    proj) bash tools/gpu_projection.sh ${TAG}/proj || exit $? ;;
    stamps) bash tools/gpu_stamps.sh ${TAG}/stamps || exit $? ;;
    sweep)
      timeout -k 10 600 python tools/precision_sweep.py --config ${arg:-c5} --scans 8 --out $OUT/precision_${arg:-c5}.json \
          > $OUT/precision_${arg:-c5}.log 2>&1 || { tail -20 $OUT/precision_${arg:-c5}.log; exit 1; }
      tail -12 $OUT/precision_${arg:-c5}.log ;;
    envab) IFS=';' read -ra specs <<< "$arg"; bash tools/gpu_envab.sh ${TAG}/envab "${specs[@]}" || exit $? ;;
    libab) bash tools/gpu_libab.sh ${TAG}/libab ${arg//,/ } || exit $? ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
echo all-done
