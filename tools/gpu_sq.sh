#!/bin/bash
# SQ occupancy / stall counters of one short bench run (own --pmc pass): wave lifetimes vs kernel durations.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/sq
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/sq/p -o run -- \
  python3 bench.py --steps 10 --cpu-baseline-seconds 0 --no-roofline "$@" > gpurun_out/sq/log 2>&1 || { tail -20 gpurun_out/sq/log; exit 1; }
ls gpurun_out/sq/p
