#!/bin/bash
# Per-dispatch clock of a shadow-rank replay: one rocprofv3 --pmc pass with
# GRBM_GUI_ACTIVE (GPU-busy cycles) and wave counters; the last N dispatches
# in time order with GRBM_GUI_ACTIVE / duration (tools/counter_dispatch.py --timeline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=${SCALE:-26}; P=${P:-8}; R=${R:-0}
rm -rf gpurun_out/sclk
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES \
  -d gpurun_out/sclk -o run --output-format csv -- \
  python3 tools/shadow_rank.py --scale $S --ranks-of $P --ranks $R --roots 1 ${SHADOW_ARGS} > gpurun_out/sclk.log 2>&1 \
  || { tail -30 gpurun_out/sclk.log; exit 1; }
python3 tools/counter_dispatch.py --kernel "${KERNEL:-}" --timeline ${N:-45} gpurun_out/sclk > gpurun_out/${TAG:-r5}_shadow_clock.txt
cat gpurun_out/${TAG:-r5}_shadow_clock.txt
