#!/bin/bash
# Hardware counters of one kernel in a shadow-rank replay (rank R of P):
# two rocprofv3 --pmc passes (kernel trace only), then the longest dispatches
# of KERNEL with their counters (tools/counter_dispatch.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=${SCALE:-26}; P=${P:-8}; R=${R:-0}
rm -rf gpurun_out/spmc1 gpurun_out/spmc2
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES FETCH_SIZE \
  -d gpurun_out/spmc1 -o run --output-format csv -- \
  python3 tools/shadow_rank.py --scale $S --ranks-of $P --ranks $R --roots 1 ${SHADOW_ARGS} > gpurun_out/spmc1.log 2>&1 \
  || { tail -30 gpurun_out/spmc1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum \
  -d gpurun_out/spmc2 -o run --output-format csv -- \
  python3 tools/shadow_rank.py --scale $S --ranks-of $P --ranks $R --roots 1 ${SHADOW_ARGS} > gpurun_out/spmc2.log 2>&1 \
  || { tail -30 gpurun_out/spmc2.log; exit 1; }
python3 tools/counter_dispatch.py --kernel ${KERNEL:-update_kernel} --top ${TOP:-12} gpurun_out/spmc1 gpurun_out/spmc2 \
  > gpurun_out/${TAG:-r5}_shadow_counters.txt
cat gpurun_out/${TAG:-r5}_shadow_counters.txt
