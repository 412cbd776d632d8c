#!/bin/bash
# Kernel timeline of a shadow-rank replay (the last traversal of the tool's
# run is rank R's replay): where a P-rank level's time goes on one rank.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3}
S=${SCALE:-26}; P=${P:-8}; R=${R:-0}
rm -rf gpurun_out/strace
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/strace -o run --output-format csv -- \
  python3 tools/shadow_rank.py --scale $S --ranks-of $P --ranks $R --roots ${ROOTS:-2} ${SHADOW_ARGS} > gpurun_out/strace.log 2>&1 \
  || { tail -30 gpurun_out/strace.log; exit 1; }
f=$(find gpurun_out/strace -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py "$f" --from-kernel init_run_kernel --runs 1 > gpurun_out/${TAG}_shadow_trace_s${S}_p${P}_r${R}.txt
m=$(find gpurun_out/strace -name "*memory_copy_trace.csv" | head -1)
[ -n "$m" ] && cp "$m" gpurun_out/${TAG}_shadow_memcpy_s${S}_p${P}_r${R}.csv
gzip -f "$f"
tail -5 gpurun_out/${TAG}_shadow_trace_s${S}_p${P}_r${R}.txt
