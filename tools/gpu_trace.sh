#!/bin/bash
# Kernel timeline of the last BFS runs of a short bench (rocprofv3 kernel trace
# only; no counters).  Output: gpurun_out/trace_summary.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SCALE=${SCALE:-26}
rm -rf gpurun_out/trace
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/trace -o run --output-format csv -- \
  python3 bench.py --scale $SCALE --steps ${STEPS:-2} --warmup 1 --no-validate ${BENCH_ARGS} > gpurun_out/trace.log 2>&1 \
  || { tail -30 gpurun_out/trace.log; exit 1; }
f=$(find gpurun_out/trace -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py "$f" --runs ${RUNS:-2} > gpurun_out/trace_summary.txt
gzip -f "$f"
tail -5 gpurun_out/trace_summary.txt
