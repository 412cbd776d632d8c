#!/bin/bash
# Kernel timeline of chosen roots (tools/run_roots.py): ROOTS="a b" OPTS="--opt x=1"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/troots
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/troots -o run --output-format csv -- \
  python3 tools/run_roots.py --scale ${SCALE:-26} --mode ${MODE:-do} --roots ${ROOTS} ${OPTS} > gpurun_out/troots.log 2>&1 || { tail -30 gpurun_out/troots.log; exit 1; }
cat gpurun_out/troots.log | grep -v "^\s*$" | tail -${#ROOTS}
f=$(find gpurun_out/troots -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py "$f" --from-kernel init_run_kernel --runs ${RUNS:-2} > gpurun_out/troots_summary.txt
gzip -f "$f"
cat gpurun_out/troots_summary.txt
