#!/bin/bash
# Session check: GPU tests, the headline bench, then a kernel trace of chosen
# roots (typical + late-switch) -- each step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3s}
SHADOW=0 TESTS=${TESTS:-1} TAG=$TAG bash tools/gpu_r3_check.sh || exit $?
if [ -n "${ROOTS}" ]; then
  echo "== trace roots"
  ROOTS="${ROOTS}" RUNS=${RUNS:-3} bash tools/gpu_trace_roots.sh > /dev/null || exit $?
  cp gpurun_out/troots_summary.txt gpurun_out/${TAG}_troots_summary.txt
  tail -3 gpurun_out/troots_summary.txt
fi
