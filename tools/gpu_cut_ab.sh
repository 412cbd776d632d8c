#!/bin/bash
# Hub-cut bottom-up levels: GPU test, then per-root A/B (cut off / on).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q -m gpu -k "hub_cut or full_scale or hub_lds" --timeout 200 --timeout-method thread > gpurun_out/cut_pytest.log 2>&1; rc=$?
  tail -4 gpurun_out/cut_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
ARGSETS="${ARGSETS:---opt bu_cut_edges=0||--opt bu_cut_edges=0|}" ROOTS=${ROOTS:-20} STEPS=${STEPS:-20} bash tools/gpu_ab_levels_args.sh
