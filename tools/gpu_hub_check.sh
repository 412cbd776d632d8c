#!/bin/bash
# Bottom-up variants: GPU tests of the bottom-up / hub paths, then an A/B of
# the headline bench over engine options (VARIANTS, see tools/gpu_ab.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== gpu tests (bottom-up)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q -m gpu --timeout 120 --timeout-method thread -k "hub or bottom_up or device_loop or rmat_modes" > gpurun_out/pytest_hub.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_hub.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B"
VARIANTS="${VARIANTS:-base}" bash tools/gpu_ab.sh
