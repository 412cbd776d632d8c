#!/bin/bash
# Session check: multi-rank GPU tests (peer transport, virtual ranks, shadow
# replay), then P = 8 shadow ranks with the defaults and with VARIANT options.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3s3}
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q -k "${TESTK:-peer or virtual or shadow or from_bitmap}" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1 || { tail -30 gpurun_out/${TAG}_t.log; exit 1; }
tail -2 gpurun_out/${TAG}_t.log
TAG=$TAG CFGS="${CFGS:-26:8:0,7}" bash tools/gpu_shadow.sh || exit 1
if [ -n "${VARIANT}" ]; then
  TAG=${TAG}v CFGS="${CFGS:-26:8:0,7}" SHADOW_ARGS="${VARIANT}" bash tools/gpu_shadow.sh || exit 1
fi
