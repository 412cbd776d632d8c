#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== gpu tests (hub)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q -m gpu --timeout 120 --timeout-method thread -k "hub or bottom_up or device_loop or rmat_modes" > gpurun_out/pytest_hub.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_hub.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B"
VARIANTS="base" BENCH_ARGS="--no-hubs" bash tools/gpu_ab.sh && cp gpurun_out/ab.txt gpurun_out/ab_nohubs.txt && VARIANTS="base" bash tools/gpu_ab.sh && cat gpurun_out/ab_nohubs.txt gpurun_out/ab.txt
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --per-level > gpurun_out/bench_hub.log 2>&1; tail -22 gpurun_out/bench_hub.log
