#!/bin/bash
# First GPU validation pass: smoke, GPU tests, bench at a small and the headline scale.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== make"; make -j16 > gpurun_out/make.log 2>&1 || { tail -30 gpurun_out/make.log; exit 1; }
echo "== smoke"; timeout -k 10 300 python __graft_entry__.py > gpurun_out/smoke.log 2>&1; rc=$?; tail -5 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== pytest gpu"; timeout -k 10 600 python -m pytest tests/test_gpu_engine.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench s20"; timeout -k 10 300 python bench.py --scale 20 --steps 8 --warmup 2 --per-level > gpurun_out/bench_s20.log 2>&1; rc=$?; tail -20 gpurun_out/bench_s20.log; [ $rc -eq 0 ] || exit $rc
echo "== bench s26"; timeout -k 10 600 python bench.py --steps 16 --warmup 3 --per-level > gpurun_out/bench_s26.log 2>&1; rc=$?; tail -25 gpurun_out/bench_s26.log; [ $rc -eq 0 ] || exit $rc
echo "== bench s26 ref"; timeout -k 10 600 python bench.py --steps 4 --warmup 1 --mode ref --no-validate > gpurun_out/bench_s26_ref.log 2>&1; rc=$?; tail -8 gpurun_out/bench_s26_ref.log; exit $rc
