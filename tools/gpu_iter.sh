#!/bin/bash
# One GPU iteration: build, GPU tests, headline bench with per-level profile,
# rocprofv3 kernel statistics.  Every GPU step has its own time limit; the
# script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SCALE=${SCALE:-26}
make -j16 > gpurun_out/make.log 2>&1 || { tail -30 gpurun_out/make.log; exit 1; }
if [ "${TESTS:-1}" = 1 ]; then
  echo "== pytest gpu"
  timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -6 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
echo "== bench"
timeout -k 10 300 python bench.py --scale $SCALE --steps 16 --warmup 3 --per-level ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$?
tail -14 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
if [ "${PROF:-1}" = 1 ]; then
  echo "== rocprofv3"
  rm -rf gpurun_out/prof
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --scale $SCALE --steps 8 --warmup 2 --no-validate ${BENCH_ARGS} > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
  f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -16 "$f" | cut -c1-200
fi
