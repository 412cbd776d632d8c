#!/bin/bash
# Iteration check: GPU tests, headline bench, top-down-only bench at RMAT-22,
# kernel timeline of the last two traversals of a short RMAT-26 bench.
#   SKIP_TESTS=1 to skip pytest; TD=0 to skip the td bench; TRACE=0 to skip the trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  echo "== pytest gpu"
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], 'GTEPS', d['ms_per_step'], 'ms', d['validated_roots'], [(l[0], round(l[1]*1e3,1)) for l in d['level_clock']['levels']])" "$@"; }
echo "== bench RMAT-26 do"
timeout -k 10 240 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/it_do26.json 2> gpurun_out/it_do26.err || { tail -20 gpurun_out/it_do26.err; exit 1; }
summ gpurun_out/it_do26.json do26
if [ "${TD:-1}" = 1 ]; then
  echo "== bench RMAT-22 td"
  timeout -k 10 240 python bench.py --scale 22 --mode td --steps 16 --warmup 3 --no-int32-pass > gpurun_out/it_td22.json 2> gpurun_out/it_td22.err || { tail -20 gpurun_out/it_td22.err; exit 1; }
  summ gpurun_out/it_td22.json td22
fi
if [ "${TRACE:-1}" = 1 ]; then
  echo "== trace"
  rm -rf gpurun_out/trace
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-validate --no-int32-pass ${TRACE_ARGS} > gpurun_out/trace.log 2>&1 || { tail -30 gpurun_out/trace.log; exit 1; }
  f=$(find gpurun_out/trace -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_summary.py "$f" --runs 2 > gpurun_out/trace_summary.txt
  gzip -f "$f"
  tail -45 gpurun_out/trace_summary.txt
fi
