#!/bin/bash
# Full GPU test file + repeated headline bench (REPS runs; noise between
# processes is several percent on a shared box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  echo "== pytest gpu"
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
echo "== bench x${REPS:-3}"
: > gpurun_out/quick.txt
for rep in $(seq ${REPS:-3}); do
  timeout -k 10 240 python bench.py --steps ${STEPS:-16} --warmup 3 ${BENCH_ARGS} > gpurun_out/quick_run.json 2> gpurun_out/quick_run.err || { tail -20 gpurun_out/quick_run.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/quick_run.json').read().strip().splitlines()[-1]); print('%8.1f GTEPS %7.3f ms/step validated %s levels %s' % (d['value'], d['ms_per_step'], d['validated'], [(l[0], l[1]) for l in d['level_profile']['levels']]))" | tee -a gpurun_out/quick.txt
done
