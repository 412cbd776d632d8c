#!/bin/bash
# Round-4 check: GPU tests (or a -k selection), the headline bench with the
# held-out roots and the soc-LiveJournal1-sized secondary block.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r4}
if [ "${TESTS:-1}" = 1 ]; then
  echo "== pytest gpu ${PYTEST_K:+-k $PYTEST_K}"
  timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
  tail -5 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  echo "== bench"
  timeout -k 10 400 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
  python3 - <<PY
import json
d = json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1])
print('%8.1f GTEPS %7.4f ms/step validated %s int32 %s' % (d['value'], d['ms_per_step'], d['validated_roots'], d['value_int32_levels']))
print('heldout', d.get('heldout'))
print('secondary', json.dumps(d.get('secondary')))
PY
fi
