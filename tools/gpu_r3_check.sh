#!/bin/bash
# Round-3 check: GPU tests, the headline bench, and the P = 8 shadow ranks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3}
if [ "${TESTS:-1}" = 1 ]; then
  echo "== pytest gpu"
  timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
  tail -5 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
echo "== bench"
timeout -k 10 300 python bench.py --steps 16 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print('%8.1f GTEPS %7.3f ms/step validated %s' % (d['value'], d['ms_per_step'], d['validated_roots']))"
if [ "${SHADOW:-1}" = 1 ]; then
  echo "== shadow"
  CFGS="${CFGS:-26:8:0,7}" TAG=$TAG bash tools/gpu_shadow.sh
fi
