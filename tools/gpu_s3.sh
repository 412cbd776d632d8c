#!/bin/bash
# Round-3 session-3 check: GPU suite, headline bench, then the fused
# tiny-level exchange (xfuse_edges) on two ranks sharing the GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-s3}
if [ "${TESTS:-1}" = 1 ]; then
  echo "== pytest gpu"
  timeout -k 10 800 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread --durations=15 ${PYTEST_ARGS} > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
  tail -25 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  echo "== bench"
  timeout -k 10 300 python bench.py --steps 16 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print('%8.1f GTEPS %7.3f ms/step validated %s' % (d['value'], d['ms_per_step'], d['validated_roots']))"
fi
if [ "${XFUSE:-1}" = 1 ]; then
  echo "== xfuse"
  export DBFS_DEVICE=0 DBFS_COMM=peer DBFS_COMM_TIMEOUT_S=20
  for x in 0 4096; do
    timeout -k 10 150 python bench.py --gpus 2 --scale 18 --steps 4 --warmup 1 --no-int32-pass --opt xfuse_edges=$x > gpurun_out/${TAG}_xfuse$x.json 2> gpurun_out/${TAG}_xfuse$x.err; rc=$?
    echo "xfuse=$x rc=$rc"; grep -E "validated|Error|error" gpurun_out/${TAG}_xfuse$x.err | head -8 | cut -c1-300
    [ $rc -eq 0 ] || exit $rc
  done
fi
