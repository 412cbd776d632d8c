#!/bin/bash
# Round-2 GPU check: GPU tests, headline bench, two self-spawned ranks on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest gpu"
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench 1 GPU"
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail -20 gpurun_out/bench1.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench1.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['validated_roots'], d['value_int32_levels'])"
echo "== bench 2 ranks on one GPU (tcp), scale 22"
DBFS_DEVICE=0 DBFS_COMM=tcp timeout -k 10 300 python bench.py --gpus 2 --scale 22 --steps 8 --warmup 2 > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { tail -20 gpurun_out/bench2.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['validated_roots'], d['comm'], d['devices'], d['mispredicted_levels'])"
