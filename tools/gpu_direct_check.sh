#!/bin/bash
# Direct owner-list exchange (td_sparse -> peers' windows -> td_sparse_apply):
# the peer-transport GPU tests, then ranks sharing device 0 (time-shared, so
# the numbers are correctness and launch counts, not speed) with the direct
# exchange on and off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-direct}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_engine.py \
  -k "peer or shared_device" > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/${TAG}_pytest.log
for P in 2 4; do
  for d in 1 0; do
    DBFS_DEVICE=0 DBFS_COMM=peer DBFS_PEER_SLOT_MB=16 timeout -k 10 200 python -u bench.py --gpus $P --scale ${SCALE:-20} \
      --steps 8 --warmup 2 --no-int32-pass --opt direct_lists=$d > gpurun_out/${TAG}_p${P}_d${d}.json 2> gpurun_out/${TAG}_p${P}_d${d}.err \
      || { tail -20 gpurun_out/${TAG}_p${P}_d${d}.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['comm'], d['validated_roots'])" gpurun_out/${TAG}_p${P}_d${d}.json "P=$P direct=$d"
  done
done
