#!/bin/bash
# Two self-spawned ranks sharing one GPU over the peer transport, fused small
# collectives on / off, alternating (a rough A/B: the ranks time-share the GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for f in 1 0 1 0; do
  DBFS_PEER_FUSED=$f DBFS_DEVICE=0 DBFS_COMM=peer timeout -k 10 200 python bench.py --gpus ${P:-2} --scale ${SCALE:-22} \
    --steps ${STEPS:-16} --warmup 2 --no-int32-pass --no-validate > gpurun_out/pab.json 2> gpurun_out/pab.err \
    || { echo "fused=$f failed"; tail -20 gpurun_out/pab.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/pab.json').read().strip().splitlines()[-1]); print('fused', sys.argv[1], d['value'], d['ms_per_step'])" $f
done
