#!/bin/bash
# P = 8 ranks sharing one GPU (self-spawned bench ranks, DBFS_DEVICE=0): the
# peer-memory transport (IPC windows on one device) and TCP, validated.  A
# correctness rehearsal of the 8-GPU run's communication schedule (the timing
# of 8 processes time-sharing one GPU means nothing).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for comm in ${COMMS:-peer tcp}; do
  DBFS_DEVICE=0 DBFS_COMM=$comm DBFS_PEER_SLOT_MB=2 timeout -k 10 300 python bench.py --gpus ${P:-8} --scale ${SCALE:-20} --steps 4 --warmup 1 --no-int32-pass \
    > gpurun_out/r8_$comm.json 2> gpurun_out/r8_$comm.err || { echo "$comm failed"; tail -30 gpurun_out/r8_$comm.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['n_gpus'], d['comm'], d['validated_roots'], d['value'], d['mispredicted_levels'], d['level_profile']['levels'])" gpurun_out/r8_$comm.json $comm
done
