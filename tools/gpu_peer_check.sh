#!/bin/bash
# Peer-memory communicator on one GPU: two self-spawned ranks (IPC windows on
# the same device), bench at RMAT-22 with the peer transport vs TCP, then a
# kernel trace of the peer run (push / wait / unpack kernels on the side
# stream next to the split bottom-up head pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== peer bench (2 ranks, 1 GPU)"
DBFS_DEVICE=0 DBFS_COMM=peer DBFS_PEER_SLOT_MB=4 timeout -k 10 200 python bench.py --gpus 2 --scale 22 --steps 8 --warmup 2 > gpurun_out/peer2.json 2> gpurun_out/peer2.err || { tail -30 gpurun_out/peer2.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/peer2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['validated_roots'], d['comm'], d['comm_note'], d['level_profile'])"
echo "== tcp bench (2 ranks, 1 GPU)"
DBFS_DEVICE=0 DBFS_COMM=tcp timeout -k 10 200 python bench.py --gpus 2 --scale 22 --steps 8 --warmup 2 > gpurun_out/tcp2.json 2> gpurun_out/tcp2.err || { tail -30 gpurun_out/tcp2.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/tcp2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['validated_roots'], d['comm'])"
