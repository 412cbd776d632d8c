#!/bin/bash
# Experiment: two RCCL ranks on ONE GPU (DBFS_DEVICE=0) through the real
# multi-process launch path.  RCCL may refuse duplicate devices; this records it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
DBFS_DEVICE=0 timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29731 bench.py --gpus 2 --scale 18 --steps 4 --warmup 1 > gpurun_out/rccl2.log 2>&1
echo "rc=$?"; grep -v "^\s*$" gpurun_out/rccl2.log | tail -12
