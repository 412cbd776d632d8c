#!/bin/bash
# The driver's multi-GPU invocation (torch.distributed.run, one process per
# rank), rehearsed with 2 ranks sharing this box's one GPU (DBFS_DEVICE=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp DBFS_DEVICE=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 8 --warmup 2 > gpurun_out/tr2.json 2> gpurun_out/tr2.err || { tail -30 gpurun_out/tr2.err; exit 1; }
grep -E "comm|validated" gpurun_out/tr2.err | head -6
tail -1 gpurun_out/tr2.json | cut -c1-700
