#!/bin/bash
# Multi-process path on ONE GPU: P ranks (torchrun, one process each) share
# device 0 and exchange through the TCP communicator (RCCL refuses two ranks on
# one device).  Exercises the real per-rank HIP kernels, partitioning, host loop
# and collectives schedule at P > 1; validation on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for P in ${PS:-2 4}; do
  DBFS_DEVICE=0 DBFS_COMM=tcp timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $P \
    --master-addr 127.0.0.1 --master-port $((29600 + P)) bench.py --gpus $P --scale ${SCALE:-20} --steps 4 --warmup 1 \
    > gpurun_out/mp_tcp_$P.json 2> gpurun_out/mp_tcp_$P.log || { echo "P=$P failed"; grep -v "^\s*$" gpurun_out/mp_tcp_$P.log | tail -15; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/mp_tcp_$P.json') if l.startswith('{')][-1]); print('P=$P', d['n_gpus'], 'validated', d['validated'], d['value'], 'GTEPS', d['level_profile'])"
done
