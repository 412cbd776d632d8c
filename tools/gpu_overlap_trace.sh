#!/bin/bash
# Kernel trace of two self-spawned ranks on one GPU (peer-memory transport):
# the split bottom-up head pass on the compute stream against the frontier
# all-gather's push / wait / unpack kernels on the communication stream.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/ovl
DBFS_DEVICE=0 DBFS_COMM=${COMM:-peer} DBFS_PEER_SLOT_MB=4 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ovl -o run_%pid% --output-format csv -- \
  python3 bench.py --gpus 2 --scale ${SCALE:-22} --steps 4 --warmup 1 --no-int32-pass > gpurun_out/ovl.log 2>&1 || { tail -30 gpurun_out/ovl.log; exit 1; }
ls gpurun_out/ovl | head
for f in $(find gpurun_out/ovl -name "*kernel_trace.csv"); do
  if grep -q bu_head_kernel "$f"; then
    echo "== $f"; python3 tools/overlap_summary.py "$f" --timeline 1 | tee -a gpurun_out/overlap_summary.txt
  fi
  gzip -f "$f"
done
