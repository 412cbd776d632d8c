#!/bin/bash
# Kernel timeline of two self-spawned ranks sharing GPU 0 over the peer
# transport (direct exchanges): which kernels a multi-rank level launches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp DBFS_DEVICE=0 DBFS_COMM=peer DBFS_PEER_SLOT_MB=${DBFS_PEER_SLOT_MB:-16}
rm -rf gpurun_out/ptrace
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ptrace -o run --output-format csv -- \
  python3 bench.py --gpus 2 --scale ${SCALE:-20} --steps 2 --warmup 1 --no-validate --no-int32-pass ${BENCH_ARGS} \
  > gpurun_out/ptrace.log 2>&1 || { tail -30 gpurun_out/ptrace.log; exit 1; }
for f in $(find gpurun_out/ptrace -name "*kernel_trace.csv"); do
  n=$(basename $(dirname $f))
  python3 tools/trace_summary.py "$f" --from-kernel init_run_kernel --runs 1 > gpurun_out/ptrace_${n}.txt || true
  gzip -f "$f"
done
ls gpurun_out/ptrace_*.txt
