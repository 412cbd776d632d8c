#!/bin/bash
# Kernel timeline of a real two-process run over the peer-memory transport
# (both ranks on this one GPU, DBFS_DEVICE=0): each rank under its own
# rocprofv3 (the program itself after --), rank 0's last traversal summarised.
# Shows the multi-rank level chains as they run -- the next bottom-up level's
# frontier pushed by the kernels that produce it (no level-end copy between
# bottom-up kernels), direct list exchanges, folded level ends.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r5p}; S=${SCALE:-24}
port() { python3 -c "import socket; s=socket.socket(); s.bind(('127.0.0.1', 0)); print(s.getsockname()[1])"; }
export WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$(port) DBFS_BOOTSTRAP_PORT=$(port) \
  DBFS_DEVICE=0 DBFS_SPAWNED=1 HSA_ENABLE_IPC_MODE_LEGACY=0 DBFS_COMM=peer
rm -rf gpurun_out/${T}_ptrace_r0 gpurun_out/${T}_ptrace_r1
pids=()
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_ptrace_r$r -o run -- \
    python3 bench.py --gpus 2 --scale $S --steps ${STEPS:-4} --warmup 1 --no-int32-pass --heldout-roots 0 --secondary none \
    ${BENCH_ARGS} > gpurun_out/${T}_ptrace_r$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
[ $rc -eq 0 ] || { tail -20 gpurun_out/${T}_ptrace_r0.log gpurun_out/${T}_ptrace_r1.log; exit $rc; }
f=$(find gpurun_out/${T}_ptrace_r0 -name "*kernel_trace.csv")
python3 tools/trace_summary.py $f --from-kernel init_run_kernel --runs 1 > gpurun_out/${T}_peer_trace_s${S}_p2_r0.txt
gzip -f $f
head -c 600 gpurun_out/${T}_ptrace_r0.log | tail -c 300
tail -3 gpurun_out/${T}_peer_trace_s${S}_p2_r0.txt
