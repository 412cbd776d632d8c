# Round-5 step: kernel timelines of shadow rank 0 for root 13702079 at P = 2 and P = 8 (RMAT-26).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
export TAG=${TAG:-r5t} ROOTS=1 SHADOW_ARGS="--root-list 13702079"
P=2 R=0 bash tools/gpu_shadow_trace.sh && P=8 R=0 bash tools/gpu_shadow_trace.sh
