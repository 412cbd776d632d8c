# Round-5 step: same-box A/B of this tree against _ab_old/ -- RMAT-26 bench (driver roots),
# RMAT-22 top-down only, shadow rank 0 of P = 8 (usual + late roots).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r5t}
ROUNDS=2 bash tools/gpu_ab_trees.sh && cp gpurun_out/ab_trees.txt gpurun_out/${T}_r26.txt &&
ROUNDS=2 BENCH_ARGS="--scale 22 --mode td" bash tools/gpu_ab_trees.sh && cp gpurun_out/ab_trees.txt gpurun_out/${T}_r22td.txt &&
SUFFIX=${T}u PS=8 ROUNDS=2 bash tools/gpu_shadow_ab_trees.sh &&
SUFFIX=${T}l PS=8 ROUNDS=2 SHADOW_ARGS="--root-list 8766153 17872028 21909223 5467067" bash tools/gpu_shadow_ab_trees.sh
