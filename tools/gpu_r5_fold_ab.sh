cd "${GRAFT_REPO_ROOT:-/root/repo}"
SUFFIX=late PS=8 ROUNDS=2 SHADOW_ARGS="--root-list 8766153 17872028 21909223 5467067" bash tools/gpu_shadow_ab_trees.sh &&
SUFFIX=usual PS="8 2" ROUNDS=2 bash tools/gpu_shadow_ab_trees.sh &&
ROUNDS=3 BENCH_ARGS="--scale 22 --mode td" bash tools/gpu_ab_trees.sh && cp gpurun_out/ab_trees.txt gpurun_out/ab_trees_r22td.txt
