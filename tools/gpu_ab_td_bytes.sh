cd "${GRAFT_REPO_ROOT:-/root/repo}"
VARIANTS="base|td_byte_edges=1048576|td_byte_edges=262144|td_byte_edges=65536" bash tools/gpu_ab.sh && cp gpurun_out/ab.txt gpurun_out/ab_do26.txt && \
SCALE=22 BENCH_ARGS="--mode td --no-int32-pass" VARIANTS="base|td_byte_edges=1048576|td_byte_edges=262144|td_byte_edges=65536|td_check_visited_min=0" bash tools/gpu_ab.sh && cp gpurun_out/ab.txt gpurun_out/ab_td22.txt
