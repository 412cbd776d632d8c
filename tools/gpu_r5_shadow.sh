# Round-5 GPU step B: shadow ranks (tools/gpu_shadow.sh) -- RMAT-26 at P = 2 / 8 on the four
# usual and four late-switch roots, RMAT-27 at P = 8, and the weak series RMAT-25 at P = 2,
# RMAT-26 at P = 4 (with RMAT-24 / 27 at P = 1 / 8 from the others).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
export TAG=${TAG:-r5s} ROOTS=8 SHADOW_ARGS="--root-list 13702079 43129764 45382682 26246917 8766153 17872028 21909223 5467067"
CFGS=${CFGS8:-"26:2:0,1;26:8:0,7"} bash tools/gpu_shadow.sh || exit 1
export ROOTS=4 SHADOW_ARGS=""
CFGS=${CFGS4:-"27:8:0,7;25:2:0,1;26:4:0,3"} bash tools/gpu_shadow.sh
