# Round-6 step: the several-rank hub cut (bu_cut_ranks) -- GPU tests that reach it, then
# shadow replays at P = 2 / 4 / 8 with the cut off (bu_cut_ranks=1) and on (the default).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r6xc}
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_engine.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "${KTESTS:-hub_cut or shadow or peer_fused or gpus or multirank or all_reached_stop_peer}" > gpurun_out/${T}_pytest.log 2>&1 \
  || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
for P in ${PS:-2 8 4}; do
  P=$P TAG=${T} CONFIGS="bu_cut_ranks=1|base" bash tools/gpu_r6_policy.sh || exit 1
done
