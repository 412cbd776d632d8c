# Round-6 step: per-level gaps of chosen RMAT-26 roots, then the P = 8 direction-policy sweep.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/run_roots.py --roots 8766153 17872028 41169583 63203320 > gpurun_out/r6gaps.txt 2>&1 || { tail -20 gpurun_out/r6gaps.txt; exit 1; }
cat gpurun_out/r6gaps.txt
bash tools/gpu_r6_policy.sh
