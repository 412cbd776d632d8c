# Round-6 step: kernel timeline of one-GPU traversals of chosen RMAT-26 roots (the last
# traversal of each root listed kernel by kernel; run_roots.py runs each root twice).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r6rt}
rm -rf gpurun_out/${T}_trace
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_trace -o run --output-format csv -- python3 tools/run_roots.py --roots ${ROOTS:-8766153} ${OPTS} > gpurun_out/${T}_roots.txt 2>&1 || { tail -20 gpurun_out/${T}_roots.txt; exit 1; }
grep -v "^W2026\|^E2026" gpurun_out/${T}_roots.txt | tail -5
k=$(find gpurun_out/${T}_trace -name "*kernel_trace.csv" | head -1)
gzip -f "$k"
