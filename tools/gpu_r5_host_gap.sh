# Round-5 step: where the wall time between back-to-back runs goes (one GPU, RMAT-26): the host
# timeline (DBFS_HOST_TIMING=1) and a kernel trace of the timed runs (gaps between runs).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r5h}
DBFS_HOST_TIMING=1 timeout -k 10 200 ./bin/bfs --rmat 26 --roots 8 --no-oracle > gpurun_out/${T}_host_timing.txt 2>&1 || { tail -20 gpurun_out/${T}_host_timing.txt; exit 1; }
grep -i "since_prev\|aggregate" gpurun_out/${T}_host_timing.txt | tail -12
rm -rf gpurun_out/${T}_trace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_trace -o run -- ./bin/bfs --rmat 26 --roots 8 --no-oracle > gpurun_out/${T}_trace.log 2>&1 || { tail -20 gpurun_out/${T}_trace.log; exit 1; }
f=$(find gpurun_out/${T}_trace -name "*kernel_trace.csv")
python3 tools/trace_summary.py $f --from-kernel init_run_kernel --runs 3 > gpurun_out/${T}_trace3.txt
gzip -f $f
grep -n "init_run" gpurun_out/${T}_trace3.txt; tail -2 gpurun_out/${T}_trace3.txt
