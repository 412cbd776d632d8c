# Round-5 step: the unvisited filter -- its GPU tests, then a same-process A/B (on / off) in top-down-only and
# direction-optimising modes on the LiveJournal-sized graphs and RMAT-22.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r5u}
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v -k "unvisited_filter or all_reached" --timeout 150 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && exit $rc
for M in td do; do
  timeout -k 10 400 python -u tools/td_option_ab.py --mode $M --roots 16 --option td_unvis_edges --a 4194304 --b 0 \
    --json gpurun_out/${T}_ab_$M.json > gpurun_out/${T}_ab_$M.txt 2>&1 || { tail -20 gpurun_out/${T}_ab_$M.txt; exit 1; }
  grep -v "^\[" gpurun_out/${T}_ab_$M.txt
done
