# Round-5 step: split top-down levels -- GPU tests, then same-process option A/Bs
# (td_split_parts A vs 1, for each A in AS) on RMAT-22 / the LJ-sized graphs, top-down only.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q -m gpu -k "split_levels or byte_map" --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1; rc=$?
tail -3 gpurun_out/split_tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/split_ab.txt
for A in ${AS:-4}; do
  timeout -k 10 400 python -u tools/td_option_ab.py --option td_split_parts --a $A --b 1 --roots 16 ${ABARGS} >> gpurun_out/split_ab.txt 2> gpurun_out/split_ab.err || { tail -20 gpurun_out/split_ab.err; exit 1; }
done
cat gpurun_out/split_ab.txt
