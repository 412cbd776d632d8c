#!/bin/bash
# Kernel timeline of one top-down-only traversal (config 2 class) on the
# soc-LiveJournal1-sized uniform graph and RMAT-22: where each level's time
# goes (compact / td_expand / hub_apply / update).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r4}
for g in "lj:--uniform 4847571:68993773" "r22:--scale 22"; do
  n=${g%%:*}; ga=${g#*:}
  rm -rf gpurun_out/tdtrace
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tdtrace -o run --output-format csv -- \
    python3 bench.py $ga --mode td --steps 3 --warmup 1 --no-validate --heldout-roots 0 --secondary none --no-int32-pass ${TD_ARGS} \
    > gpurun_out/${TAG}_td_trace_$n.json 2> gpurun_out/${TAG}_td_trace_$n.err || { tail -20 gpurun_out/${TAG}_td_trace_$n.err; exit 1; }
  f=$(find gpurun_out/tdtrace -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_summary.py "$f" --from-kernel init_run_kernel --runs 1 > gpurun_out/${TAG}_td_trace_$n.txt
  echo "== $n"; cat gpurun_out/${TAG}_td_trace_$n.txt | cut -c1-100
done
