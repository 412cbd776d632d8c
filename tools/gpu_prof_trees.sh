#!/bin/bash
# Per-kernel statistics of two builds on the same box (rocprofv3 --kernel-trace
# --stats): the older build in _ab_old/ and this tree, the headline config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in old new; do
  d=.; [ $t = old ] && d=_ab_old
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$t -o run -- python3 $d/bench.py --steps 10 --warmup 3 \
    --heldout-roots 0 --secondary none --no-int32-pass --no-validate ${BENCH_ARGS} > gpurun_out/prof_$t.log 2>&1 || { tail -20 gpurun_out/prof_$t.log; exit 1; }
done
find gpurun_out/prof_old gpurun_out/prof_new -name "*kernel_stats.csv" | head
