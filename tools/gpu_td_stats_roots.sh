#!/bin/bash
# Top-down event counters (diagnostic build -DDBFS_TD_STATS in a copy of the
# tree), host loop so every level's dispatch reports in order.
#   ROOTS="4145886" SCALE=22 MODE=td tools/gpu_td_stats_roots.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$PWD
mkdir -p gpurun_out
d=/tmp/td_stats_tree
rm -rf $d && mkdir -p $d && tar -C "$ROOT" --exclude=./gpurun_out --exclude=./build-asan -cf - . | tar -C $d -xf -
(cd $d && make clean > /dev/null && make -j16 EXTRA_HIPFLAGS="-DDBFS_TD_STATS" > $ROOT/gpurun_out/td_stats_make.log 2>&1) || { tail -20 gpurun_out/td_stats_make.log; exit 1; }
timeout -k 10 240 python $d/tools/run_roots.py --scale ${SCALE:-22} --mode ${MODE:-td} --roots ${ROOTS} ${OPTS} > gpurun_out/td_stats_roots.log 2>&1 || { tail -20 gpurun_out/td_stats_roots.log; exit 1; }
grep -vE "^\s*$" gpurun_out/td_stats_roots.log | tail -40
