#!/bin/bash
# Bottom-up event counters (diagnostic build -DDBFS_BU_STATS in a copy of the
# tree) for chosen roots, host loop so every level's dispatch reports in order.
#   ROOTS="17872028 57360758" tools/gpu_bu_stats_roots.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$PWD
mkdir -p gpurun_out
d=/tmp/bu_stats_tree
rm -rf $d && mkdir -p $d && tar -C "$ROOT" --exclude=./gpurun_out --exclude=./build-asan -cf - . | tar -C $d -xf -
(cd $d && make clean > /dev/null && make -j16 EXTRA_HIPFLAGS="-DDBFS_BU_STATS" > $ROOT/gpurun_out/bu_stats_make.log 2>&1) || { tail -20 gpurun_out/bu_stats_make.log; exit 1; }
timeout -k 10 240 python $d/tools/run_roots.py --scale ${SCALE:-26} --roots ${ROOTS} --opt device_loop=0 > gpurun_out/bu_stats_roots.log 2>&1 || { tail -20 gpurun_out/bu_stats_roots.log; exit 1; }
grep -vE "^\s*$" gpurun_out/bu_stats_roots.log | tail -30
