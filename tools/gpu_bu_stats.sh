#!/bin/bash
# Bottom-up event counters (diagnostic build -DDBFS_BU_STATS in a copy of the
# tree, one report per bottom-up launch, synchronised).
#   ROOTS="8766153 17872028" bash tools/gpu_bu_stats.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$PWD
mkdir -p gpurun_out
d=/tmp/bu_stats_tree
rm -rf $d && mkdir -p $d && tar -C "$ROOT" --exclude=./gpurun_out --exclude=./build-asan -cf - . | tar -C $d -xf -
(cd $d && make clean > /dev/null && make -j16 EXTRA_HIPFLAGS="-DDBFS_BU_STATS" > $ROOT/gpurun_out/bu_stats_make.log 2>&1) || { tail -20 gpurun_out/bu_stats_make.log; exit 1; }
timeout -k 10 240 python3 $d/tools/run_roots.py --roots ${ROOTS:-8766153 17872028 41169583} > gpurun_out/bu_stats.txt 2>&1 || { tail -20 gpurun_out/bu_stats.txt; exit 1; }
grep -E "bu-stats|^[0-9]" gpurun_out/bu_stats.txt | tail -30
