#!/bin/bash
# Bottom-up event counters (diagnostic build -DDBFS_BU_STATS in a copy of the
# tree, device loop off so each level's dispatch is reported in order).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$PWD
mkdir -p gpurun_out
d=/tmp/bu_stats_tree
rm -rf $d && mkdir -p $d && tar -C "$ROOT" --exclude=./gpurun_out --exclude=./build-asan -cf - . | tar -C $d -xf -
(cd $d && make clean > /dev/null && make -j16 EXTRA_HIPFLAGS="-DDBFS_BU_STATS" > $ROOT/gpurun_out/bu_stats_make.log 2>&1) || { tail -20 gpurun_out/bu_stats_make.log; exit 1; }
timeout -k 10 240 python $d/bench.py --steps 2 --warmup 1 --no-validate --opt device_loop=0 ${BENCH_ARGS} > gpurun_out/bu_stats.json 2> gpurun_out/bu_stats.log || { tail -20 gpurun_out/bu_stats.log; exit 1; }
grep -E "bu-stats|timed root" gpurun_out/bu_stats.log | tail -20
