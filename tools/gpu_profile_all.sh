#!/bin/bash
# Everything profiles/ records for one version: headline bench (JSON + per-level
# log), rocprofv3 kernel statistics, bottom-up per-dispatch counters.
#   TAG=v10 tools/gpu_profile_all.sh   -> gpurun_out/prof_<TAG>/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-cur}
OUT=gpurun_out/prof_$TAG
rm -rf $OUT && mkdir -p $OUT
echo "== bench"
timeout -k 10 300 python bench.py --steps 16 --warmup 3 --per-level > $OUT/bench.json 2> $OUT/bench.log || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.json
echo "== rocprofv3 --kernel-trace --stats"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/rp -o bench --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-validate > $OUT/rocprof.log 2>&1 || { tail -20 $OUT/rocprof.log; exit 1; }
f=$(find $OUT/rp -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv
t=$(find $OUT/rp -name "*kernel_trace.csv" | head -1); python3 tools/trace_summary.py "$t" --runs 2 > $OUT/trace_summary.txt
rm -rf $OUT/rp
head -12 $OUT/kernel_stats.csv | cut -c1-150
echo "== bottom-up counters"
bash tools/gpu_counters_bu.sh > /dev/null && cp gpurun_out/counters_bu.txt $OUT/counters_bu.txt && head -5 $OUT/counters_bu.txt
