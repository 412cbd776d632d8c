#!/bin/bash
# Same-box A/B of two builds: ab/old (a copy of the previous build's package,
# bench.py and tools/run_roots.py) against the working tree.  Per-level
# device-clock times of chosen roots for each option set, then the headline
# bench twice per tree.
#   ROOTS="17872028 57360758" OPTSETS="|bu_lane_limit=4" NEW_BENCH_ARGS="--bu-lane-limit 4" tools/gpu_ab_trees.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/ab_trees.txt
: > $out
ROOTS=${ROOTS:-"8766153 17872028 21909223 22823737 5467067 31770031 57360758 13702079"}
IFS='|' read -ra OS <<< "${OPTSETS:-}"
echo "== ab/old defaults" | tee -a $out
timeout -k 10 200 python ab/old/tools/run_roots.py --roots $ROOTS >> $out 2>&1 || { tail -5 $out; exit 1; }
for tree in .; do
  for o in "${OS[@]}"; do
    args=""
    for kv in $o; do args="$args --opt $kv"; done
    echo "== $tree opts '$o'" | tee -a $out
    timeout -k 10 200 python $tree/tools/run_roots.py --roots $ROOTS $args >> $out 2>&1 || { tail -5 $out; exit 1; }
  done
done
for rep in 1 2; do
  for tree in ab/old .; do
    extra=""
    [ "$tree" = "." ] && extra="${NEW_BENCH_ARGS}"
    timeout -k 10 240 python $tree/bench.py --steps ${STEPS:-32} --warmup 3 --no-validate ${BENCH_ARGS} $extra > gpurun_out/ab_run.json 2> gpurun_out/ab_run.err || { tail -5 gpurun_out/ab_run.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_run.json').read().strip().splitlines()[-1]); print('bench %-8s %8.1f GTEPS %7.3f ms/step' % (sys.argv[1], d['value'], d['ms_per_step']))" "$tree" | tee -a $out
  done
done
