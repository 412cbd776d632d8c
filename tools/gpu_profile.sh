#!/bin/bash
# Per-level timing, rocprofv3 kernel statistics and a small heuristic sweep at RMAT-26.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SCALE=${SCALE:-26}
echo "== per-level"
timeout -k 10 300 python bench.py --scale $SCALE --steps 8 --warmup 2 --per-level > gpurun_out/perlevel.log 2>&1 || { tail -30 gpurun_out/perlevel.log; exit 1; }
tail -14 gpurun_out/perlevel.log
echo "== rocprofv3"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --scale $SCALE --steps 8 --warmup 2 --no-validate > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -20 "$f"
echo "== sweep"
for ll in 4 16 32; do
  timeout -k 10 200 python bench.py --scale $SCALE --steps 8 --warmup 2 --no-validate --bu-lane-limit $ll 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lane_limit $ll', d['value'], d['ms_per_step'])" || exit 1
done
for a in 6 30 60; do
  timeout -k 10 200 python bench.py --scale $SCALE --steps 8 --warmup 2 --no-validate --alpha $a 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('alpha $a', d['value'], d['ms_per_step'])" || exit 1
done
for b in 8 64 256; do
  timeout -k 10 200 python bench.py --scale $SCALE --steps 8 --warmup 2 --no-validate --beta $b 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('beta $b', d['value'], d['ms_per_step'])" || exit 1
done
