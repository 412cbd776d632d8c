#!/bin/bash
# End-of-session evidence: headline bench JSON (RMAT-26, 1 GPU), top-down-only
# RMAT-22 and direction-optimising RMAT-24 / RMAT-27 bench JSONs, and a
# rocprofv3 kernel-statistics pass over a short RMAT-26 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
O=gpurun_out/final
run() {  # name, timeout, bench args...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $t python bench.py "$@" > $O/$name.json 2> $O/$name.log || { tail -20 $O/$name.log; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%s %.1f GTEPS %.4f ms/step validated %s int32 %s' % (sys.argv[2], d['value'], d['ms_per_step'], d.get('validated_roots'), d.get('value_int32_levels')))" $O/$name.json $name
}
run rmat26_do 400 --steps 16 --warmup 3 --per-level &&
run rmat22_td 300 --scale 22 --mode td --steps 16 --warmup 3 &&
run rmat24_do 300 --scale 24 --steps 16 --warmup 3 &&
run rmat27_do 500 --scale 27 --steps 8 --warmup 2 &&
echo "== rocprofv3 stats" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-validate --no-int32-pass > $O/prof.log 2>&1 &&
f=$(find $O/prof -name "*kernel_stats.csv" | head -1) && cp "$f" $O/rmat26_kernel_stats.csv && head -12 $O/rmat26_kernel_stats.csv | cut -c1-160 &&
find $O/prof -name "*kernel_trace.csv" -delete
