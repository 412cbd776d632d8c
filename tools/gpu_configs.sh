#!/bin/bash
# The BASELINE.json single-GPU configurations beyond the headline: RMAT-24
# direction-optimising, a soc-LiveJournal1-sized synthetic stand-in (RMAT-22,
# edge factor 16: 4.2 M vertices / 67 M edges; the real file is not available
# offline) top-down and direction-optimising, RMAT-27 (the 8-GPU graph) on one
# GPU, and the reference algorithm on RMAT-22 / RMAT-24 for the ratio.
#   tools/gpu_configs.sh -> gpurun_out/configs/*.json + summary.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/configs
rm -rf $OUT && mkdir -p $OUT
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.log || { echo "$name failed"; tail -5 $OUT/$name.log; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-28s %10.2f GTEPS %9.3f ms/BFS (mean %8.3f) validated %s depth %.1f' % (sys.argv[2], d['value'], d['ms_per_step'], d['bfs_ms_mean'], d['validated'], d['depth_mean']))" $OUT/$name.json $name | tee -a $OUT/summary.txt
}
run rmat24_do --scale 24 --mode do --steps 16 --warmup 3 &&
run rmat22_td --scale 22 --mode td --steps 16 --warmup 3 &&
run rmat22_do --scale 22 --mode do --steps 16 --warmup 3 &&
run rmat27_do --scale 27 --mode do --steps 8 --warmup 2 &&
run rmat22_ref --scale 22 --mode ref --steps 4 --warmup 1 &&
run rmat24_ref --scale 24 --mode ref --steps 2 --warmup 1
