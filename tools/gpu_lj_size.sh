#!/bin/bash
# soc-LiveJournal1-sized configuration (BASELINE config 2) through the
# reference's file path: a synthetic uniform-random edge list with exactly
# LiveJournal's 4,847,571 vertices (odd N: the reference's D5 tail case) and
# 68,993,773 edges, written in the reference format, then
#   1. bench.py --graph <file> --mode td   (top-down only, as the reference)
#   2. bench.py --graph <file> --mode do
#   3. ./bin/bfs 0 <file>                  (reference CLI contract + CPU oracle)
# No dataset ships with the repo and the pool has no network: parity with the
# real soc-LiveJournal1 is unpinned; the RMAT-22 runs are the power-law stand-in.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/lj
export TMPDIR=/tmp
F=/tmp/lj_size_uniform.txt
O=gpurun_out/lj
timeout -k 10 300 python3 -c "
import sys, distributed_cuda_bfs_amd as dbfs
dbfs.native.write_generated_edge_list(sys.argv[1], dbfs.uniform_params(4847571, 68993773, 7), 16)
" "$F" || { echo "write failed"; exit 1; }
ls -la "$F"
for mode in td do; do
  timeout -k 10 400 python bench.py --graph "$F" --mode $mode --steps 16 --warmup 3 > $O/bench_$mode.json 2> $O/bench_$mode.log \
    || { tail -20 $O/bench_$mode.log; rm -f "$F"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], 'GTEPS', d['ms_per_step'], 'ms/step', d['validated_roots'], 'int32', d.get('value_int32_levels'), 'load', d['generate_s'], 's rss', d['host_peak_rss_gb'])" $O/bench_$mode.json $mode
done
timeout -k 10 300 ./bin/bfs 0 "$F" > $O/cli.log 2>&1; rc=$?
head -12 $O/cli.log
rm -f "$F"
exit $rc
