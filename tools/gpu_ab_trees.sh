#!/bin/bash
# Same-box A/B of two builds: this tree's bench against an older build copied
# into _ab_old/ (bench.py + the package with its extension), alternating
# OLD / NEW ROUNDS times on the headline config (driver's roots unless
# BENCH_ARGS says otherwise).  One line per run into gpurun_out/ab_trees.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ab_trees.txt
for r in $(seq 1 ${ROUNDS:-2}); do
  for t in ${TREES:-_ab_old .}; do
    timeout -k 10 240 python $t/bench.py --steps ${STEPS:-20} --warmup 5 --heldout-roots 0 --secondary none --no-int32-pass ${BENCH_ARGS} \
      > gpurun_out/abt.json 2> gpurun_out/abt.err || { echo "tree $t failed"; tail -20 gpurun_out/abt.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/abt.json').read().strip().splitlines()[-1]); print('%-8s %8.1f GTEPS %7.4f ms/step %s held-out %s clock %s' % (sys.argv[1], d['value'], d['ms_per_step'], d['validated_roots'], (d.get('heldout') or {}).get('value'), [(l[0], round(l[1] * 1e3, 1)) for l in d.get('level_clock', {}).get('levels', [])]))" "$t" | tee -a gpurun_out/ab_trees.txt
  done
done
