#!/bin/bash
# Same-box A/B of a compile-time kernel variant: the tree as is (A) against a copy built with
# EXTRA_HIPFLAGS="$FLAGS" (B), alternating bench runs, then per-level times of chosen roots.
#   FLAGS="-DDBFS_BU_DEEP" ROOTS="41169583 8766153" bash tools/gpu_variant_ab2.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
ROOT=$PWD; T=${TAG:-vab}
d=/tmp/vab_tree
rm -rf $d && mkdir -p $d && tar -C "$ROOT" --exclude=./gpurun_out --exclude=./build-asan -cf - . | tar -C $d -xf -
(cd $d && make clean > /dev/null && make -j16 EXTRA_HIPFLAGS="$FLAGS" > $ROOT/gpurun_out/${T}_make.log 2>&1) || { tail -20 gpurun_out/${T}_make.log; exit 1; }
for rep in 1 2; do
  for side in A B; do
    dir=$ROOT; [ $side = B ] && dir=$d
    timeout -k 10 300 python3 -u $dir/bench.py --steps 16 --warmup 2 --secondary none --no-int32-pass > gpurun_out/${T}_$side$rep.json 2> gpurun_out/${T}_$side$rep.err || { tail -20 gpurun_out/${T}_$side$rep.err; exit 1; }
    python3 - gpurun_out/${T}_$side$rep.json $side <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "headline", r["value"], "heldout", r["heldout"]["value"], r["validated_roots"], r["heldout"]["validated_roots"])
PY
  done
done
for side in A B; do
  dir=$ROOT; [ $side = B ] && dir=$d
  echo "== $side"; timeout -k 10 200 python3 -u $dir/tools/run_roots.py --roots ${ROOTS:-41169583 8766153 63203320} 2>&1 | cut -c1-230
done
