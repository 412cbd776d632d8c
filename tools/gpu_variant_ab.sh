#!/bin/bash
# A/B of compile-time kernel variants: the tree is copied per variant, built
# with EXTRA_HIPFLAGS, and the headline bench run from the copy.
#   FLAGSETS="|-DDBFS_BU_BATCH=8" tools/gpu_variant_ab.sh   (empty = default build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/variant_ab.txt
IFS='|' read -ra FS <<< "${FLAGSETS:-}"
i=0
for f in "${FS[@]}"; do
  d=/tmp/variant_$i; i=$((i+1))
  rm -rf $d && mkdir -p $d && tar -C "$ROOT" --exclude=./gpurun_out --exclude=./build-asan -cf - . | tar -C $d -xf -
  (cd $d && make clean > /dev/null && make -j16 EXTRA_HIPFLAGS="$f" > $ROOT/gpurun_out/variant_make.log 2>&1) || { echo "build failed: $f"; tail -20 gpurun_out/variant_make.log; exit 1; }
  for rep in 1 2; do
    timeout -k 10 240 python $d/bench.py --steps ${STEPS:-16} --warmup 3 --no-validate ${BENCH_ARGS} > gpurun_out/variant_run.json 2> gpurun_out/variant_run.err || { echo "variant '$f' failed"; tail -20 gpurun_out/variant_run.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/variant_run.json').read().strip().splitlines()[-1]); print('%-40s %8.1f GTEPS %7.3f ms/step  levels %s' % (sys.argv[1] or 'default', d['value'], d['ms_per_step'], [l[1] for l in d['level_profile']['levels']]))" "$f" | tee -a gpurun_out/variant_ab.txt
  done
done
