#!/bin/bash
# Compile-time kernel variants, headline bench per variant with per-root level
# times (same roots):  FLAGSETS="|-DDBFS_X=0" ROOTS=8 tools/gpu_variant_levels.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS='|' read -ra FS <<< "${FLAGSETS:-}"
i=0
for f in "${FS[@]}"; do
  d=/tmp/variant_$i; i=$((i+1))
  rm -rf $d && mkdir -p $d && tar -C "$ROOT" --exclude=./gpurun_out --exclude=./build-asan -cf - . | tar -C $d -xf -
  (cd $d && make clean > /dev/null && make -j16 EXTRA_HIPFLAGS="$f" > $ROOT/gpurun_out/variant_make.log 2>&1) || { echo "build failed: $f"; tail -20 gpurun_out/variant_make.log; exit 1; }
  timeout -k 10 240 python $d/bench.py --scale ${SCALE:-26} --steps ${STEPS:-20} --warmup 3 --no-validate --no-int32-pass ${BENCH_ARGS} > gpurun_out/vl_run.json 2> gpurun_out/vl_run.err || { echo "variant '$f' failed"; tail -20 gpurun_out/vl_run.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/vl_run.json').read().strip().splitlines()[-1]); print('%-40s %8.1f GTEPS %7.3f ms/step' % (sys.argv[1] or 'default', d['value'], d['ms_per_step']))" "$f"
  python3 - gpurun_out/vl_run.err ${ROOTS:-6} <<'PY'
import re, sys
n = 0
for line in open(sys.argv[1]):
    m = re.search(r"timed root (\d+): ([\d.]+) ms .* levels (\w+) frontier-edges (\[.*?\]) level-us (\[.*?\])", line)
    if m and n < int(sys.argv[2]):
        n += 1
        print("   ", m.group(1), m.group(2), m.group(3), m.group(5))
PY
done
