#!/bin/bash
# Per-root, per-level device times of the headline bench for a few option sets
# (same roots every run): VARIANTS="base|td_byte_edges=65536" tools/gpu_ab_levels.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS='|' read -ra VS <<< "${VARIANTS:-base}"
i=0
for v in "${VS[@]}"; do
  args=()
  if [ "$v" != "base" ]; then IFS=',' read -ra kvs <<< "$v"; for kv in "${kvs[@]}"; do args+=(--opt "$kv"); done; fi
  timeout -k 10 240 python bench.py --scale ${SCALE:-26} --steps ${STEPS:-20} --warmup 3 --no-validate --no-int32-pass "${args[@]}" ${BENCH_ARGS} \
    > gpurun_out/abl_$i.json 2> gpurun_out/abl_$i.err || { echo "variant $v failed"; tail -20 gpurun_out/abl_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-40s %8.1f GTEPS %7.3f ms/step' % (sys.argv[2], d['value'], d['ms_per_step']))" gpurun_out/abl_$i.json "$v"
  python3 - gpurun_out/abl_$i.err ${ROOTS:-8} <<'PY'
import re, sys
n = 0
for line in open(sys.argv[1]):
    m = re.search(r"timed root (\d+): ([\d.]+) ms .* levels (\w+) frontier-edges (\[.*?\]) level-us (\[.*?\])", line)
    if m and n < int(sys.argv[2]):
        n += 1
        print("   ", m.group(1), m.group(2), m.group(3), m.group(4), m.group(5))
PY
  i=$((i+1))
done
