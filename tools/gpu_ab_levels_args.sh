#!/bin/bash
# A/B of bench.py argument sets with per-root level times (same roots):
#   ARGSETS="|--bu-lane-limit 32" ROOTS=20 tools/gpu_ab_levels_args.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS='|' read -ra AS <<< "${ARGSETS:-}"
for a in "${AS[@]}"; do
  timeout -k 10 240 python bench.py --scale ${SCALE:-26} --steps ${STEPS:-20} --warmup 3 --no-validate --no-int32-pass $a ${BENCH_ARGS} \
    > gpurun_out/abl_run.json 2> gpurun_out/abl_run.err || { echo "args '$a' failed"; tail -20 gpurun_out/abl_run.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/abl_run.json').read().strip().splitlines()[-1]); print('%-40s %8.1f GTEPS %7.3f ms/step' % (sys.argv[1] or 'default', d['value'], d['ms_per_step']))" "$a"
  python3 - gpurun_out/abl_run.err ${ROOTS:-20} <<'PY'
import re, sys
n = 0
for line in open(sys.argv[1]):
    m = re.search(r"timed root (\d+): ([\d.]+) ms .* levels (\w+) frontier-edges (\[.*?\]) level-us (\[.*?\])", line)
    if m and n < int(sys.argv[2]):
        n += 1
        print("   ", m.group(1), m.group(2), m.group(3), m.group(5))
PY
done
