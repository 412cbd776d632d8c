#!/bin/bash
# A/B of bench.py argument sets (one bench run each, same roots):
#   ARGSETS="|--no-id-order" SCALE=26 tools/gpu_ab_args.sh   (empty = defaults)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS='|' read -ra AS <<< "${ARGSETS:-}"
for a in "${AS[@]}"; do
  timeout -k 10 240 python bench.py --scale ${SCALE:-26} --steps ${STEPS:-16} --warmup 3 --no-validate --no-int32-pass $a ${BENCH_ARGS} \
    > gpurun_out/aba_run.json 2> gpurun_out/aba_run.err || { echo "args '$a' failed"; tail -20 gpurun_out/aba_run.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/aba_run.json').read().strip().splitlines()[-1]); print('%-50s %8.1f GTEPS %7.3f ms/step build %.2fs clock %s' % (sys.argv[1] or 'default', d['value'], d['ms_per_step'], d['generate_s'], [(l[0], round(l[1] * 1e3, 1)) for l in d.get('level_clock', {}).get('levels', [])]))" "$a ${BENCH_ARGS}"
done
