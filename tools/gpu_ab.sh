#!/bin/bash
# A/B of engine options on the headline bench: one bench run per variant.
#   VARIANTS="base|device_loop=0|alpha=16" tools/gpu_ab.sh
# ("base" = defaults; options are comma-separated NAME=VALUE).  One line of
# GTEPS / ms per variant into gpurun_out/ab.txt.  The roots come from a tuning
# seed (ROOT_SEED, default 4242), not the bench's default 12345 that the
# driver times: options are not tuned on the headline's own roots.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SCALE=${SCALE:-26}
STEPS=${STEPS:-16}
: > gpurun_out/ab.txt
IFS='|' read -ra VS <<< "${VARIANTS:-base|device_loop=0}"
for v in "${VS[@]}"; do
  args=()
  if [ "$v" != "base" ]; then
    IFS=',' read -ra kvs <<< "$v"
    for kv in "${kvs[@]}"; do args+=(--opt "$kv"); done
  fi
  timeout -k 10 240 python bench.py --scale $SCALE --steps $STEPS --warmup 3 --no-validate --root-seed ${ROOT_SEED:-4242} \
    --heldout-roots 0 --secondary none "${args[@]}" ${BENCH_ARGS} \
    > gpurun_out/ab_run.json 2> gpurun_out/ab_run.err || { echo "variant $v failed"; tail -20 gpurun_out/ab_run.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_run.json').read().strip().splitlines()[-1]); print('%-40s %8.1f GTEPS %7.3f ms/step hm %7.1f clock %s' % (sys.argv[1], d['value'], d['ms_per_step'], d['harmonic_mean_gteps'], [(l[0], round(l[1] * 1e3, 1)) for l in d.get('level_clock', {}).get('levels', [])]))" "$v" | tee -a gpurun_out/ab.txt
done
