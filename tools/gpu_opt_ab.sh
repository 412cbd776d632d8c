#!/bin/bash
# Same-box option A/B with the bench itself: default vs --opt OPTS, alternating
# ROUNDS times (headline config unless BENCH_ARGS says otherwise).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
: > gpurun_out/opt_ab.txt
args=""; for o in ${OPTS}; do args="$args --opt $o"; done
for r in $(seq 1 ${ROUNDS:-2}); do
  for side in base opt; do
    a=""; [ $side = opt ] && a="$args"
    timeout -k 10 240 python bench.py --steps ${STEPS:-20} --warmup 5 --heldout-roots 0 --secondary none --no-int32-pass ${BENCH_ARGS} $a \
      > gpurun_out/oab.json 2> gpurun_out/oab.err || { echo "$side failed"; tail -20 gpurun_out/oab.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/oab.json').read().strip().splitlines()[-1]); print('%-5s %8.1f GTEPS %7.4f ms/step %s clock %s' % (sys.argv[1], d['value'], d['ms_per_step'], d['validated_roots'], [(l[0], round(l[1] * 1e3, 1)) for l in d.get('level_clock', {}).get('levels', [])]))" "$side" | tee -a gpurun_out/opt_ab.txt
  done
done
