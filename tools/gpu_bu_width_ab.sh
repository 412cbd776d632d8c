#!/bin/bash
# RMAT-26 one GPU: bottom-up words per wave -- whole units (default), 16-word
# waves (bu_whole_units=-1), 4-word first levels (+ bu_small_waves=1); same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/bu_width_ab.txt
for r in 1 2; do
  for v in "whole:" "w16:--opt bu_whole_units=-1" "w4:--opt bu_whole_units=-1 --opt bu_small_waves=1"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --heldout-roots 0 --secondary none --no-int32-pass ${BENCH_ARGS} $a > gpurun_out/bw.json 2> gpurun_out/bw.err || { tail -20 gpurun_out/bw.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/bw.json').read().strip().splitlines()[-1]); print('%-6s %8.1f GTEPS %7.4f ms %s clock %s' % (sys.argv[1], d['value'], d['ms_per_step'], d['validated_roots'], [(l[0], round(l[1]*1e3,1)) for l in d['level_clock']['levels']]))" $n | tee -a gpurun_out/bu_width_ab.txt
  done
done
