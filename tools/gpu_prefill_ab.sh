#!/bin/bash
# 32-bit-level pass with the level prefill on / off (value_int32_levels), RMAT-26, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in "on:" "off:--opt prefill_levels=0"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --heldout-roots 0 --secondary none $a > gpurun_out/pf_$n.json 2> gpurun_out/pf_$n.err || { tail -20 gpurun_out/pf_$n.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-4s %8.1f GTEPS  int32 %8.1f  %s' % (sys.argv[2], d['value'], d['value_int32_levels'], d['validated_roots']))" gpurun_out/pf_$n.json $n | tee -a gpurun_out/r4_s3i_prefill_ab.txt
  done
done
