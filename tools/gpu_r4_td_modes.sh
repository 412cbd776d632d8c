#!/bin/bash
# Top-down-only A/B of the direct level stores' mode (td_store_mode 0 / 1 / 2)
# on RMAT-22 and the soc-LiveJournal1-sized uniform graph (tuning root seed).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r4}
: > gpurun_out/${TAG}_td_modes.txt
for g in "--scale 22" "--uniform 4847571:68993773"; do
  for m in ${MODES:-0 1 2}; do
    timeout -k 10 200 python bench.py $g --mode td --steps 16 --warmup 3 --root-seed 4242 --heldout-roots 0 --secondary none \
        --no-int32-pass --opt td_store_mode=$m > gpurun_out/tdm.json 2> gpurun_out/tdm.err || { tail -20 gpurun_out/tdm.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/tdm.json').read().strip().splitlines()[-1]); print('%-32s store_mode %s %8.2f GTEPS %7.4f ms/step %s' % (sys.argv[1], sys.argv[2], d['value'], d['ms_per_step'], d['validated_roots']))" "$g" "$m" | tee -a gpurun_out/${TAG}_td_modes.txt
  done
done
