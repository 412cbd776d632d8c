#!/bin/bash
# Sweep of bench arguments on one box: each entry of VARIANTS (';'-separated
# argument strings) runs the headline bench with its held-out roots once.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS=';' read -ra vs <<< "${VARIANTS:---alpha 24 --beta 96}"
i=0
for v in "${vs[@]}"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-int32-pass --secondary none $v > gpurun_out/sweep_$i.json 2> gpurun_out/sweep_$i.err || { echo "variant '$v' failed"; tail -20 gpurun_out/sweep_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); h=d.get('heldout') or {}; print('%-28s %8.1f %s  heldout %s %s' % (sys.argv[2], d['value'], d['validated_roots'], h.get('value'), h.get('validated_roots')))" gpurun_out/sweep_$i.json "$v"
  i=$((i+1))
done
