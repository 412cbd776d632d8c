#!/bin/bash
# Hub cut on / off, validated benches (every timed root checked), same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for a in "" "--opt bu_cut_edges=0" "" "--opt bu_cut_edges=0"; do
  timeout -k 10 300 python bench.py --steps 32 --warmup 3 --no-int32-pass $a > gpurun_out/cutv.json 2> gpurun_out/cutv.err || { tail -20 gpurun_out/cutv.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/cutv.json').read().strip().splitlines()[-1]); print('%-24s %8.1f GTEPS %7.4f ms/step validated %s' % (sys.argv[1] or 'default', d['value'], d['ms_per_step'], d['validated_roots']))" "$a"
done
