#!/bin/bash
# Hub cut with 32-bit levels: GPU tests, then validated benches reporting both
# the narrow-level value and value_int32_levels, cut on / off, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q -m gpu -k "hub_cut or long_row or hub_lds or narrow" --timeout 200 --timeout-method thread > gpurun_out/cutw_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/cutw_pytest.log; [ $rc -eq 0 ] || exit $rc
for a in "" "--opt bu_cut_edges=0" ""; do
  timeout -k 10 300 python bench.py --steps 32 --warmup 3 $a > gpurun_out/cutw.json 2> gpurun_out/cutw.err || { tail -20 gpurun_out/cutw.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/cutw.json').read().strip().splitlines()[-1]); print('%-24s %8.1f GTEPS  int32 levels %8.1f GTEPS  validated %s' % (sys.argv[1] or 'default', d['value'], d['value_int32_levels'], d['validated_roots']))" "$a"
done
