#!/bin/bash
# Many validated roots (every timed root checked by the device validator and
# against its rerun's totals): RMAT-26 128, RMAT-24 128, RMAT-27 48, and
# RMAT-26 with 32-bit levels only in the timed loop.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift
  timeout -k 10 500 python bench.py "$@" > gpurun_out/many_$name.json 2> gpurun_out/many_$name.err || { tail -20 gpurun_out/many_$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-10s %8.1f GTEPS validated %s int32 %s' % (sys.argv[2], d['value'], d['validated_roots'], d.get('value_int32_levels')))" gpurun_out/many_$name.json $name; }
run s26 --steps 128 --warmup 3 --root-seed 777 &&
run s24 --scale 24 --steps 128 --warmup 3 --root-seed 778 &&
run s27 --scale 27 --steps 48 --warmup 2 --root-seed 779 &&
run s26w --steps 64 --warmup 3 --root-seed 780 --opt narrow_levels=0
