#!/bin/bash
# Top-down-only (config 2) per-level profile: the soc-LiveJournal1-sized
# uniform graph and RMAT-22, mode td.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r4}
timeout -k 10 300 python bench.py --uniform 4847571:68993773 --mode td --steps 16 --warmup 3 --per-level --heldout-roots 0 --secondary none --no-int32-pass ${TD_ARGS} > gpurun_out/${TAG}_td_lj.json 2> gpurun_out/${TAG}_td_lj.err || { tail -20 gpurun_out/${TAG}_td_lj.err; exit 1; }
timeout -k 10 300 python bench.py --scale 22 --mode td --steps 16 --warmup 3 --per-level --heldout-roots 0 --secondary none --no-int32-pass ${TD_ARGS} > gpurun_out/${TAG}_td_r22.json 2> gpurun_out/${TAG}_td_r22.err || { tail -20 gpurun_out/${TAG}_td_r22.err; exit 1; }
python3 - <<PY
import json
for n in ("td_lj", "td_r22"):
    d = json.loads(open(f"gpurun_out/${TAG}_{n}.json").read().strip().splitlines()[-1])
    print(n, "%.1f GTEPS %.4f ms/step validated %s" % (d["value"], d["ms_per_step"], d["validated_roots"]))
PY
grep -h "per-level\|  level" gpurun_out/${TAG}_td_lj.err gpurun_out/${TAG}_td_r22.err | head -60
