#!/bin/bash
# Range-staged top-down levels: GPU tests, then top-down-only benches (config 2
# class: soc-LiveJournal1-sized uniform graph, RMAT-22) with the range-staged
# levels on (default) and off, and a kernel trace with them on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r4}
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q -m gpu --timeout 200 --timeout-method thread -k "${PYTEST_K:-td_range or td_direct or rmat_modes}" > gpurun_out/${TAG}_pytest_range.log 2>&1; rc=$?
  tail -3 gpurun_out/${TAG}_pytest_range.log; [ $rc -eq 0 ] || exit $rc
fi
for g in "lj:--uniform 4847571:68993773" "r22:--scale 22"; do
  n=${g%%:*}; ga=${g#*:}
  IFS='|' read -ra VS <<< "${VARIANTS:-on:|off:--opt td_range_edges=0}"
  for v in "${VS[@]}"; do
    vn=${v%%:*}; va=${v#*:}
    timeout -k 10 300 python bench.py $ga --mode td --steps 16 --warmup 3 --heldout-roots 0 --secondary none --no-int32-pass $va ${TD_ARGS} > gpurun_out/${TAG}_td_${n}_${vn}.json 2> gpurun_out/${TAG}_td_${n}_${vn}.err || { tail -20 gpurun_out/${TAG}_td_${n}_${vn}.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.1f GTEPS %.4f ms validated %s' % (d['value'], d['ms_per_step'], d['validated_roots']), [round(l[1]*1000,1) for l in d['level_clock']['levels']])" gpurun_out/${TAG}_td_${n}_${vn}.json "$n $vn"
  done
done
if [ "${TRACE:-1}" = 1 ]; then TAG=${TAG}_range bash tools/gpu_td_trace.sh; fi
