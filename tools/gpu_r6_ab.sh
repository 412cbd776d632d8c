# Round-6 step: GPU suite + grid probe + default bench (an A/B point of the current tree).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r6ab}
if [ -z "$NOSUITE" ]; then
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 200 python3 -u tools/grid_probe.py > gpurun_out/${T}_probe.txt 2>&1 || { tail -20 gpurun_out/${T}_probe.txt; exit 1; }
cat gpurun_out/${T}_probe.txt
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
python3 - gpurun_out/${T}_bench.json <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("headline", r["value"], "ms", r["ms_per_step"], "int32", r.get("value_int32_levels"), "heldout", (r.get("heldout") or {}).get("value"))
for k, b in (r.get("secondary") or {}).items():
    print(k, {m: (b[m]["value"], b[m].get("us_per_level")) for m in ("td", "do")})
PY
