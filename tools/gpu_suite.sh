# GPU suite + default bench on one MI355X (run through gpurun from the repo root).
# Usage: bash tools/gpu_suite.sh TAG [pytest -k expression]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
tag=${1:-suite}; k=${2:-}
args=(tests/ -x -v -m gpu --timeout 150 --timeout-method thread)
[ -n "$k" ] && args+=(-k "$k")
timeout -k 10 900 python -u -m pytest "${args[@]}" > gpurun_out/${tag}_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/${tag}_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err; rc=$?
tail -c 1500 gpurun_out/${tag}_bench.json
exit $rc
