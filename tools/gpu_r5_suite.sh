# Round-5 step: the full GPU test suite and the smoke entry point.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r5k}
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_smoke.log; exit $rc
