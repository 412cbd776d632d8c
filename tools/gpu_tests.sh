cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/s3d_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/s3d_pytest.log; exit $rc
