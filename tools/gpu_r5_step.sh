cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/r5e_pytest.log 2>&1; rc=$?
tail -12 gpurun_out/r5e_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/shard_rehearsal.py --ranks 8 --roots 4 --json gpurun_out/r5e_friendster_p8.json > gpurun_out/r5e_friendster_p8.out 2> gpurun_out/r5e_friendster_p8.err; rc=$?
tail -14 gpurun_out/r5e_friendster_p8.err; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r5e_bench.json 2> gpurun_out/r5e_bench.err; rc=$?
grep "secondary\|held-out" gpurun_out/r5e_bench.err
[ $rc -ne 0 ] && exit $rc
export TAG=r5e ROOTS=8 SHADOW_ARGS="--root-list 13702079 43129764 45382682 26246917 8766153 17872028 21909223 5467067"
CFGS="26:2:0,1;26:8:0,7" bash tools/gpu_shadow.sh || exit 1
export ROOTS=4 SHADOW_ARGS=""
CFGS="27:8:0,7" bash tools/gpu_shadow.sh
