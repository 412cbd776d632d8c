# Round-5 GPU step A: full GPU suite, Friendster-sized 8-rank shard rehearsal, default bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r5e}
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/shard_rehearsal.py --ranks 8 --roots 4 --json gpurun_out/${T}_friendster_p8.json > gpurun_out/${T}_friendster_p8.out 2> gpurun_out/${T}_friendster_p8.err; rc=$?
tail -14 gpurun_out/${T}_friendster_p8.err; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err; rc=$?
grep "secondary\|held-out" gpurun_out/${T}_bench.err; head -c 400 gpurun_out/${T}_bench.json; exit $rc
