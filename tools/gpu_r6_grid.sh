# Round-6 step: the high-diameter grid on one GPU (tests, bench row) and its P = 8 shadow replay.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r6g}
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v -k "high_diameter_grid" --timeout 150 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 --heldout-roots 16 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
grep -E "secondary|GTEPS" gpurun_out/${T}_bench.err | tail -12
timeout -k 10 300 python -u tools/shadow_rank.py --grid 1024:1024 --ranks-of 8 --ranks 0 7 --root-list 0 524800 --mode do > gpurun_out/${T}_shadow_p8.txt 2> gpurun_out/${T}_shadow_p8.err || { tail -20 gpurun_out/${T}_shadow_p8.err; exit 1; }
grep -E "^(sum|per)|^root|exact" gpurun_out/${T}_shadow_p8.txt
