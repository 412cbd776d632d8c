# Round-5 step: top-down-only A/B of the late levels (LJ-sized uniform / power-law, RMAT-22) and a
# kernel-stats profile of the LJ-sized uniform top-down traversal.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r5f}
timeout -k 10 400 python -u tools/td_late_ab.py --roots 16 --json gpurun_out/${T}_td_late_ab.json > gpurun_out/${T}_td_late_ab.txt 2>&1; rc=$?
cat gpurun_out/${T}_td_late_ab.txt | grep -v "^\[" ; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_lj -o lj -- python3 tools/td_late_ab.py --graphs lj --roots 8 > gpurun_out/${T}_prof_lj.log 2>&1; rc=$?
exit $rc
