# Round-5 step: the unvisited filter's host gate (td_unvis_vis_frac) A/Bs, top-down only.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r5w}
for pair in ${PAIRS:-0.85:0.6 0.95:0.85}; do
  A=${pair%%:*}; B=${pair##*:}
  timeout -k 10 400 python -u tools/td_option_ab.py --mode td --roots 16 --option td_unvis_vis_frac --a $A --b $B \
    > gpurun_out/${T}_gate_${A}_${B}.txt 2>&1 || { tail -20 gpurun_out/${T}_gate_${A}_${B}.txt; exit 1; }
  grep -v "^\[" gpurun_out/${T}_gate_${A}_${B}.txt | grep GTEPS
done
