#!/bin/bash
# Kernel timeline of one traversal on a bench secondary graph (tools/td_option_ab.py's last run:
# the per-level profile run of side b).  GRAPH: lj | lj_pl | r22; MODE: td | do; OPTION/A/B as the tool.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r5g}; G=${GRAPH:-lj}; M=${MODE:-td}
rm -rf gpurun_out/${T}_gtrace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_gtrace -o run -- \
  python3 tools/td_option_ab.py --graphs $G --mode $M --roots 2 --option ${OPTION:-td_sparse_grid} --a ${A:-256} --b ${B:-256} \
  > gpurun_out/${T}_gtrace.log 2>&1 || { tail -20 gpurun_out/${T}_gtrace.log; exit 1; }
f=$(find gpurun_out/${T}_gtrace -name "*kernel_trace.csv")
python3 tools/trace_summary.py $f --from-kernel init_run_kernel --runs 1 > gpurun_out/${T}_trace_${G}_${M}.txt
gzip -f $f
grep -v "^\[" gpurun_out/${T}_gtrace.log | grep -v "^W2026\|^E2026\|^ ::" | tail -4
cat gpurun_out/${T}_trace_${G}_${M}.txt
