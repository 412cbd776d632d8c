# Round-5 step: option A/Bs on RMAT-26, direction-optimising (tools/td_option_ab.py, 32 roots).
# ABS: ";"-separated "option:a:b" triples.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r5r}
IFS=';' read -ra abs <<< "${ABS:-td_sparse_edges:262144:65536;td_bin_edges:1e15:2097152}"
for ab in "${abs[@]}"; do
  IFS=':' read -r o a b <<< "$ab"
  timeout -k 10 400 python -u tools/td_option_ab.py --mode ${MODE:-do} --roots ${ROOTS:-32} --graphs ${GRAPHS:-r26} --option $o --a $a --b $b \
    > gpurun_out/${T}_${o}.txt 2>&1 || { tail -20 gpurun_out/${T}_${o}.txt; exit 1; }
  grep -v "^\[" gpurun_out/${T}_${o}.txt
done
