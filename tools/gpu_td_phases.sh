# Diagnostic: phase clocks of one-rank td_sparse launches (a copy built with -DDBFS_TD_PHASES).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
ROOT=$PWD; T=${TAG:-tdph}; d=/tmp/tdph_tree
rm -rf $d && mkdir -p $d && tar -C "$ROOT" --exclude=./gpurun_out -cf - . | tar -C $d -xf -
(cd $d && make clean > /dev/null && make -j16 EXTRA_HIPFLAGS="-DDBFS_TD_PHASES" > $ROOT/gpurun_out/${T}_make.log 2>&1) || { tail -20 gpurun_out/${T}_make.log; exit 1; }
timeout -k 10 200 python3 -u $d/tools/run_roots.py --roots ${ROOTS:-8766153 41169583 43129764} > gpurun_out/${T}_roots.txt 2>&1 || { tail -20 gpurun_out/${T}_roots.txt; exit 1; }
grep -E "td-phases|ms TT" gpurun_out/${T}_roots.txt | cut -c1-260
