# Same-box A/B of the tree as is (A) against an older commit's tree (B, shipped as
# commit_ab_tree/, built on the box): bench.py twice each (headline, held-out, int32 pass).
#   bash tools/gpu_commit_ab.sh     (after: git archive <commit> | tar -x -C commit_ab_tree)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
ROOT=$PWD; T=${TAG:-cab}; d=/tmp/cab_tree
rm -rf $d && mkdir -p $d && tar -C commit_ab_tree -cf - . | tar -C $d -xf - && (cd $d && make -j16 > $ROOT/gpurun_out/${T}_make.log 2>&1) || { tail -20 gpurun_out/${T}_make.log; exit 1; }
for rep in 1 2; do
  for side in A B; do
    dir=$ROOT; [ $side = B ] && dir=$d
    timeout -k 10 300 python3 -u $dir/bench.py --steps 16 --warmup 2 --secondary none ${BENCH_ARGS} > gpurun_out/${T}_$side$rep.json 2> gpurun_out/${T}_$side$rep.err || { tail -20 gpurun_out/${T}_$side$rep.err; exit 1; }
    python3 - gpurun_out/${T}_$side$rep.json $side <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "headline", r["value"], "heldout", r["heldout"]["value"], "int32", r.get("value_int32_levels"))
PY
  done
done
