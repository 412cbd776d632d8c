# Same-box A/B of a compile-time variant on shadow replays: the tree as is (A) against a copy
# built with EXTRA_HIPFLAGS="$FLAGS" (B), P ranks, ranks 0 and P-1, four RMAT-26 roots, twice each.
#   FLAGS="-DSOME_VARIANT" P=8 bash tools/gpu_replay_ab.sh   (round 6: the LDS-kept tiny-level counts, since reverted)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
ROOT=$PWD; T=${TAG:-rab}; P=${P:-8}; d=/tmp/rab_tree
ROOTS=${ROOTS:-8766153 17872028 13702079 43129764}
rm -rf $d && mkdir -p $d && tar -C "$ROOT" --exclude=./gpurun_out -cf - . | tar -C $d -xf -
(cd $d && make clean > /dev/null && make -j16 EXTRA_HIPFLAGS="$FLAGS" > $ROOT/gpurun_out/${T}_make.log 2>&1) || { tail -20 gpurun_out/${T}_make.log; exit 1; }
for rep in 1 2; do
  for side in A B; do
    dir=$ROOT; [ $side = B ] && dir=$d
    timeout -k 10 600 python3 -u $dir/tools/shadow_rank.py --ranks-of $P --ranks 0 $((P - 1)) --root-list $ROOTS > gpurun_out/${T}_$side$rep.txt 2> gpurun_out/${T}_$side$rep.err || { tail -20 gpurun_out/${T}_$side$rep.err; exit 1; }
    echo "== $side$rep"; grep -E "^root|^sum" gpurun_out/${T}_$side$rep.txt | paste - - | sed 's/  */ /g'
  done
done
