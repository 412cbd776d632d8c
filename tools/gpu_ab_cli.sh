# Same-box A/B of two bfs CLI builds: alternating runs, RMAT-26, K random roots.
# Usage: bash tools/gpu_ab_cli.sh TAG BIN_A BIN_B [extra bfs flags...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
tag=$1; a=$2; b=$3; shift 3
for i in 1 2 3; do
  for bin in "$a" "$b"; do
    out=gpurun_out/${tag}_$(basename $bin)_$i.txt
    timeout -k 10 180 "$bin" --rmat 26 --roots 32 --no-oracle --json "$@" > $out 2>&1 || exit 1
    echo "$bin run $i: $(grep 'aggregate GTEPS' $out)"
  done
done
