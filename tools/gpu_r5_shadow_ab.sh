# Round-5 step: shadow-rank A/B of engine options (RMAT-26, rank 0 of P = 2 and of P = 8, 4 roots).
# OPTSETS: ";"-separated sets of space-separated NAME=VALUE (empty set: defaults).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r5a}
IFS=";" read -ra sets <<< "${OPTSETS:-;bu_merge_visited=0}"
for P in ${PS:-2 8}; do
  i=0
  for set in "${sets[@]}"; do
    args=""; for o in $set; do args="$args --opt $o"; done
    out=gpurun_out/${T}_p${P}_set${i}.txt
    timeout -k 10 300 python -u tools/shadow_rank.py --scale ${SCALE:-26} --ranks-of $P --ranks 0 --roots 4 $args ${SHADOW_ARGS} > $out 2> ${out%.txt}.err || { tail -20 ${out%.txt}.err; exit 1; }
    echo "P=$P [$set]: $(grep '^sum' $out | awk '{s1+=$2; s2+=$3} END {printf "1 GPU %.1f  rank0 %.1f us (4 roots)", s1, s2}')"
    i=$((i+1))
  done
done
