# Round-6 step: direction policy at P ranks from shadow replays (RMAT-26, ranks 0 and P-1, four roots:
# two late-switch, two early-switch), one line per configuration and root.
#   P=8 CONFIGS="base|beta=384|beta=1536" bash tools/gpu_r6_policy.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
P=${P:-8}; T=${TAG:-r6pol}_p$P
ROOTS=${ROOTS:-8766153 17872028 13702079 43129764}
IFS='|' read -ra CFG <<< "${CONFIGS:-base}"
for c in "${CFG[@]}"; do
  opts=""
  if [ "$c" != "base" ]; then for kv in ${c//,/ }; do opts="$opts --opt $kv"; done; fi
  timeout -k 10 600 python3 -u tools/shadow_rank.py --ranks-of $P --ranks 0 $((P - 1)) --root-list $ROOTS $opts \
    > gpurun_out/${T}_${c//[=,]/_}.txt 2> gpurun_out/${T}_${c//[=,]/_}.err || { tail -20 gpurun_out/${T}_${c//[=,]/_}.err; exit 1; }
  echo "== $c"; grep -E "^root|^sum|exact" gpurun_out/${T}_${c//[=,]/_}.txt | paste - - | sed 's/  */ /g'
done
