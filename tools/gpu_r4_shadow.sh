#!/bin/bash
# Round-4 shadow ranks: RMAT-26 at P = 8 for the four usual roots and four
# late-switch roots, ranks 0 and 7, per variant (VARIANTS: "name:opt=v,opt=v|...";
# default: the new defaults, and hub-split levels + multi-rank hub cut off).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r4}
ROOTS=${ROOTS:-"13702079 43129764 45382682 26246917 8766153 17872028 21909223 5467067"}
IFS='|' read -ra VS <<< "${VARIANTS:-new:|old:hx_levels=0,bu_cut_ranks=0}"
for v in "${VS[@]}"; do
  name=${v%%:*}; opts=${v#*:}
  args=()
  if [ -n "$opts" ]; then IFS=',' read -ra kvs <<< "$opts"; for kv in "${kvs[@]}"; do args+=(--opt "$kv"); done; fi
  echo "== $name ${opts}"
  timeout -k 10 600 python -u tools/shadow_rank.py --scale ${SCALE:-26} --ranks-of ${P:-8} --ranks ${RANKS:-0 7} \
      --root-list $ROOTS "${args[@]}" ${SHADOW_ARGS} --json gpurun_out/${TAG}_shadow_${name}.json \
      > gpurun_out/${TAG}_shadow_${name}.txt 2> gpurun_out/${TAG}_shadow_${name}.err
  rc=$?
  grep -E "^sum|exact" gpurun_out/${TAG}_shadow_${name}.txt
  [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_shadow_${name}.err; exit $rc; }
done
