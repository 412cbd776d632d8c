#!/bin/bash
# Round-4 shadow ranks: RMAT-26 at P = 8 for the four usual roots and four
# late-switch roots, hub-split levels on (default) and off, ranks 0 and 7.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r4}
ROOTS=${ROOTS:-"13702079 43129764 45382682 26246917 8766153 17872028 21909223 5467067"}
for hx in ${HX_SET:-4 0}; do
  echo "== hx_levels=$hx"
  timeout -k 10 600 python -u tools/shadow_rank.py --scale ${SCALE:-26} --ranks-of ${P:-8} --ranks ${RANKS:-0 7} \
      --root-list $ROOTS --opt hx_levels=$hx ${SHADOW_ARGS} --json gpurun_out/${TAG}_shadow_hx${hx}.json \
      > gpurun_out/${TAG}_shadow_hx${hx}.txt 2> gpurun_out/${TAG}_shadow_hx${hx}.err
  rc=$?
  grep -E "^sum|exact" gpurun_out/${TAG}_shadow_hx${hx}.txt
  [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_shadow_hx${hx}.err; exit $rc; }
done
