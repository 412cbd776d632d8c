#!/bin/bash
# Shadow-rank measurements (tools/shadow_rank.py): rank r of a P-GPU
# traversal replayed alone on this GPU; per-level times next to the 1-GPU run.
# CFGS: "scale:P:r,r,...;..." configurations.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3}
IFS=';' read -ra cfgs <<< "${CFGS:-26:8:0,3,7;26:4:0,3;26:2:0,1;27:8:0,7}"
for cfg in "${cfgs[@]}"; do
  IFS=':' read -r s P ranks <<< "$cfg"
  ranks=${ranks//,/ }
  echo "== RMAT-$s P=$P ranks $ranks"
  timeout -k 10 400 python -u tools/shadow_rank.py --scale $s --ranks-of $P --ranks $ranks --roots ${ROOTS:-4} \
      --json gpurun_out/${TAG}_shadow_s${s}_p${P}.json ${SHADOW_ARGS} > gpurun_out/${TAG}_shadow_s${s}_p${P}.txt 2> gpurun_out/${TAG}_shadow_s${s}_p${P}.err
  rc=$?
  tail -4 gpurun_out/${TAG}_shadow_s${s}_p${P}.txt
  [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_shadow_s${s}_p${P}.err; exit $rc; }
done
