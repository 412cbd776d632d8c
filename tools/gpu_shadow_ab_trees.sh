#!/bin/bash
# Same-box A/B of two builds in shadow-rank replay: this tree's tools/shadow_rank.py against the
# copy in _ab_old/ (its package and tools/shadow_rank.py), alternating, rank 0 of P, RMAT-26, 4 roots.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
: > gpurun_out/ab_shadow${SUFFIX}.txt
for P in ${PS:-2 8}; do
  for r in $(seq 1 ${ROUNDS:-2}); do
    for t in _ab_old .; do
      out=gpurun_out/abs_${P}.txt
      timeout -k 10 300 python3 $t/tools/shadow_rank.py --scale ${SCALE:-26} --ranks-of $P --ranks 0 --roots 4 ${SHADOW_ARGS} > $out 2> ${out%.txt}.err || { tail -20 ${out%.txt}.err; exit 1; }
      cp $out gpurun_out/abs_${P}${SUFFIX}_$(basename $t).txt
      echo "P=$P $t: $(grep '^sum' $out | awk '{s1+=$2; s2+=$3} END {printf "1 GPU %.1f  rank0 %.1f us (4 roots)", s1, s2}')" | tee -a gpurun_out/ab_shadow${SUFFIX}.txt
    done
  done
done
