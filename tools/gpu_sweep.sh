#!/bin/bash
# Sweep bench.py flag sets (";"-separated in $SWEEP) at RMAT-$SCALE on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
SCALE=${SCALE:-26}
make -j16 > gpurun_out/make.log 2>&1 || { tail -30 gpurun_out/make.log; exit 1; }
IFS=';' read -ra SETS <<< "${SWEEP:---alpha 14}"
for s in "${SETS[@]}"; do
  timeout -k 10 200 python bench.py --scale $SCALE --steps ${STEPS:-16} --warmup 3 --no-validate $s > gpurun_out/sweep.json 2>gpurun_out/sweep.err || { tail -20 gpurun_out/sweep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sweep.json')); print('$s'.ljust(40), d['value'], d['ms_per_step'])"
done
