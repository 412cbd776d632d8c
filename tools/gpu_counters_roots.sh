#!/bin/bash
# Per-kernel PMC counters of chosen roots (tools/run_roots.py), two passes.
#   ROOTS="33465303" OPTS="--opt x=1" tools/gpu_counters_roots.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/cr1 gpurun_out/cr2
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES FETCH_SIZE \
  -d gpurun_out/cr1 -o run --output-format csv -- python3 tools/run_roots.py --scale ${SCALE:-26} --mode ${MODE:-do} --roots ${ROOTS} ${OPTS} > gpurun_out/cr1.log 2>&1 || { tail -30 gpurun_out/cr1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum ${PMC2_EXTRA} \
  -d gpurun_out/cr2 -o run --output-format csv -- python3 tools/run_roots.py --scale ${SCALE:-26} --mode ${MODE:-do} --roots ${ROOTS} ${OPTS} > gpurun_out/cr2.log 2>&1 || { tail -30 gpurun_out/cr2.log; exit 1; }
: > gpurun_out/counters_roots.txt
for k in ${KERNELS:-td_expand update_kernel bu_hub}; do
  echo "== $k" >> gpurun_out/counters_roots.txt
  python3 tools/counter_dispatch.py --kernel $k --top ${TOP:-4} gpurun_out/cr1 gpurun_out/cr2 >> gpurun_out/counters_roots.txt
done
find gpurun_out/cr1 gpurun_out/cr2 -name "*.csv" -exec gzip -f {} \;
cat gpurun_out/counters_roots.txt
