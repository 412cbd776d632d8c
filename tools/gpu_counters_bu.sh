#!/bin/bash
# Per-dispatch counters of the bottom-up kernel (three --pmc passes, kernel
# trace only).  Output: gpurun_out/counters_bu.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${KERNEL:-bu_hub_kernel}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS"
P2="FETCH_SIZE TCC_HIT_sum"
P3="TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VALU SQ_INSTS_SALU"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1)); rm -rf gpurun_out/pmcbu$i
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/pmcbu$i -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-validate ${BENCH_ARGS} > gpurun_out/pmcbu$i.log 2>&1 \
    || { tail -20 gpurun_out/pmcbu$i.log; exit 1; }
done
python3 tools/counter_dispatch.py --kernel $K gpurun_out/pmcbu1 gpurun_out/pmcbu2 gpurun_out/pmcbu3 > gpurun_out/counters_bu.txt
for i in 1 2 3; do find gpurun_out/pmcbu$i -name "*.csv" -size +1M -exec gzip -f {} \; ; done
cat gpurun_out/counters_bu.txt
