#!/bin/bash
# Hardware counters of the BFS kernels (rocprofv3 --pmc, kernel trace only: no
# sys/runtime/hip/hsa/marker tracing in a counter run).  Two passes (TCC slots:
# FETCH_SIZE costs 3, WRITE_SIZE 2).  Output: gpurun_out/counters_summary.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SCALE=${SCALE:-26}
rm -rf gpurun_out/pmc1 gpurun_out/pmc2
timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY FETCH_SIZE \
  -d gpurun_out/pmc1 -o run --output-format csv -- \
  python3 bench.py --scale $SCALE --steps ${STEPS:-2} --warmup 1 --no-validate ${BENCH_ARGS} > gpurun_out/pmc1.log 2>&1 \
  || { tail -30 gpurun_out/pmc1.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum \
  -d gpurun_out/pmc2 -o run --output-format csv -- \
  python3 bench.py --scale $SCALE --steps ${STEPS:-2} --warmup 1 --no-validate ${BENCH_ARGS} > gpurun_out/pmc2.log 2>&1 \
  || { tail -30 gpurun_out/pmc2.log; exit 1; }
f1=$(find gpurun_out/pmc1 -name "*counter_collection.csv" | head -1)
f2=$(find gpurun_out/pmc2 -name "*counter_collection.csv" | head -1)
python3 tools/counter_summary.py "$f1" "$f2" > gpurun_out/counters_summary.txt
gzip -f "$f1" "$f2"
cat gpurun_out/counters_summary.txt
