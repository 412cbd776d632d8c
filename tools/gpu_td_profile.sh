#!/bin/bash
# Top-down-only profile (BASELINE config 2 class): RMAT-22 --mode td bench,
# per-level device-clock times of a few roots, and the kernel statistics.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-td}
S=${SCALE:-22}
timeout -k 10 240 python bench.py --scale $S --mode td --steps 16 --warmup 3 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
  || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', d['value'], 'GTEPS', d['ms_per_step'], 'ms/step', d['validated_roots'])" gpurun_out/${TAG}_bench.json
timeout -k 10 200 python tools/run_roots.py --scale $S --mode td --roots 1 100 1000 12345 ${ROOT_ARGS} > gpurun_out/${TAG}_roots.txt 2>&1 || { tail -20 gpurun_out/${TAG}_roots.txt; exit 1; }
cat gpurun_out/${TAG}_roots.txt
if [ -n "$PROF" ]; then
  rm -rf gpurun_out/${TAG}_prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
    python3 bench.py --scale $S --mode td --steps 8 --warmup 2 --no-validate > /dev/null 2>&1 || { echo "rocprof failed"; exit 1; }
  f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/${TAG}_kernel_stats.csv
  head -15 gpurun_out/${TAG}_kernel_stats.csv | cut -c1-200
  find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -exec gzip -f {} \;
fi
