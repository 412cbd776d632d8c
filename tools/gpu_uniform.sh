#!/bin/bash
# soc-LiveJournal1-sized uniform-random graph generated on the device
# (bench.py --uniform; BASELINE config 2 without the 1 GB text file):
# top-down-only and direction-optimising benches, then a kernel trace of
# the top-down levels of two roots.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
U=${U:-4847571:68993773}
for mode in td do; do
  timeout -k 10 300 python bench.py --uniform $U --mode $mode --steps 16 --warmup 3 --per-level ${BENCH_ARGS} > gpurun_out/uni_$mode.json 2> gpurun_out/uni_$mode.err || { tail -20 gpurun_out/uni_$mode.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], 'GTEPS', d['ms_per_step'], 'ms/step', d['validated_roots'], [(l[0], round(l[1]*1e3,1)) for l in d.get('level_clock',{}).get('levels',[])])" gpurun_out/uni_$mode.json $mode
done
if [ "${TRACE:-1}" = 1 ]; then
  rm -rf gpurun_out/utrace
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/utrace -o run --output-format csv -- \
    python3 bench.py --uniform $U --mode td --steps 2 --warmup 1 --no-validate --no-int32-pass ${BENCH_ARGS} > gpurun_out/utrace.log 2>&1 || { tail -20 gpurun_out/utrace.log; exit 1; }
  f=$(find gpurun_out/utrace -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_summary.py "$f" --from-kernel init_run_kernel --runs 1 > gpurun_out/uni_td_trace.txt
  gzip -f "$f"
  cat gpurun_out/uni_td_trace.txt
fi
