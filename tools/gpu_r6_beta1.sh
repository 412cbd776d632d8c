# Round-6 step: beta at one GPU (96 vs 384), same box, held-out roots; then a kernel trace of two roots.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for b in 96 384 96 384; do
  timeout -k 10 300 python3 -u bench.py --steps 16 --warmup 2 --secondary none --no-int32-pass --beta $b > gpurun_out/r6b1_$b.json 2> gpurun_out/r6b1_$b.err || { tail -20 gpurun_out/r6b1_$b.err; exit 1; }
  python3 - gpurun_out/r6b1_$b.json $b <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("beta", sys.argv[2], "headline", r["value"], "heldout", r["heldout"]["value"], r["validated_roots"], r["heldout"]["validated_roots"])
PY
done
rm -rf gpurun_out/r6tr
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6tr -o run --output-format csv -- python3 tools/run_roots.py --roots 41169583 13702079 > gpurun_out/r6tr.log 2>&1 || { tail -20 gpurun_out/r6tr.log; exit 1; }
f=$(find gpurun_out/r6tr -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py "$f" --runs 2 > gpurun_out/r6tr_summary.txt 2>&1; gzip -f "$f"; tail -60 gpurun_out/r6tr_summary.txt
