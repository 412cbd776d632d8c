# Round-6 step: the grid's per-level cost -- probe, then a kernel trace of one traversal.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r6gt}
timeout -k 10 200 python3 -u tools/grid_probe.py ${PROBE_ARGS} > gpurun_out/${T}_probe.txt 2>&1 || { tail -20 gpurun_out/${T}_probe.txt; exit 1; }
cat gpurun_out/${T}_probe.txt
rm -rf gpurun_out/${T}_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace -o run --output-format csv -- python3 tools/grid_probe.py --roots 524800 --reps 1 > gpurun_out/${T}_trace.log 2>&1 || { tail -20 gpurun_out/${T}_trace.log; exit 1; }
f=$(find gpurun_out/${T}_trace -name "*kernel_stats.csv" | head -1); head -15 "$f"
k=$(find gpurun_out/${T}_trace -name "*kernel_trace.csv" | head -1)
python3 - "$k" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last traversal: the last ~2500 kernels
tail = rows[-3000:]
gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(tail, tail[1:])]
durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tail]
names = {}
for r, d in zip(tail, durs):
    n = r["Kernel_Name"].split("(")[0][-60:]
    c = names.setdefault(n, [0, 0])
    c[0] += 1; c[1] += d
print("last 3000 kernels: mean duration %.2f us, mean gap %.2f us, median gap %.2f us" % (
    sum(durs) / len(durs) / 1e3, sum(gaps) / len(gaps) / 1e3, sorted(gaps)[len(gaps) // 2] / 1e3))
for n, (c, d) in sorted(names.items(), key=lambda x: -x[1][1])[:8]:
    print(f"  {c:6d} x {d / c / 1e3:7.2f} us  {n}")
PY
gzip -f "$k"
