# Round-6 step: which launches a tiny tail level costs at P = 8 -- a kernel trace of one
# replayed rank (shadow_rank.py), the last traversal's kernels listed in order.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r6tt}
ROOT=${ROOT:-17872028}
rm -rf gpurun_out/${T}_trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace -o run --output-format csv -- python3 tools/shadow_rank.py --scale 26 --ranks-of ${P:-8} --ranks 0 --root-list ${ROOT} ${SHADOW_ARGS} > gpurun_out/${T}_shadow.txt 2>&1 || { tail -20 gpurun_out/${T}_shadow.txt; exit 1; }
cat gpurun_out/${T}_shadow.txt
k=$(find gpurun_out/${T}_trace -name "*kernel_trace.csv" | head -1)
python3 - "$k" "${NK:-70}" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tail = rows[-int(sys.argv[2]):]
t0 = int(tail[0]["Start_Timestamp"])
prev = None
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    prev = e
    n = r["Kernel_Name"].split("(")[0].replace("dbfs::kern::", "")[-48:]
    print(f"{(s - t0) / 1e3:9.2f} +{gap:6.2f} {(e - s) / 1e3:8.2f} grid {r.get('Grid_Size', r.get('Grid_Size_X', '?')):>8} {n}")
PY
gzip -f "$k"
