# Round-6 step: td_sparse grid A/B (DBFS_AB_SPARSE_GRID), same box: per-root level times and held-out.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for g in 256 512 1024 256 512 1024; do
  DBFS_AB_SPARSE_GRID=$g timeout -k 10 300 python3 -u bench.py --steps 16 --warmup 2 --secondary none --no-int32-pass > gpurun_out/r6sg_$g.json 2> gpurun_out/r6sg_$g.err || { tail -20 gpurun_out/r6sg_$g.err; exit 1; }
  python3 - gpurun_out/r6sg_$g.json $g <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("grid", sys.argv[2], "headline", r["value"], "heldout", r["heldout"]["value"], r["validated_roots"], r["heldout"]["validated_roots"])
PY
done
DBFS_AB_SPARSE_GRID=1024 timeout -k 10 200 python3 -u tools/run_roots.py --roots 41169583 63203320 13702079 > gpurun_out/r6sg_roots_1024.txt 2>&1
DBFS_AB_SPARSE_GRID=256 timeout -k 10 200 python3 -u tools/run_roots.py --roots 41169583 63203320 13702079 > gpurun_out/r6sg_roots_256.txt 2>&1
cat gpurun_out/r6sg_roots_256.txt gpurun_out/r6sg_roots_1024.txt | cut -c1-200
