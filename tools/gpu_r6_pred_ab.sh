# Round-6 step: the rising-phase predictor A/B (same box, held-out roots), then the default policy replayed at P = 2 / 8.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in 0 1 0 1; do
  DBFS_AB_RISING=$v timeout -k 10 300 python3 -u bench.py --steps 16 --warmup 2 --secondary none > gpurun_out/r6pred2_$v.json 2> gpurun_out/r6pred2_$v.err || { tail -20 gpurun_out/r6pred2_$v.err; exit 1; }
  python3 - gpurun_out/r6pred2_$v.json $v <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
h = r["heldout"]
print("rising", sys.argv[2], "headline", r["value"], "mispred", r["mispredicted_levels"], "heldout", h["value"], "mispred", h.get("mispredicted_levels"), "valid", r["validated_roots"], h["validated_roots"])
PY
done
TAG=r6def P=2 CONFIGS="base" bash tools/gpu_r6_policy.sh
TAG=r6def P=8 CONFIGS="base" bash tools/gpu_r6_policy.sh
