# Same-box sweep of one engine option over the bench (headline 16 roots + held-out 128), twice each.
#   OPT=td_sparse_edges VALUES="65536 131072 262144" bash tools/gpu_opt_sweep.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-osw}
for rep in 1 2; do
  for v in ${VALUES}; do
    timeout -k 10 300 python3 -u bench.py --steps 16 --warmup 2 --secondary none --no-int32-pass --opt ${OPT}=$v > gpurun_out/${T}_${v}_$rep.json 2> gpurun_out/${T}_${v}_$rep.err || { tail -20 gpurun_out/${T}_${v}_$rep.err; exit 1; }
    python3 - gpurun_out/${T}_${v}_$rep.json "${OPT}=$v" <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "headline", r["value"], "heldout", r["heldout"]["value"], r["validated_roots"], r["heldout"]["validated_roots"], "mispredicted", r["heldout"].get("mispredicted_levels"))
PY
  done
done
