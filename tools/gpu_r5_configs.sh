# Round-5 step: the per-config 1-GPU benches (BASELINE.md results table): RMAT-27 / RMAT-24 direction-optimising,
# RMAT-22 top-down only.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r5c}
for cfg in "27 do" "24 do" "22 td"; do
  set -- $cfg
  timeout -k 10 400 python -u bench.py --scale $1 --mode $2 --heldout-roots 0 --secondary none \
    > gpurun_out/${T}_rmat$1_$2.json 2> gpurun_out/${T}_rmat$1_$2.err || { tail -20 gpurun_out/${T}_rmat$1_$2.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['validated_roots'], d.get('value_int32_levels'))" gpurun_out/${T}_rmat$1_$2.json "RMAT-$1 $2"
done
