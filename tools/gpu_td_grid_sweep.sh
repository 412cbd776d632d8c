cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for g in 512 768 1024 1536 2048; do
  timeout -k 10 200 python bench.py --scale 22 --mode td --steps 16 --warmup 3 --no-validate --opt td_grid_filter_max=$g --opt td_grid_max=$g > gpurun_out/tdsw.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/tdsw.json').read().strip().splitlines()[-1]); print('grid', sys.argv[1], d['value'], [round(l[1]*1e3,1) for l in d['level_clock']['levels']])" $g
done
