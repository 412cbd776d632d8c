#!/bin/bash
# Sharded file ingestion on the GPU: write a synthetic reference-format edge
# list (generator edges), then bench.py --graph on it (each rank parses its
# byte range, the CSR shard is built on the GPU), validated; host peak RSS and
# load time in the JSON.  SCALE / EF choose the graph (26 / 27 ~ Friendster:
# 67 M vertices, 1.8 B edges).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
DIR=${GRAPH_DIR:-/tmp}
df -h "$DIR" /dev/shm 2>/dev/null | tail -n +1
free -g | head -2
F=$DIR/rmat${SCALE:-22}_ef${EF:-16}.txt
t0=$(date +%s)
( while sleep 20; do echo "[ingest] writing $(du -sh "$F" 2>/dev/null | cut -f1)"; done ) & hb=$!
timeout -k 10 ${WRITE_TIMEOUT:-300} python3 -c "
import sys, distributed_cuda_bfs_amd as dbfs
p = dbfs.rmat_params(${SCALE:-22}, ${EF:-16}, 1)
dbfs.native.write_generated_edge_list(sys.argv[1], p, 16)
" "$F" || { kill $hb; echo "write failed"; exit 1; }
kill $hb
t1=$(date +%s)
ls -la "$F"; echo "write_s $((t1 - t0))"
( while sleep 20; do echo "[ingest] bench running"; done ) & hb=$!
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py --graph "$F" --steps ${STEPS:-8} --warmup 2 --no-int32-pass ${BENCH_ARGS} \
  > gpurun_out/ingest.json 2> gpurun_out/ingest.err; rc=$?
kill $hb
rm -f "$F"
[ $rc -eq 0 ] || { tail -20 gpurun_out/ingest.err; exit $rc; }
python3 -c "import json; d=json.loads(open('gpurun_out/ingest.json').read().strip().splitlines()[-1]); print({k: d[k] for k in ('value','ms_per_step','validated_roots','generate_s','host_peak_rss_gb','n_gpus')}, d['config'])"
